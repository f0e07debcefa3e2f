#!/bin/bash
# Round-5 GPU diagnostics of the report copy-out, the streamed entries and cfg4 batching, one mode per call
# (each step under its own time limit; the first failure ends the call).  Outputs under gpurun_out/$TAG.
#   stream      tools/stream_probe.py on 1M cfg2 texts: native vs Python callback, chunked vs one chunk,
#               shader copy-out vs copy engine (GG_D2H_PUSH=0), CU-masked variants (GG_PUSH_CUS)
#   blocks      the streamed entry with 64 K / 128 K / 32 K documents per report block (render occupancy)
#   report_ab   tools/report_ab.py (session vs streamed report in one process) under $VARIANTS, each an
#               env assignment or "default" (e.g. VARIANTS="default GG_D2H_PUSH=32 GPU_MAX_HW_QUEUES=16")
#   rate        tools/report_rate.py: repeated reports of one session, idle pauses, copy engine vs blit
#   frag        tools/d2h_frag.py: device-to-host rate of fresh vs old buffers around allocation churn
#   numa        tools/numa_probe.py: the streamed entry with the process pinned to each NUMA node
#   push_tests  the device-report / stream GPU tests with the shader copy-out forced on every path
#   cfg4_batch  bench.py cfg4 kernel-only lines with GG_LANE_DOCS = 16, 64, 8
#   stats_cfg4  tools/kernel_stats.py on 2048 cfg4 plans with the stats build (build.py stats first)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-copyout}; mkdir -p $O; cd $R
mode=$1
probe() {  # name, args, env...
  local name=$1 args=$2; shift 2
  echo "[copyout] $(date +%T) $name"
  env "$@" timeout -k 10 240 python3 -u tools/stream_probe.py $args > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  tail -1 $O/$name.log
}
case $mode in
  stream)
    probe native_262k "1000000 262144 native" GG_STREAM_TRACE=1
    probe py_262k "1000000 262144 py" GG_STREAM_TRACE=1
    probe native_1chunk "1000000 1000000 native" GG_STREAM_TRACE=1
    probe sdma "1000000 262144 native" GG_D2H_PUSH=0
    for c in 16 32; do probe cus$c "1000000 262144 native" GG_PUSH_CUS=$c; done;;
  blocks)
    for b in 65536 131072 32768; do probe block$b "1000000 262144 native" GG_DREPORT_BLOCK=$b; done;;
  report_ab)
    for v in ${VARIANTS:-default}; do
      e=$v; [ "$v" = default ] && e=GG_NONE=0
      echo "[copyout] $(date +%T) report_ab $v"
      env $e GG_PINNED_TRACE=1 timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab_$v.log 2> $O/report_ab_$v.err \
        || { tail -20 $O/report_ab_$v.err; exit 1; }
      cat $O/report_ab_$v.log
    done;;
  rate)
    timeout -k 10 300 python3 -u tools/report_rate.py 262144 0,0,20,0,45,0 > $O/rate_sdma.log 2>&1 || { tail -20 $O/rate_sdma.log; exit 1; }
    cat $O/rate_sdma.log
    HSA_ENABLE_SDMA=0 timeout -k 10 300 python3 -u tools/report_rate.py 262144 0,0,0 > $O/rate_blit.log 2>&1 || { tail -20 $O/rate_blit.log; exit 1; }
    cat $O/rate_blit.log;;
  frag)
    timeout -k 10 240 python3 -u tools/d2h_frag.py > $O/d2h_frag.log 2>&1 || { tail -20 $O/d2h_frag.log; exit 1; }
    cat $O/d2h_frag.log;;
  numa)
    for N in $(ls -d /sys/devices/system/node/node[0-9]* | sed 's/.*node//' | sort -n); do
      timeout -k 10 240 python3 -u tools/numa_probe.py $N > $O/numa_node_$N.log 2>&1 || { tail -20 $O/numa_node_$N.log; exit 1; }
      grep -v "^\[" $O/numa_node_$N.log | tail -2
    done;;
  push_tests)
    GG_D2H_PUSH=64 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "device_report or stream or multidevice" > $O/pytest_push.log 2>&1 || { tail -30 $O/pytest_push.log; exit 1; }
    tail -2 $O/pytest_push.log;;
  cfg4_batch)
    for L in 16 64 8; do
      GG_LANE_DOCS=$L timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
        > $O/cfg4_L$L.json 2> $O/cfg4_L$L.log || { tail -10 $O/cfg4_L$L.log; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('L', sys.argv[2], d['ms_per_step'], d['value'], d['detail']['lane_tiles_retried_in_wave_mode'])" $O/cfg4_L$L.json $L
    done;;
  stats_cfg4)
    GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_stats.so PACK=cfg4 timeout -k 10 300 python -u tools/kernel_stats.py 2048 \
      > $O/kernel_stats_cfg4.json 2> $O/kernel_stats_cfg4.err || { tail -20 $O/kernel_stats_cfg4.err; exit 1; }
    head -c 1500 $O/kernel_stats_cfg4.json;;
  *) echo "usage: gpu_copyout.sh stream|blocks|report_ab|rate|frag|numa|push_tests|cfg4_batch|stats_cfg4"; exit 2;;
esac
echo "[copyout] $(date +%T) done"
