#!/bin/bash
# cfg4 documents-per-batch A/B, and the report copy-out with more hardware queues per process
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-zf}; mkdir -p $O; cd $R
for L in 16 64 8; do
  echo "[zf] $(date +%T) cfg4 GG_LANE_DOCS=$L"
  GG_LANE_DOCS=$L timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
    > $O/cfg4_L$L.json 2> $O/cfg4_L$L.log || { tail -10 $O/cfg4_L$L.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('L', sys.argv[2], d['ms_per_step'], d['value'], d['detail']['lane_tiles_retried_in_wave_mode'])" $O/cfg4_L$L.json $L
done
for Q in 4 16; do
  echo "[zf] $(date +%T) report_ab GPU_MAX_HW_QUEUES=$Q"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab_q$Q.log 2> $O/report_ab_q$Q.err || { tail -20 $O/report_ab_q$Q.err; exit 1; }
  cat $O/report_ab_q$Q.log
  echo "[zf] $(date +%T) stream GPU_MAX_HW_QUEUES=$Q"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 240 python3 -u tools/stream_probe.py 1000000 262144 native > $O/stream_q$Q.log 2>&1 || { tail -20 $O/stream_q$Q.log; exit 1; }
  tail -1 $O/stream_q$Q.log
done
echo "[zf] done"
