set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
B="python -u bench.py --workload cfg4 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline"
for v in "" "GG_LANE_GROUP=4" "GG_LANE_GROUP=64" "GG_LANE_DOCS=16"; do
  echo "== $v"
  env $v timeout -k 10 240 $B > $O/b_${v#*=}.json 2> $O/b_${v#*=}.err || { echo fail $v; tail -3 $O/b_${v#*=}.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/b_${v#*=}.json')); print(d['value'], d['ms_per_step'], d['detail']['lane_tiles_retried_in_wave_mode'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --workload cfg4 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline > $O/prof.json 2> $O/prof.err
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -12
