set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG}; mkdir -p $O; cd $R
for v in $VARIANTS; do
  GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --steps 3 $BARGS > $O/bench_$v.json 2> $O/bench_$v.log || { tail -5 $O/bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], d['detail']['kernel_ms_mean'])"
done
