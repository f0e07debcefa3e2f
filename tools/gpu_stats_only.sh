set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03stats; mkdir -p $O; cd $R
for P in cfg5 cfg2; do
  GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_stats.so PACK=$P timeout -k 10 300 python -u tools/kernel_stats.py 20000 > $O/kernel_stats_$P.json 2> $O/kernel_stats_$P.err || { echo "kernel_stats failed"; tail -20 $O/kernel_stats_$P.err; exit 1; }
done
echo stats done
