#!/bin/bash
# Per-pass kernel times of the device JSON loader (rocprofv3 kernel trace of a device-loader bench).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-loader_prof}
mkdir -p $O
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then lib=$R/cloudformation-guard_amd/libcfnguard_mi355x.so; else lib=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so; fi
  GG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 $R/bench.py --loader device --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/$v.log 2>&1 || { echo "prof $v failed"; tail -3 $O/$v.log; [ $v = base ] && exit 1; }
  grep '^{"metric"' $O/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['detail']['device_loader'])"
  grep -i "json\|Name" $O/$v/run_kernel_stats.csv | cut -d, -f1-4
done
