#!/bin/bash
# per-rules-file kernel times (tools/kernel_stats.py, 20000 templates per file) for each library in $LIBS
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-perfile}; mkdir -p $O; cd $R
for v in $LIBS; do
  GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so timeout -k 10 300 python3 tools/kernel_stats.py ${NDOCS:-20000} > $O/perfile_$v.json 2> $O/perfile_$v.log || { tail -5 $O/perfile_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/perfile_$v.json'))
print('$v', ' '.join('%s=%.3f' % (k[:12], v['kernel_ms']) for k, v in d.items()))"
done
