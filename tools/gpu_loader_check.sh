#!/bin/bash
# Device loader: the GPU loader tests on the product library (and on each $VARIANTS library), then the
# per-pass kernel times of a device-loader bench for all of them.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-lchk}
mkdir -p $O
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then lib=$PWD/cloudformation-guard_amd/libcfnguard_mi355x.so; else lib=$PWD/cloudformation-guard_amd/libcfnguard_mi355x_$v.so; fi
  GG_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "loader tests $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
TAG=${TAG:-lchk} bash tools/gpu_loader_prof.sh
