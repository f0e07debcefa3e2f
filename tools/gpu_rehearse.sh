#!/bin/bash
# One GPU call: full GPU tests, then a 2-rank rehearsal of the multi-GPU bench path on ONE GPU
# (gloo tallies, both ranks pinned to device 0).  Never N=8: that is the driver's run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rehearse
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GG_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --docs ${DOCS:-100000} --dist-backend gloo --no-cpu-baseline > $O/bench2.log 2>&1 || { echo "2-rank bench failed"; tail -30 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | tail -1
