#!/bin/bash
# streamed batch timeline (GG_STREAM_TRACE) after off-thread session teardown
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04u}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
GG_STREAM_TRACE=1 GG_DREPORT_TRACE=1 timeout -k 10 300 python -u tools/stream_probe.py 1000000 262144 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -E "evals/s|\[stream\]" $O/probe.log
