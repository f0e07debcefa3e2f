#!/bin/bash
# the shader copy-out (GG_D2H_PUSH) -- parity through the device-report and stream tests, then copy rates
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-push}; mkdir -p $O; cd $R
echo "[push] $(date +%T) tests with GG_D2H_PUSH=64"
GG_D2H_PUSH=64 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "device_report or stream or multidevice" > $O/pytest_push.log 2>&1 || { tail -30 $O/pytest_push.log; exit 1; }
tail -2 $O/pytest_push.log
for b in 32 64 128; do
  echo "[push] $(date +%T) report_ab push $b"
  GG_D2H_PUSH=$b timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab_push$b.log 2> $O/report_ab_push$b.err || { tail -20 $O/report_ab_push$b.err; exit 1; }
  cat $O/report_ab_push$b.log
done
echo "[push] done"
