#!/bin/bash
# repeated device reports of one session: copy-out rate over time and after idle pauses (tools/report_rate.py),
# with the SDMA engines and with blit-kernel copies; GPU clocks / power / temperature around the runs
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-rrate}; mkdir -p $O; cd $R
snap() { timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp > $O/smi_$1.log 2>&1 || true; grep -E "sclk|socclk|fclk|mclk|Power|Temperature" $O/smi_$1.log | head -12; }
snap before
echo "[rrate] $(date +%T) sdma"
timeout -k 10 300 python3 -u tools/report_rate.py 262144 0,0,20,0,45,0 > $O/rate_sdma.log 2>&1 || { tail -20 $O/rate_sdma.log; exit 1; }
cat $O/rate_sdma.log
snap after_sdma
echo "[rrate] $(date +%T) blit"
HSA_ENABLE_SDMA=0 timeout -k 10 300 python3 -u tools/report_rate.py 262144 0,0,0 > $O/rate_blit.log 2>&1 || { tail -20 $O/rate_blit.log; exit 1; }
cat $O/rate_blit.log
snap after_blit
echo "[rrate] done"
