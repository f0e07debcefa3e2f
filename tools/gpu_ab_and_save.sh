#!/bin/bash
# One GPU call: variant A/B on the cfg-2 bench (VARIANTS), then save a cfg-2 evaluation's results for
# CPU profiling of the report writer (tools/report_replay.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
if [ -n "${VARIANTS:-}" ]; then bash tools/ab_variants.sh || exit 1; fi
mkdir -p gpurun_out/replay
timeout -k 10 200 python -u tools/report_replay.py save gpurun_out/replay/cfg2_${SAVE_DOCS:-4000}.bin ${SAVE_DOCS:-4000} || exit 1
ls -la gpurun_out/replay
