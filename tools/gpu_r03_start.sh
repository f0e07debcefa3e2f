#!/bin/bash
# Round 3 session start: GPU suite + smoke, then FETCH/WRITE PMC passes for cfg5 and cfg3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=r03j bash tools/gpu_tests.sh || exit 1
WORKLOAD=cfg5 DOCS=303031 bash tools/pmc_traffic.sh || exit 1
WORKLOAD=cfg3 bash tools/pmc_traffic.sh || exit 1
echo all done
