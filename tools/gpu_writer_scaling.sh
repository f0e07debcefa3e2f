#!/bin/bash
# Host report-writer thread scaling on the GPU box (diagnostic); the results file is kept in /tmp.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-writer}
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/report_replay.py save /tmp/replay20k.bin 20000 > $O/save.log 2>&1 || { echo save failed; tail $O/save.log; exit 1; }
for t in 1 2 4 8 16; do
  REPS=2 GG_REPORT_THREADS=$t timeout -k 10 200 python -u tools/report_replay.py time /tmp/replay20k.bin 20000 2>&1 | grep json
done
lscpu | grep -E "Model name|Thread|Core|Socket|NUMA node\(s\)"
python -c "import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:32])"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
