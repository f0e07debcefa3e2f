#!/bin/bash
# NUMA placement of the streamed entry's host memory (tools/numa_probe.py), node by node
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-numa}; mkdir -p $O; cd $R
NODES=$(ls -d /sys/devices/system/node/node[0-9]* | sed 's/.*node//' | sort -n | tr '\n' ' ')
echo "nodes: $NODES"
for N in $NODES; do
  echo "[numa] $(date +%T) node $N"
  timeout -k 10 240 python3 -u tools/numa_probe.py $N > $O/node_$N.log 2>&1 || { tail -20 $O/node_$N.log; exit 1; }
  cat $O/node_$N.log | grep -v "^\[" | tail -2
done
echo "[numa] done"
