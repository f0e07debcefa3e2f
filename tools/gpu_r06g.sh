#!/bin/bash
# cfg4 evaluator counters after split walks (stats build)
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
L=cloudformation-guard_amd/libcfnguard_mi355x_stats.so
PACK=cfg4 GG_LIB=$L timeout -k 10 300 python -u tools/kernel_stats.py 8192 > $O/stats_split.json 2> $O/stats_split.err &&
PACK=cfg4 GG_SPLIT_WALK=0 GG_LIB=$L timeout -k 10 300 python -u tools/kernel_stats.py 8192 > $O/stats_nosplit.json 2> $O/stats_nosplit.err
