#!/bin/bash
# cfg4: per-rule kernel times at G=16/32, and one 2000-resource plan alone (latency)
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
GROUPS=16,32 PACK=cfg4 timeout -k 10 500 python -u tools/rule_split_timing.py 8192 > $O/rules.jsonl 2> $O/rules.err || exit 1
GROUPS=1,16,64 SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/solo.jsonl 2> $O/solo.err
