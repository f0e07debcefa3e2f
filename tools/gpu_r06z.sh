#!/bin/bash
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
GSIZES=16 EXTRA=tools/cfg4_variants4.guard SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/v4.jsonl 2> $O/v4.err
