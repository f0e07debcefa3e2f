#!/bin/bash
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
GSIZES=1,16 EXTRA=tools/cfg4_variants3.guard SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/v3.jsonl 2> $O/v3.err || exit 1
GG_SPLIT_WALK=0 GSIZES=16 EXTRA=tools/cfg4_variants3.guard SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/v3_nosplit.jsonl 2> $O/v3_nosplit.err
