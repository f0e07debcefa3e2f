#!/bin/bash
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
run() { env GG_LIB=bisect_libs/lib_$1.so $2 timeout -k 10 120 python -u tools/nfa_diff.py > $O/nfa_$1_$3.txt 2>&1 || exit 1; echo "$1 $2"; grep "^mode" $O/nfa_$1_$3.txt; }
run nowalk GG_RX_MEMO=1 a
run quicknowalk GG_RX_MEMO=1 b
