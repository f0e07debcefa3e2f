#!/bin/bash
set -o pipefail
O=gpurun_out/r06C; mkdir -p $O
timeout -k 10 120 python -u tools/nfa_diff.py > $O/prod.txt 2>&1; grep "^mode" $O/prod.txt
GG_LIB=cloudformation-guard_amd/libcfnguard_mi355x_ab.so timeout -k 10 120 python -u tools/nfa_diff.py > $O/flat.txt 2>&1; grep "^mode" $O/flat.txt
