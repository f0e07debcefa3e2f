#!/bin/bash
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
for sb in 16384 32768; do
GG_STACK_BYTES=$sb GG_LIB=cloudformation-guard_amd/libcfnguard_mi355x_ab.so timeout -k 10 200 python -u tools/tf_oracle_diff.py > $O/diff_stack$sb.txt 2>&1
echo stack $sb; grep -E "^G " $O/diff_stack$sb.txt
done
