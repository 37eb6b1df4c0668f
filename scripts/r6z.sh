#!/bin/bash
# round 6: masked attention after the constant-bit-position select (three workgroups per CU) —
# parity, then GraphCodeBERT-shaped and random-mask timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6z}; mkdir -p $OUT
K="attention_pp" bash scripts/gpu.sh ${TAG:-r6z} tests || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --variants pp66,pp74,pp67 --rounds 9 --planes --mask --mask-gcb --L 640 >> $OUT/attn_gcb640.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/attn_bench.py --variants pp66,pp74 --rounds 9 --planes --mask --mask-gcb --L 640 --ragged >> $OUT/attn_gcb640_ragged.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --variants pp66,pp74 --rounds 9 --planes --mask --L 512 >> $OUT/attn_random512.log 2>&1 || exit $?
grep -h variant $OUT/attn_*.log | cut -c1-200
