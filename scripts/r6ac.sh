#!/bin/bash
# round 6: attention variant 75 (74 + waves with no query skip the work) — parity, then timing on
# ragged batches (where last q-blocks are partly empty), full batches, GraphCodeBERT-shaped masks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6ac}; mkdir -p $OUT
K="attention_pp" bash scripts/gpu.sh ${TAG:-r6ac} tests || exit $?
for a in "--ragged" "" "--ragged --mask --mask-gcb --L 640" "--mask --mask-gcb --L 640"; do
  echo "== $a" >> $OUT/attn.log
  timeout -k 10 200 python -u tools/attn_bench.py --variants pp74,pp75,pp74,pp75 --rounds 9 --planes $a >> $OUT/attn.log 2>&1 || exit $?
done
grep -v amdgpu $OUT/attn.log | cut -c1-160
