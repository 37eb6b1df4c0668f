#!/bin/bash
# round 6: masked attention fast path (variant 74) vs 66, repeated GraphCodeBERT-shaped timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6w}; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/attn_bench.py --variants pp66,pp74,pp66,pp74 --rounds 9 --planes --mask --mask-gcb --L 640 >> $OUT/attn_gcb640.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/attn_bench.py --variants pp66,pp74 --rounds 9 --planes --mask --mask-gcb --L 640 --ragged >> $OUT/attn_gcb640_ragged.log 2>&1 || exit $?
grep variant $OUT/*.log | sed 's/"n": 64, //' | cut -c1-220
