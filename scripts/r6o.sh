#!/bin/bash
# round 6: folded QKV / FFN1 on the two-per-CU 128 x 192 kernel — float64 tests, then A/B timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6o}; mkdir -p $OUT
K="fold_matches_f64" bash scripts/gpu.sh ${TAG:-r6o} tests && \
timeout -k 10 300 python -u tools/fold_bench.py --p2 --only qkv_fold,ffn1_fold,qkv_fold_p2_g8,qkv_fold_p2_g4,qkv_fold_p2_g16,ffn1_fold_p2_g8,ffn1_fold_p2_g4,ffn1_fold_p2_g16 > $OUT/fold_full.log 2>&1 && cat $OUT/fold_full.log && \
timeout -k 10 300 python -u tools/fold_bench.py --p2 --m 16384 --only qkv_fold,ffn1_fold,qkv_fold_p2_g8,qkv_fold_p2_g4,ffn1_fold_p2_g8,ffn1_fold_p2_g4 > $OUT/fold_half.log 2>&1 && cat $OUT/fold_half.log
