#!/bin/bash
# round 6: gemm_pp192_kernel with K-tile kt+2's A pieces spread over phases 1 and 2 (DV 1, tools
# variant 3 of ae_bench_gemm_packed_res_stats) — float64 tests, then O-projection / FFN2 timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6ag}; mkdir -p $OUT
K="res_stats_matches_f64" bash scripts/gpu.sh ${TAG:-r6ag} tests || exit $?
for m in 32768 16384 32768 16384; do
  timeout -k 10 300 python -u tools/fold_bench.py --p2 --m $m --rounds 9 --only oproj_stats,ffn2_stats,oproj_stats_p2v3_g0,ffn2_stats_p2v3_g0 >> $OUT/fold.log 2>&1 || exit $?
done
grep launch $OUT/fold.log
