# round 5: residual prefetch A/B (diag 0 = prefetch added, 60 = none, 61 = cache-warm only)
set -o pipefail
CMD="for M in 16384 32768; do timeout -k 10 200 python -u tools/gemm_bench.py --M \$M --shapes oproj_res,ffn2_res --variants 0@192,60@192,61@192 --rounds 9 || exit 1; timeout -k 10 200 python -u tools/gemm_bench.py --M \$M --shapes oproj_ln,ffn2_ln --variants 0,6 --rounds 9 || exit 1; done" bash scripts/gpu.sh r5d cmd
