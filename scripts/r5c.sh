# round 5: residual prefetch of the 256x192 GEMM — kernel / engine parity, A/B, short bench
set -o pipefail
TESTS="tests/test_kernels_gpu.py tests/test_engine_gpu.py" bash scripts/gpu.sh r5c tests || exit $?
CMD="for M in 32768 16384; do timeout -k 10 200 python -u tools/gemm_bench.py --M \$M --shapes oproj_res,ffn2_res --variants 0@192,60@192 --rounds 9 || exit 1; timeout -k 10 200 python -u tools/gemm_bench.py --M \$M --shapes oproj_ln,ffn2_ln --variants 0,6 --rounds 9 || exit 1; done" bash scripts/gpu.sh r5c cmd short
