#!/bin/bash
# GPU parity tests, then the packed-GEMM diagnostic microbenchmark (tools/gemm_bench.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/gemm_bench.py --shapes ffn1,ffn2,qkv,oproj --variants 0,0:1,1,2,3,4,5,6,7 --rounds 5 > gpurun_out/gemm_diag.log 2>&1
rc=$?; cat gpurun_out/gemm_diag.log | tail -40; echo "gemm_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; exit $rc
