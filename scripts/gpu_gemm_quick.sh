#!/bin/bash
# Packed-GEMM kernel tests + microbenchmark (variants in $V, default production np2/np1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/kernels.log 2>&1
rc=$?; tail -5 gpurun_out/kernels.log; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/gemm_bench.py --shapes ffn1,ffn2,qkv,oproj --variants ${V:-0,0:1} --rounds 7 > gpurun_out/gemm_quick.log 2>&1
rc=$?; cat gpurun_out/gemm_quick.log | grep shape; echo "gemm_bench rc=$rc"; exit $rc
