#!/bin/bash
# Kernel tests (GEMM + attention), then the FFN1 GEMM (production ping-pong kernel, and diag 4 =
# no epilogue) and attention microbenchmarks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/kernels.log; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_bench.py --shapes ffn1,ffn2,qkv --variants 0@512,4@512 --rounds 7 > gpurun_out/gemm_ab.log 2>&1
rc=$?; grep shape gpurun_out/gemm_ab.log; echo "gemm_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants 0,3 --rounds 7 > gpurun_out/attn_ab.log 2>&1
rc=$?; grep variant gpurun_out/attn_ab.log; echo "attn_bench rc=$rc"; exit $rc
