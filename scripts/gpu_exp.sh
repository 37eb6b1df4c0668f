#!/bin/bash
# Combined experiments: attention_pp kernel tests + pp1/pp2 A/B, then the GEMM stagger A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k attention_pp > gpurun_out/exp/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/exp/kernels.log; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants pp1,pp2 --rounds 9 > gpurun_out/exp/attn_ab.log 2>&1
rc=$?; grep variant gpurun_out/exp/attn_ab.log; echo "attn_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants pp1,pp2 --rounds 7 --ragged > gpurun_out/exp/attn_ab_ragged.log 2>&1
rc=$?; grep variant gpurun_out/exp/attn_ab_ragged.log; echo "attn_bench ragged rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --shapes ffn1,qkv --variants 0@512,116@512,132@512,208@512,216@512 --rounds 9 > gpurun_out/exp/gemm_stagger.log 2>&1
rc=$?; grep shape gpurun_out/exp/gemm_stagger.log; echo "gemm_bench rc=$rc"; exit $rc
