#!/bin/bash
# attention_pp variants: kernel tests, then the A/B at B=64 x L=512 (uniform and ragged).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/app
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k attention_pp > gpurun_out/app/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/app/kernels.log; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants pp1,pp2 --rounds 9 > gpurun_out/app/attn_ab.log 2>&1
rc=$?; grep variant gpurun_out/app/attn_ab.log; echo "attn_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants pp1,pp2 --rounds 7 --ragged > gpurun_out/app/attn_ab_ragged.log 2>&1
rc=$?; grep variant gpurun_out/app/attn_ab_ragged.log; echo "attn_bench ragged rc=$rc"; exit $rc
