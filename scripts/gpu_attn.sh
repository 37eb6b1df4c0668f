#!/bin/bash
# Attention kernel variants: GPU parity tests, then the microbenchmark A/B (variants in $V).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k attention > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -5 gpurun_out/attn_tests.log; echo "attn tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants ${V:-0,1,2,3} --rounds 7 > gpurun_out/attn_ab.log 2>&1
rc=$?; cat gpurun_out/attn_ab.log | grep variant; echo "attn_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants ${V:-0,1,2,3} --rounds 5 --ragged > gpurun_out/attn_ab_ragged.log 2>&1
rc=$?; cat gpurun_out/attn_ab_ragged.log | grep variant; echo "attn_bench ragged rc=$rc"; exit $rc
