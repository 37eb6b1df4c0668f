#!/bin/bash
# attention_pp bring-up: kernel tests, attention A/B, the whole GPU suite, then a short bench with
# the config-4 leg only.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pp
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pp/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/pp/kernels.log; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --variants pp,pp1 --rounds 7 > gpurun_out/pp/attn_ab.log 2>&1
rc=$?; grep variant gpurun_out/pp/attn_ab.log; echo "attn_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pp/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pp/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 > gpurun_out/pp/bench.log 2>&1
rc=$?; tail -c 2500 gpurun_out/pp/bench.log; echo "bench rc=$rc"; exit $rc
