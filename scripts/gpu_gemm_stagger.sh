#!/bin/bash
# Staggered-first-round A/B of the ping-pong GEMM (ae_bench_gemm_packed diag 1tt / 2tt).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_bench.py --shapes ffn1,qkv --variants ${V:-0@512,116@512,132@512,208@512,216@512} --rounds 9 > gpurun_out/gemm_stagger.log 2>&1
rc=$?; grep shape gpurun_out/gemm_stagger.log; echo "gemm_bench rc=$rc"; exit $rc
