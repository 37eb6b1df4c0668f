#!/bin/bash
# Packed-GEMM microbenchmark A/B only (variants in $V, shapes in $S).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_bench.py --shapes ${S:-ffn1,ffn2,qkv,oproj} --variants ${V:-0} --rounds 7 > gpurun_out/gemm_ab.log 2>&1
rc=$?; grep shape gpurun_out/gemm_ab.log; echo "gemm_bench rc=$rc"; exit $rc
