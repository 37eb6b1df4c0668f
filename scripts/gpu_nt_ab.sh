#!/bin/bash
# Non-temporal vs plain epilogue stores: ping-pong GEMM A/B (diag 0 = production, 8 = the other
# store flavour), then a short scoring-only bench of the production engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nt
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_bench.py --shapes ffn1,qkv --variants 0@512,8@512 --rounds 9 > gpurun_out/nt/gemm256.log 2>&1
rc=$?; grep shape gpurun_out/nt/gemm256.log; echo "gemm256 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --shapes oproj,ffn2 --variants 0@192,8@192 --rounds 11 > gpurun_out/nt/gemm192.log 2>&1
rc=$?; grep shape gpurun_out/nt/gemm192.log; echo "gemm192 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1 > gpurun_out/nt/bench.log 2>&1
rc=$?; tail -c 700 gpurun_out/nt/bench.log; echo "bench rc=$rc"; exit $rc
