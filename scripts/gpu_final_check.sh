#!/bin/bash
# Whole GPU suite + smoke, then an O-proj / FFN2 tile A/B (256x192 vs 256x256 ping-pong).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fc
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fc/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/fc/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/fc/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --shapes oproj,ffn2 --variants 0@192,0@512 --rounds 9 > gpurun_out/fc/tiles.log 2>&1
rc=$?; grep shape gpurun_out/fc/tiles.log; echo "gemm_bench rc=$rc"; exit $rc
