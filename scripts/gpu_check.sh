#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench.  Stops at the first crash-class exit
# (fault/abort/segv/timeout); an ordinary test failure (exit 1) still lets the bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { local rc=$1; [ "$rc" -ge 124 ] && [ "$rc" -ne 0 ]; }
echo "== host: $(nproc) cpus"
timeout -k 10 900 python -m pytest tests -m gpu -x -q 2>&1 | tee gpurun_out/pytest_gpu.log
rc=$?; echo "pytest rc=$rc"; crash $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log
rc=$?; echo "smoke rc=$rc"; crash $rc && exit $rc
timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds ${CPU_SECONDS:-10} 2>&1 | tee gpurun_out/bench.log
rc=$?; echo "bench rc=$rc"; exit $rc
