#!/bin/bash
# GPU pass for precision modes: engine parity tests, then the scoring bench in each mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { local rc=$1; [ "$rc" -ge 124 ]; }
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py -x -q 2>&1 | tee gpurun_out/pytest_modes.log
rc=$?; echo "pytest rc=$rc"; crash $rc && exit $rc
for P in ${MODES:-fp32 f32x3 bf16}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --attack-seconds 0 --precision $P 2>&1 | tee gpurun_out/bench_$P.log
  rc=$?; echo "bench $P rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
