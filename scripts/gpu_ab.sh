#!/bin/bash
# A/B of the split-bf16 GEMM variants (LDS-DMA ring vs register-staged) after the parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { local rc=$1; [ "$rc" -ge 124 ]; }
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py -x -q 2>&1 | tee gpurun_out/pytest_ab.log
rc=$?; echo "pytest rc=$rc"; crash $rc && exit $rc
for V in 1 0; do
  for P in ${MODES:-f32x3 bf16}; do
    AE_GEMM_VARIANT=$V timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --attack-seconds 0 --precision $P 2>&1 | tee gpurun_out/bench_v${V}_$P.log
    rc=$?; echo "bench v$V $P rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
