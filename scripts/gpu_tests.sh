#!/bin/bash
# GPU parity tests only (optionally a -k filter in $K); log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; exit $rc
