#!/bin/bash
# Whole GPU suite, then the default bench (every leg); logs under gpurun_out/$1/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-fb}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; tail -c 400 gpurun_out/$TAG/bench.log; echo "bench rc=$rc"; exit $rc
