#!/bin/bash
# Whole GPU suite, then a scoring-only bench (with the fp32-mode line); logs under gpurun_out/tb/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tb
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tb/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/tb/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1 > gpurun_out/tb/bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/tb/bench.log; echo "bench rc=$rc"; exit $rc
