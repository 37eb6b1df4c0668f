#!/bin/bash
# GA divergence debug, then the default bench (all legs); logs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/ga_divergence.py 2 > gpurun_out/ga_div.log 2>&1
rc=$?; tail -5 gpurun_out/ga_div.log; echo "ga_div rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -3 gpurun_out/bench_default.log; echo "bench rc=$rc"; exit $rc
