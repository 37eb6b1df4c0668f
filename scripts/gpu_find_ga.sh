#!/bin/bash
# Debug scan for GA-success examples (tools/debug/find_ga_success.py); log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/debug/find_ga_success.py > gpurun_out/find_ga.log 2>&1
rc=$?; tail -8 gpurun_out/find_ga.log; echo "find_ga rc=$rc"; exit $rc
