#!/bin/bash
# rocprofv3 kernel trace + stats of the scoring-only bench; outputs under gpurun_out/$1/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tr}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
SHORT="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/trace" -o run -- python3 $SHORT > gpurun_out/$TAG/trace.log 2>&1
rc=$?; grep '^{' gpurun_out/$TAG/trace.log | cut -c1-200; echo "trace rc=$rc"; exit $rc
