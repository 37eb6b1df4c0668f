#!/bin/bash
# rocprofv3 kernel stats of a short scoring-only bench (LayerNorm store-flavour check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lnnt
export TMPDIR=/tmp
SHORT="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/lnnt/trace" -o run -- python3 $SHORT > gpurun_out/lnnt/trace.log 2>&1
rc=$?; grep '^{"metric"' gpurun_out/lnnt/trace.log | cut -c1-80; echo "trace rc=$rc"; exit $rc
