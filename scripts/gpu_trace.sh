#!/bin/bash
# Kernel trace (+stats) of a short bench in the given precision; per-kernel table printed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=${1:-f32x3}; TAG=${2:-trace_$P}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --attack-seconds 0 --precision $P > "$OUT/log.txt" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/log.txt" && exit $rc
python3 tools/kernel_table.py "$OUT/run_kernel_trace.csv"
grep -o '"value": [0-9.]*' "$OUT/log.txt"
