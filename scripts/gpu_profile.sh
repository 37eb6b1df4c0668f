#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Outputs under gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}
STEPS=${STEPS:-5}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --attack-seconds 0 ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/trace" -o run -- python3 $B 2>&1 | tee gpurun_out/$TAG/trace.log
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/pmc_$C" -o run -- python3 $B 2>&1 | tee gpurun_out/$TAG/pmc_$C.log
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
find gpurun_out/$TAG -name "*.csv" | head -50
exit 0
