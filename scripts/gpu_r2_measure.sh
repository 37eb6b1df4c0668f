#!/bin/bash
# Round-2 measurement: GPU parity tests, the default bench (all legs), then rocprofv3 kernel
# trace + stats over a short scoring-only bench and one PMC pass per TCC counter (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950).  Everything under gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?; tail -4 gpurun_out/$TAG/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_FULL_ARGS:-} > gpurun_out/$TAG/bench.log 2>&1
  rc=$?; tail -c 3000 gpurun_out/$TAG/bench.log; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
SHORT="$GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/trace" -o run -- python3 $SHORT > gpurun_out/$TAG/trace.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/trace.log; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/pmc_$C" -o run -- python3 $SHORT > gpurun_out/$TAG/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/$TAG/pmc_$C.log && exit $rc
done
exit 0
