#!/bin/bash
# One parameterised GPU-box driver:  scripts/gpu.sh TAG STEP [STEP ...]
# Steps run in order; the first failing step ends the call (no retries).  Everything lands under
# gpurun_out/TAG/.
#   rebuild   make clean + __graft_entry__.build() on the box (proves the tree builds from source)
#   tests     pytest -m gpu            (K=<-k filter>, MAXFAIL=<n>, default -x; KEEPGOING=1: go on
#             to the next step after test failures, never after a crash / abort / time limit)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py $BENCH_FULL_ARGS        (the default run: every leg)
#   short     scoring-only bench, 20 steps             ($BENCH_ARGS appended)
#   trace     rocprofv3 --kernel-trace --stats over the scoring-only bench
#   pmc       one rocprofv3 --pmc pass per ';'-separated group in $PASSES over the scoring-only bench
#   gemm      tools/gemm_bench.py   (S=shapes, V=variants, ROUNDS)
#   attn      tools/attn_bench.py   (AV=variants, ROUNDS)
#   cmd       run "$CMD" under a 900 s limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT="$GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1 ${BENCH_ARGS:-}"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -c "${TAILC:-1500}" "$OUT/$name.log"; echo; echo "$name rc=$rc"
  return $rc
}
for S in "$@"; do
  case $S in
    rebuild) run rebuild 600 bash -c 'make clean && python -c "import __graft_entry__ as g; g.build()" && ls -l attack-pretrain-models-of-code_amd/lib' || exit $? ;;
    tests) XF="-x"; [ -n "$MAXFAIL" ] && XF="--maxfail=$MAXFAIL"
           run pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -m gpu $XF -v --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} ${K:+-k "$K"}
           rc=$?
           # KEEPGOING=1: test FAILURES (pytest rc 1) do not end the call; a crash, abort or
           # time limit (any other non-zero rc) still does.  pytest-timeout's thread method ends
           # a hung test with os._exit(1), so rc 1 counts as failures only when no timeout banner
           # is in the log and pytest reached its final summary line.
           if [ $rc -eq 1 ] && { grep -q '+++ Timeout +++' "$OUT/pytest_gpu.log" || \
                                 ! grep -Eq '^=+ .*(failed|passed).* in [0-9.]+s' "$OUT/pytest_gpu.log"; }; then
             echo "pytest_gpu: timeout or no final summary: not a plain test failure"; exit 124
           fi
           if [ $rc -ne 0 ] && ! { [ "${KEEPGOING:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 1000 python -u bench.py ${BENCH_FULL_ARGS:-} || exit $? ;;
    short) run short 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --attack-examples 0 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --clone-examples 0 --no-config1 ${BENCH_ARGS:-} || exit $? ;;
    trace) run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $SHORT || exit $? ;;
    pmc)
      IFS=';' read -ra PS <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE}"
      i=0
      for C in "${PS[@]}"; do
        echo "== pmc p$i: $C"
        timeout -s KILL 120 rocprofv3 --pmc ${C//,/ } --kernel-trace --output-format csv -d "$OUT/pmc_p$i" -o run -- python3 ${PMC_CMD:-$SHORT} > "$OUT/pmc_p$i.log" 2>&1
        rc=$?; echo "pmc p$i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/pmc_p$i.log" && exit $rc
        i=$((i+1))
      done ;;
    gemm) run gemm 400 python -u tools/gemm_bench.py --shapes ${S_:-ffn1,ffn2,qkv,oproj} --variants ${V:-0} --rounds ${ROUNDS:-7} || exit $? ;;
    attn) run attn 300 python -u tools/attn_bench.py --variants ${AV:-pp1} --rounds ${ROUNDS:-7} ${ATTN_EXTRA:-} || exit $? ;;
    cmd) run cmd 900 bash -c "$CMD" || exit $? ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
exit 0
