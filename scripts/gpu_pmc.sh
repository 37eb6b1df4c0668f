#!/bin/bash
# PMC counter passes over a 2-step bench for each GEMM variant / precision given in RUNS
# ("variant:precision ..."), counters in PASSES ("C1,C2,...;C3,..."). Outputs gpurun_out/pmc/<run>/<pass>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RUNS=${RUNS:-"0:f32x3 1:f32x3"}
PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE;TCC_HIT_sum,TCC_MISS_sum,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE"}
IFS=';' read -ra PS <<< "$PASSES"
for R in $RUNS; do
  V=${R%%:*}; P=${R##*:}
  i=0
  for C in "${PS[@]}"; do
    OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/v${V}_$P/p$i"
    mkdir -p "$OUT"
    AE_GEMM_VARIANT=$V timeout -k 10 400 rocprofv3 --pmc ${C//,/ } --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --attack-seconds 0 --precision $P > "$OUT/log.txt" 2>&1
    rc=$?; echo "run v$V $P pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/log.txt" && exit $rc
    i=$((i+1))
  done
done
exit 0
