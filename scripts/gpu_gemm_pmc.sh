#!/bin/bash
# PMC passes over the packed-GEMM microbenchmark (one shape in $S, variant in $V); each pass is
# its own rocprofv3 run (counter-slot limits: <= 8 SQ, 4 TCC, 2 GRBM per pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=${S:-ffn2}; V=${V:-0}
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
        "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
i=0
for C in "${PASSES[@]}"; do
  OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_${S}_$V/p$i"; mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gemm_bench.py" --shapes $S --variants $V --rounds 1 --iters 3 > "$OUT/log.txt" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/log.txt" && exit $rc
  i=$((i+1))
done
python3 tools/pmc_table.py "$GRAFT_REPO_ROOT/gpurun_out" gemm_pk_kernel
exit 0
