#!/bin/bash
# Tile-shape A/B for the register-staged split-bf16 GEMM, with a kernel trace of each run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for T in 0 128 256; do
  OUT="$GRAFT_REPO_ROOT/gpurun_out/tiles/t$T"; mkdir -p "$OUT"
  AE_GEMM_VARIANT=0 AE_X3_TILE=$T timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --attack-seconds 0 --precision f32x3 > "$OUT/log.txt" 2>&1
  rc=$?; echo "tile $T rc=$rc"; tail -1 "$OUT/log.txt" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
exit 0
