#!/bin/bash
# round 6: the two-per-CU 128 x 192 kernel in the two-stream engine (AE_GEMM_P2 bit mask:
# 1 QKV, 2 FFN1, 4 O-projection, 8 FFN2) against the production launches, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6p}; mkdir -p $OUT
timeout -k 10 600 python -u tools/engine_ab.py --rounds ${ROUNDS:-7} --steps 10 \
  --configs "${CONFIGS:-prod:;q:AE_GEMM_P2=1;o:AE_GEMM_P2=4;f2:AE_GEMM_P2=8;qo:AE_GEMM_P2=5;qof2:AE_GEMM_P2=13}" \
  > $OUT/engine_ab.log 2>&1; rc=$?; tail -4 $OUT/engine_ab.log; exit $rc
