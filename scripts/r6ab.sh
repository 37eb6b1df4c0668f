#!/bin/bash
# round 6: unmasked attention (PIPE 67) before / after the constant-bit-position select, alternating
# processes on one box (the old loop in lib/exp/libalert_engine_tools_oldsel.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6ab}; mkdir -p $OUT
OLD=attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_tools_oldsel.so
for r in 1 2 3; do
  for L in "" "$OLD"; do
    for R in "" "--ragged"; do
      echo "lib=${L:-new} $R" >> $OUT/attn_lib_ab.log
      timeout -k 10 120 python -u tools/attn_bench.py --variants pp67 --rounds 7 --planes $R ${L:+--lib $L} >> $OUT/attn_lib_ab.log 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids $OUT/attn_lib_ab.log | cut -c1-170
