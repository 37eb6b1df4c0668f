# Same-box A/B of engine libraries built from different attention_pp.hip sources
# (profiles/r4z_attn_*_ab.log): the production library against experiment builds under
# attack-pretrain-models-of-code_amd/lib/exp/ (LIBS, space-separated), alternating processes.
set -o pipefail
LIBS=${LIBS:-attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so}
for r in 1 2 3; do
  for L in "" $LIBS; do
    echo "LIB=${L:-production} r=$r"
    timeout -k 10 120 python -u tools/attn_bench.py --variants ${AV:-pp67,pp72} --planes --rounds 9 ${L:+--lib $L} || exit 1
  done
done
if [ -n "$GCB" ]; then
  for L in "" $LIBS "" $LIBS; do
    echo "LIB=${L:-production} gcb"
    timeout -k 10 120 python -u tools/attn_bench.py --variants pp66,pp72 --planes --L 640 --mask --mask-gcb --rounds 5 ${L:+--lib $L} || exit 1
  done
fi
