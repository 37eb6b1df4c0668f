# Same-box A/B of tools libraries built from different sources: alternating processes of
# tools/gemm_bench.py over the libraries in $LIBS ("" = the in-tree tools library), $REPS times.
#   LIBS=" lib/exp/libalert_engine_tools_old.so" SHAPES=ffn1,qkvp VARIANTS=0@512,4@512 bash tools/lib_ab.sh
set -o pipefail
for r in $(seq ${REPS:-2}); do
  for L in ${LIBS:-""} ""; do
    echo "LIB=${L:-in-tree}"
    timeout -k 10 150 python -u tools/gemm_bench.py --shapes ${SHAPES:-ffn1,qkvp} --variants ${VARIANTS:-0@512} --rounds ${ROUNDS:-7} ${L:+--lib $L} || exit 1
  done
done
