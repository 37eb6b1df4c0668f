set -o pipefail
for L in "" attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_noslp.so "" attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_noslp.so; do
  echo "LIB=$L"
  timeout -k 10 150 python -u tools/gemm_bench.py --shapes ffn1,qkvp --variants 0@512 --rounds 7 ${L:+--lib $L} || exit 1
  timeout -k 10 150 python -u tools/gemm_bench.py --shapes ffn2_res,oproj_res --variants 0@192 --rounds 7 ${L:+--lib $L} || exit 1
done
