# Same-box A/B of engine libraries built with different gemm_planes.hip sources / flags
# (profiles/r3af_gemm_lib_ab.log): the production library against
#   lib/exp/libalert_engine_old.so    (the previous gemm_planes.hip)
#   lib/exp/libalert_engine_noslp.so  (gemm_planes.hip under -fno-slp-vectorize)
# each linked from the in-tree objects with only gemm_planes.o replaced, e.g.
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -fno-slp-vectorize -c \
#     -o /tmp/gp.o attack-pretrain-models-of-code_amd/csrc/gemm_planes.hip
#   hipcc --offload-arch=gfx950 -shared -fPIC -o attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_noslp.so \
#     $(ls attack-pretrain-models-of-code_amd/build/*.o | grep -v gemm_planes) /tmp/gp.o
# Alternating processes, production kernels only (256x256 for N != 768, 256x192 for N = 768).
set -o pipefail
for L in "" attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_noslp.so "" attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_noslp.so; do
  echo "LIB=$L"
  timeout -k 10 150 python -u tools/gemm_bench.py --shapes ffn1,qkvp --variants 0@512 --rounds 7 ${L:+--lib $L} || exit 1
  timeout -k 10 150 python -u tools/gemm_bench.py --shapes ffn2_res,oproj_res --variants 0@192 --rounds 7 ${L:+--lib $L} || exit 1
done
