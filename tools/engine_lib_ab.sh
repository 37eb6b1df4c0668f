# Alternating-process A/B of two engine libraries on one box (tools/engine_lib_ab.py):
#   LIB=attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_prefold.so REPS=3 bash tools/engine_lib_ab.sh
set -o pipefail
for r in $(seq ${REPS:-3}); do
  for L in "$LIB" ""; do
    timeout -k 10 180 python -u tools/engine_lib_ab.py ${L:+--lib $L} || exit 1
  done
done
