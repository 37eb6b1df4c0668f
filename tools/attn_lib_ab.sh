set -o pipefail
OLD=attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_old.so
for r in 1 2 3; do
  for L in "" $OLD; do
    echo "LIB=${L:-new} r=$r"
    timeout -k 10 120 python -u tools/attn_bench.py --variants pp67,pp72 --planes --rounds 9 ${L:+--lib $L} || exit 1
  done
done
for L in "" $OLD "" $OLD; do
  echo "LIB=${L:-new} gcb"
  timeout -k 10 120 python -u tools/attn_bench.py --variants pp66,pp72 --planes --L 640 --mask --mask-gcb --rounds 5 ${L:+--lib $L} || exit 1
done
