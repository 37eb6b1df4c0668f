# config-2 GA leg (400 examples) under two engine environments, alternating processes on one box:
#   bash tools/attack_env_ab.sh TAG "A_ENV" "B_ENV"   (e.g. "" "AE_SPLIT_BALANCE=1")
set -o pipefail
mkdir -p gpurun_out/$1
for E in "$2" "$3" "$2" "$3"; do
  echo "ENV=[$E]"
  env $E timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    --no-fp32-mode --subs-seconds 0 --mhm-examples 0 --mhm-seq-examples 0 --aa-examples 0 \
    --aa-gcb-examples 0 --clone-examples 0 --no-config1 > gpurun_out/$1/run.log 2>&1 || exit 1
  grep -E '^\{' gpurun_out/$1/run.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); a=d['attack']; print(d['value'], a['victim_queries_per_s'], a['attacked_examples_per_min'], a['wall_s'], a['victim_queries'])"
done
