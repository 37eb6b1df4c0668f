# round 6: config 3 at its stated size in two calls: bash scripts/c6.sh START END
set -o pipefail
mkdir -p gpurun_out/c6
timeout -k 10 1080 python -u tools/get_substitutes.py --eval_data_file data/devign/test_funcs.jsonl \
  --store_path gpurun_out/c6/subs_$1_$2.jsonl --index $1 $2 --precision f32x3 > gpurun_out/c6/run_$1_$2.log 2>&1
rc=$?; tail -3 gpurun_out/c6/run_$1_$2.log; exit $rc
