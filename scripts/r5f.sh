# round 5: config-3 tie analysis (round-3 run vs this round's) + the attention / kernel GPU tests
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u tools/config3_ties.py scratch/config3/r3_0_1300.jsonl,scratch/config3/r3_1300_2732.jsonl \
  scratch/config3/subs_0_1300.jsonl,scratch/config3/subs_1300_2732.jsonl > gpurun_out/r5f/config3_ties.json 2> gpurun_out/r5f/config3_ties.log || exit $?
TESTS="tests/test_kernels_gpu.py" K=attention bash scripts/gpu.sh r5f tests
