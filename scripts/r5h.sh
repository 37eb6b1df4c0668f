set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 900 python -u tools/config3_ties.py scratch/config3/r3_0_1300.jsonl,scratch/config3/r3_1300_2732.jsonl \
  scratch/config3/subs_0_1300.jsonl,scratch/config3/subs_1300_2732.jsonl > gpurun_out/r5h/config3_ties.json 2> gpurun_out/r5h/config3_ties.log
