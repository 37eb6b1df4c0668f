# round 6: near-tie analysis of the config-3 run on this tree against round 5's (tools/config3_ties.py)
set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 1000 python -u tools/config3_ties.py scratch/config3/r5_0_1300.jsonl,scratch/config3/r5_1300_2732.jsonl \
  scratch/config3/r6_0_1300.jsonl,scratch/config3/r6_1300_2732.jsonl > gpurun_out/r6h/config3_ties.json 2> gpurun_out/r6h/config3_ties.log
