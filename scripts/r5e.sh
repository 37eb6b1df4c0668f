# round 5: attention A/B (in-tree = maximum3 row max + psum without the leading 0; attn_old =
# the previous loop; attn_noslp = in-tree source under -fno-slp-vectorize), the config-3 tie
# analysis (round-3 run vs this round's), and the attention / kernel GPU tests
set -o pipefail
LIBS="attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_tools_attn_old.so attack-pretrain-models-of-code_amd/lib/exp/libalert_engine_tools_attn_noslp.so" AV=pp67 GCB=1 \
  CMD="bash tools/attn_lib_ab.sh" bash scripts/gpu.sh r5e cmd || exit $?
mkdir -p gpurun_out/r5e
timeout -k 10 600 python -u tools/config3_ties.py scratch/config3/r3_0_1300.jsonl,scratch/config3/r3_1300_2732.jsonl \
  scratch/config3/subs_0_1300.jsonl,scratch/config3/subs_1300_2732.jsonl > gpurun_out/r5e/config3_ties.json 2> gpurun_out/r5e/config3_ties.log || exit $?
TESTS="tests/test_kernels_gpu.py" K=attention bash scripts/gpu.sh r5e tests
