#!/bin/bash
# round 6: the two-blocks-per-wave attention (variants 80 / 81 / 86) — parity tests, then A/B timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
K="attention_pp" bash scripts/gpu.sh ${TAG:-r6k} tests && \
AV=${AV:-pp67,pp81,pp86} ATTN_EXTRA="--planes" bash scripts/gpu.sh ${TAG:-r6k} attn && \
cp gpurun_out/${TAG:-r6k}/attn.log gpurun_out/${TAG:-r6k}/attn_full.log && \
AV=${AV:-pp67,pp81,pp86} ATTN_EXTRA="--planes --ragged" bash scripts/gpu.sh ${TAG:-r6k} attn
