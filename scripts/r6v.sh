#!/bin/bash
# round 6: masked attention fast path (variant 74) — parity, then GraphCodeBERT-shaped timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
K="attention_pp" bash scripts/gpu.sh ${TAG:-r6v} tests && \
AV=pp66,pp74 ATTN_EXTRA="--planes --mask --mask-gcb --L 640" bash scripts/gpu.sh ${TAG:-r6v} attn && \
cp gpurun_out/${TAG:-r6v}/attn.log gpurun_out/${TAG:-r6v}/attn_gcb.log && \
AV=pp66,pp74 ATTN_EXTRA="--planes --mask --L 512" bash scripts/gpu.sh ${TAG:-r6v} attn
