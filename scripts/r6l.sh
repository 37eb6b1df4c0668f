#!/bin/bash
# round 6: timing diagnostics of the two-blocks-per-wave attention (82-85: results wrong)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
AV=${AV:-pp67,pp81,pp82,pp83,pp84,pp85} ATTN_EXTRA="--planes" bash scripts/gpu.sh ${TAG:-r6l} attn
