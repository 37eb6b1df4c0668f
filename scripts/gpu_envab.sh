#!/bin/bash
# Bench A/B over environment settings: ENVS="A=1,B=2 A=3" (each item: comma-separated VAR=VAL
# list, "-" = none), precision P.  Prints one value per setting; logs under gpurun_out/envab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
P=${P:-f32x3}
for E in ${ENVS:--}; do
  TAG=${E//[,=]/_}
  ( [ "$E" != "-" ] && export ${E//,/ }; timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --attack-seconds 0 --subs-seconds 0 --mhm-examples 0 --precision $P > gpurun_out/envab/$TAG.log 2>&1 )
  rc=$?; echo "$E rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/envab/$TAG.log)"; [ $rc -ne 0 ] && tail -5 gpurun_out/envab/$TAG.log && exit $rc
done
exit 0
