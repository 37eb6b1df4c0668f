# Config-2 attack leg alone: plain run (tokens / s), then under a kernel trace (GPU busy fraction)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r5t; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode --attack-examples 400 --subs-seconds 0 --mhm-examples 0 --aa-examples 0 --aa-gcb-examples 0 --clone-examples 0 --no-config1 --no-microbench"
timeout -k 10 400 python3 -u bench.py $ARGS > $OUT/attack.log 2>&1 || exit $?
tail -c 600 $OUT/attack.log
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 -u bench.py $ARGS > $OUT/attack_trace.log 2>&1 || exit $?
echo traced
