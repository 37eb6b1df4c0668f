# Config-3 substitutes leg alone under a kernel trace: GPU busy fraction of the leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r5sub; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode --attack-examples 0 --subs-seconds 20 --mhm-examples 0 --aa-examples 0 --aa-gcb-examples 0 --clone-examples 0 --no-config1 --no-microbench"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 -u bench.py $ARGS > $OUT/subs_trace.log 2>&1 || exit $?
echo traced
