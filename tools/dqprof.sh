set -o pipefail
R=$GRAFT_REPO_ROOT
VARIANTS="g1 w1 g3" ROUNDS=2 timeout -k 10 400 bash tools/dec_ab.sh dqg || exit 1
mkdir -p $R/gpurun_out/dqp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dqp/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $R/gpurun_out/dqp/trace.log 2>&1 || exit 2
echo prof-done
