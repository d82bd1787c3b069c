# decoder kernel trace (gpurun): bench decompress leg under rocprofv3 --kernel-trace --stats
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-dqp}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $R/gpurun_out/$TAG/trace.log 2>&1 || exit 2
echo prof-done
