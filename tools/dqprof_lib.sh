# decoder kernel trace of a variant library (gpurun): usage bash tools/dqprof_lib.sh TAG LIB
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
CUDA_ZSTD_HIP_LIB=$R/$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $R/gpurun_out/$TAG/trace.log 2>&1 || exit 2
echo prof-done
