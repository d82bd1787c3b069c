# the decoder's kernels in isolation (ZH_DEC_SYNC=1: one group, synchronised per kernel)
set -e
mkdir -p gpurun_out
T=${TAG:-deciso}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ZH_DEC_SYNC=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu-baseline --no-verify --no-legs --steps 2 --warmup 1 > gpurun_out/${T}_prof.log 2>&1
