set -e
TAG=r02i bash tools/gpu_quick.sh
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02i_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $GRAFT_REPO_ROOT/gpurun_out/r02i_prof.log 2>&1
