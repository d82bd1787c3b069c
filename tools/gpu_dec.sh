# decoder check: the decode GPU tests, the bench decompress leg, the rocprof kernel stats of it
set -e
mkdir -p gpurun_out
T=${TAG:-dec}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dec or frame or stream or dict or capi" > gpurun_out/${T}_gputests.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-verify --no-legs > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu-baseline --no-verify --no-legs --steps 3 --warmup 1 > gpurun_out/${T}_prof.log 2>&1
