# quick GPU check: the -m gpu suite, the bench line with the random leg, the 2048-chunk bench
set -e
mkdir -p gpurun_out
T=${TAG:-quick}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-verify --no-decompress > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err
timeout -k 10 120 python bench.py --chunks 2048 --no-legs --no-decompress --no-cpu-baseline --no-verify > gpurun_out/${T}_sc2048.json 2>/dev/null
