# quick GPU check: the -m gpu suite, one bench line, the K3/K1/K2 stamps of the full batch
set -e
mkdir -p gpurun_out
T=${TAG:-quick}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1
timeout -k 10 180 python bench.py --no-cpu-baseline --no-verify --no-decompress --no-legs > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err
timeout -k 10 200 python tools/stamps.py mix 16384 > gpurun_out/${T}_stamps.log 2>&1
