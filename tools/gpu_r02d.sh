set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02d_gputests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02d_bench.json 2> gpurun_out/r02d_bench.err || exit 2
echo all-done
