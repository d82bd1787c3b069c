set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_multi.py tests/test_gpu_dict.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02b_gputests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err || exit 2
bash tools/profile_sq.sh r02b || exit 3
echo all-done
