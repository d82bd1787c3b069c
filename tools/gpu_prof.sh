set -o pipefail
bash tools/profile.sh r02g || exit 1
bash tools/profile_sq.sh r02g || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r02g_bench.json 2> gpurun_out/r02g_bench.err || exit 3
echo all-done
