# Full measurement set for one tag (run on the GPU box via gpurun): rocprofv3 trace + HBM
# counters (tools/profile.sh), one SQ counter pass (tools/profile_sq.sh), the default bench
# line.  Summaries: python tools/prof_summary.py TAG; python tools/sq_summary.py TAG.
set -o pipefail
TAG=${TAG:-r02h}
bash tools/profile.sh $TAG || exit 1
bash tools/profile_sq.sh $TAG || exit 2
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 3
echo all-done
