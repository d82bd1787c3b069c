# lists the PMC counters rocprofv3 offers on the box's GPU (for choosing --pmc passes)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
