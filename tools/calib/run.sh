#!/bin/bash
# On the box: FETCH_SIZE and WRITE_SIZE passes (separate runs) over tools/calib/calib.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/calib_fetch -o run --output-format csv -- $R/tools/calib/calib > $R/gpurun_out/calib_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/calib_write -o run --output-format csv -- $R/tools/calib/calib > $R/gpurun_out/calib_write.log 2>&1 || exit 2
echo calib-ok
