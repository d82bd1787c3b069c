#!/bin/bash
# Build the A/B libraries here: tools/libA.so from git revision $1 (default HEAD~1, built in a
# throwaway worktree), tools/libB.so (+ stamps tools/libBS.so) from the working tree, which is
# also left built in-tree.  Variants: tools/variants.sh build ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD~1}
W=/tmp/ab_worktree
rm -rf $W
git -C $R worktree prune
git -C $R worktree add -f -q --detach $W $REV
make -s -C $W/custom-nvcomp-with-zstd_amd >/dev/null 2>&1
cp $W/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so $R/tools/libA.so
git -C $R worktree remove --force $W
make -s -C $R/custom-nvcomp-with-zstd_amd >/dev/null 2>&1
cp $R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so $R/tools/libB.so
make -s -C $R/custom-nvcomp-with-zstd_amd stamps >/dev/null 2>&1
cp $R/tools/libcuda_zstd_hip_stamps.so $R/tools/libBS.so
make -s -C $R/oracle >/dev/null
echo "A = $(git -C $R rev-parse --short $REV), B = working tree"
