#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/run10.sh || exit 1
bash tools/run11.sh || exit 2
