#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/run16.sh || exit 1
bash tools/run17.sh || exit 2
