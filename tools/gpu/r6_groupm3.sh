#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
GM_LIST="2 4 6 8" bash tools/gpu/r6_groupm.sh
