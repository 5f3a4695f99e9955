#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_lntest.sh && bash tools/gpu/r6_k64v.sh
