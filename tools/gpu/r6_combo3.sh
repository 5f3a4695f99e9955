#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_ln.sh && bash tools/gpu/r6_inkernel.sh
