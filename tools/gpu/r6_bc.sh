#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_c.sh && bash tools/gpu/r6_b.sh
