#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_step_pmc.sh && bash tools/gpu/r6_attn_pmc.sh
