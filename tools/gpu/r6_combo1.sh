#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_lab.sh && bash tools/gpu/r6_data_trace.sh && bash tools/gpu/r6_llm_prof.sh
