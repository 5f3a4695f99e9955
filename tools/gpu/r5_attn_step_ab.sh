#!/bin/bash
# GPT-2-XL step: late-round-5 attention kernels vs their predecessors (env switches), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attn_step_ab
for r in 1 2; do
for v in new old; do
if [ $v = old ]; then export CAAMD_FA64_STG=0 CAAMD_FA64_DKDV_OPT=0 CAAMD_FA64_FWD_PRE=0; else unset CAAMD_FA64_STG CAAMD_FA64_DKDV_OPT CAAMD_FA64_FWD_PRE; fi
timeout -k 10 300 python -u bench.py > gpurun_out/attn_step_ab/$v$r.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/attn_step_ab/$v$r.log; exit 1; }
echo "$v $(grep '"metric"' gpurun_out/attn_step_ab/$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
