#!/bin/bash
# rocprofv3 kernel stats of Llama-3-8B serving with the decode GEMM on qkv / o.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dgllm_prof
mkdir -p $O
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt${TAG} -- python3 $R/tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/kt${TAG}.log 2>&1
echo prof=$?; grep metric $O/kt${TAG}.log | tail -1 | grep -o '"steady_tpot_p50_ms": [0-9.]*'
python3 - <<'PY'
import csv,glob,os
R=os.environ['GRAFT_REPO_ROOT']
T=os.environ.get('TAG','')
f=sorted(glob.glob(R+'/gpurun_out/dgllm_prof/kt'+T+'/*/*kernel_stats.csv'))[-1]
rows=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
with open(R+'/gpurun_out/dgllm_prof/top'+T+'.txt','w') as fo:
    for r in rows[:16]:
        line=f"{r['Name'][:100]} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} ms | {float(r['AverageNs'])/1e3:.1f} us"
        print(line); fo.write(line+'\n')
PY
