set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/llm_kt
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/llm_kt/kt -- python3 $R/tools/bench_llm.py --num-prompts 128 --max-num-seqs 128 --input-len 512 --output-len 128 > $R/gpurun_out/llm_kt/kt.log 2>&1
echo prof=$?; grep metric $R/gpurun_out/llm_kt/kt.log | tail -1
python3 - <<'PY'
import csv,glob,os
R=os.environ['GRAFT_REPO_ROOT']
f=sorted(glob.glob(R+'/gpurun_out/llm_kt/kt/*/*kernel_stats.csv'))[-1]
rows=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(r['Name'][:90], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), round(float(r['AverageNs'])/1e3,1))
PY
