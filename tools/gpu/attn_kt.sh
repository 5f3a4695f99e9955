set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/attn_kt
cd $R && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_llm_gpu.py -x -q -k "flash" --timeout 120 --timeout-method thread > $R/gpurun_out/attn_kt/test.log 2>&1
echo test=$?; tail -2 $R/gpurun_out/attn_kt/test.log
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/attn_kt/kt -- python3 $R/tools/bench_attn.py > $R/gpurun_out/attn_kt/kt.log 2>&1
echo prof=$?; tail -1 $R/gpurun_out/attn_kt/kt.log
python3 - <<'PY'
import csv,glob,os
R=os.environ['GRAFT_REPO_ROOT']
f=sorted(glob.glob(R+'/gpurun_out/attn_kt/kt/*/*kernel_stats.csv'))[-1]
for r in csv.DictReader(open(f)):
    if 'fa' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
