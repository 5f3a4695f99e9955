#!/bin/bash
# late round-2 checks: LLM + vision GPU tests, Data TTFB, LLM serving bench + decode kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/late
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py tests/test_vision.py -x -v --timeout 120 --timeout-method thread -m gpu \
  > $O/pytest_llm_vision.log 2>&1 || { tail -30 $O/pytest_llm_vision.log; exit 1; }
tail -2 $O/pytest_llm_vision.log
timeout -k 10 240 python -u tools/data_ttfb.py > $O/ttfb_phases.log 2>&1 || { tail -20 $O/ttfb_phases.log; exit 1; }
grep '{' $O/ttfb_phases.log
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/bench_data.log 2>&1 || { tail -20 $O/bench_data.log; exit 1; }
head -c 1000 $O/bench_data.log; echo
timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 128 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/bench_llm.log 2>&1 || { tail -20 $O/bench_llm.log; exit 1; }
grep metric $O/bench_llm.log | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 $R/tools/bench_llm.py --num-prompts 128 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/kt.log 2>&1
echo prof=$?
python3 - <<'PY'
import csv,glob,os
R=os.environ['GRAFT_REPO_ROOT']
f=sorted(glob.glob(R+'/gpurun_out/late/kt/*/*kernel_stats.csv'))[-1]
rows=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:16]: print(r['Name'][:80], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), round(float(r['AverageNs'])/1e3,1))
PY
