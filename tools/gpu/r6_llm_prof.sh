#!/bin/bash
# Round 6: per-dispatch decode kernel times of the serving bench (qkv / o / down told
# apart by grid size), for the TPOT work.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_llm
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/r6llm -o run -- python3 -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/bench.log 2>&1 || { echo "prof failed"; tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-400
timeout -k 10 120 python3 tools/kernel_trace_groups.py $(find /tmp/r6llm -name "*kernel_trace.csv" | head -1) > $O/groups.txt && cat $O/groups.txt
