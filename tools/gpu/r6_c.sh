#!/bin/bash
# Round 6 call C: gemm.hip vs hipBLASLt (heuristic and TunableOp) on the plain NT shapes.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_c
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/gemm_vs_blaslt.py > $O/plain.jsonl 2>$O/plain.err || { tail -5 $O/plain.err; exit 1; }
cat $O/plain.jsonl
timeout -k 10 600 python -u tools/gemm_vs_blaslt.py --tune > $O/tuned.jsonl 2>$O/tuned.err || { tail -5 $O/tuned.err; exit 1; }
grep blaslt_tuned $O/tuned.jsonl
cp /tmp/tunable_r6*.csv $O/ 2>/dev/null || true
