#!/bin/bash
# dK/dV ablation timings (per-kernel times from rocprofv3 --stats)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_abl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in 0 1 2 3 4 7; do
CAAMD_FA64_BWD_ABL=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$a -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $O/abl$a.log 2>&1 || { echo "abl $a failed"; tail -20 $O/abl$a.log; exit 1; }
f=$(find $O/p$a -name "run_kernel_stats.csv" | head -1)
echo "ABL=$a $(grep '"bwd_us"' $O/abl$a.log | head -1)"
grep -E "bwd_dkdv|bwd_dq|fwd_kernel" "$f" | awk -F, '{print "   ", $2, $3, $4}' | cut -c1-200
done
