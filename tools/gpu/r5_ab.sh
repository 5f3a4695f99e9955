#!/bin/bash
# Round 5: alternating same-box A/B runs of the default bench under env knobs.
# usage: r5_ab.sh "<envA>" "<envB>" [rounds]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ab_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
A="$1"; B="$2"; N=${3:-2}
for i in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${tag}_$i.log 2>&1 || { echo "bench $tag failed"; tail -20 $O/bench_${tag}_$i.log; exit 1; }
    echo "$tag [$E] $(grep -o '"value": [0-9.]*' $O/bench_${tag}_$i.log)"
  done
done
