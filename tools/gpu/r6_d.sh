#!/bin/bash
# Round 6 call D: in-step A/B of library (TunableOp-selected) plain NT GEMMs vs gemm.hip,
# alternating runs on one box (bench.py --mode spmd, 10 timed steps).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_d
mkdir -p $O
cd $GRAFT_REPO_ROOT
ARMS=("CAAMD_LIB_NT=" "CAAMD_LIB_NT=1600x6400,1600x4800,4800x1600" "CAAMD_LIB_NT=1600x6400,1600x4800,4800x1600,1600x1600" "CAAMD_LIB_NT=1600x6400")
for i in 1 2; do
  for j in 0 1 2 3; do
    E="${ARMS[$j]}"
    env $E timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${j}_$i.log 2>&1 || { echo "bench $j failed"; tail -20 $O/bench_${j}_$i.log; exit 1; }
    echo "arm$j [$E] $(grep -o '"value": [0-9.]*' $O/bench_${j}_$i.log)"
  done
done
