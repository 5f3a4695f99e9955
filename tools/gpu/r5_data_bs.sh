#!/bin/bash
# ResNet-50 graph at bs 1024 and the Data bench at batch 512 vs 1024
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/data_bs
timeout -k 10 120 python -u tools/bench_resnet.py --batch-size 1024 --iters 20 > gpurun_out/data_bs/resnet1024.log 2>&1 || { tail -10 gpurun_out/data_bs/resnet1024.log; exit 1; }
grep "{" gpurun_out/data_bs/resnet1024.log | tail -1
for r in 1 2; do
for bs in 512 1024; do
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 --batch-size $bs > gpurun_out/data_bs/d$bs.log 2>&1 || { echo "bench $bs failed"; tail -20 gpurun_out/data_bs/d$bs.log; exit 1; }
echo "bs=$bs $(grep '"metric"' gpurun_out/data_bs/d$bs.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["time_to_first_batch_s"], d["steady_state_rows_per_s"])')"
done
done
