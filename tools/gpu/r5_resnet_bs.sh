#!/bin/bash
# ResNet-50 graph throughput vs batch size (LLC residency of the activations)
set -o pipefail
cd $GRAFT_REPO_ROOT
for bs in 512 256 128 64 32; do
timeout -k 10 120 python -u tools/bench_resnet.py --batch-size $bs --iters 20 > gpurun_out/resnet_bs$bs.log 2>&1 || { tail -10 gpurun_out/resnet_bs$bs.log; exit 1; }
grep "{" gpurun_out/resnet_bs$bs.log | tail -1
done
