#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/conv1x1_gemm_probe.py > gpurun_out/conv_probe.log 2>&1 || { tail -20 gpurun_out/conv_probe.log; exit 1; }
grep shape gpurun_out/conv_probe.log
