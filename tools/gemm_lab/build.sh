#!/bin/bash
# Build the standalone GEMM lab (gemm.hip + lab.hip) for gfx950, on the CPU host.
set -e
D=$(cd "$(dirname "$0")" && pwd)
R=$D/../..
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$R/csrc/kernels $R/csrc/kernels/gemm.hip $D/lab.hip -o $D/gemm_lab "$@"
