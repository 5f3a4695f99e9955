cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 python -u tools/diag_rccl.py eager 2>&1 | tee gpurun_out/diag_rccl.log | grep -v "^\s*$" | tail -8
[ ${PIPESTATUS[0]} -eq 0 ] || exit 9
bash tools/gpu/run8.sh
