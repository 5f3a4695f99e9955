#!/bin/bash
# Round 6 call B: HF Llama parity (GPU), compiled-graph asyncio/overlap IPC test,
# record_stream negative control, AdamW variants.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_b
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_llama_hf_parity_gpu.py tests/test_gpu_runtime.py::test_compiled_dag_ipc_asyncio_overlap -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log; grep "HF argmax" $O/pytest.log; [ $rc -eq 0 ] || exit $rc
# negative control: without record_stream the race test must see wrong values
CAAMD_XFER_NO_RECORD_STREAM=1 timeout -k 10 200 python -u -m pytest tests/test_device_transfer_gpu.py -v --timeout 120 --timeout-method thread > $O/neg.log 2>&1; echo "negative control rc=$? (nonzero expected)"; grep -E "PASSED|FAILED" $O/neg.log
timeout -k 10 200 python -u tools/bench_adamw.py > $O/adamw.log 2>&1 || { tail -5 $O/adamw.log; exit 1; }
cat $O/adamw.log
timeout -k 10 600 python -u -m pytest tests/test_rllib_gpu_runners.py tests/test_rllib_learner_ipc_gpu.py "tests/test_llm_gpu.py::test_llama_engine_one_step_ahead_matches_sync" -x -v --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1; rc=$?
tail -6 $O/pytest2.log; exit $rc
