#!/bin/bash
# Relay/entry/DDP GPU tests, then the split-cost timing experiment.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_gemm_exp.py > gpurun_out/r5d_exp.jsonl 2> gpurun_out/r5d_exp.err; rc1=$?
cat gpurun_out/r5d_exp.jsonl
[ $rc1 -eq 0 ] || exit $rc1
timeout -k 10 1000 python -u -m pytest tests/test_relay_gpu.py tests/test_entry_gpu.py tests/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5d_pytest.log 2>&1; rc=$?
tail -40 gpurun_out/r5d_pytest.log
exit $rc
