#!/bin/bash
# Host input pipeline + bucket rebuild + logger on the GPU, then the full GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_host_data.py tests/test_sync_gpu.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2c_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/r2c_new.log | grep -v "^tests.*PASSED" | tail -20; tail -2 gpurun_out/r2c_new.log; fatal $rc new
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_sync_gpu.py --deselect tests/test_host_data.py > gpurun_out/r2c_all.log 2>&1
rc=$?; tail -3 gpurun_out/r2c_all.log; fatal $rc all
