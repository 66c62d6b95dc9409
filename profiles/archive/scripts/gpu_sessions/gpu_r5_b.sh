#!/bin/bash
# Relay (W ranks on one GPU) device-path tests, entry-point capture tests, DDP GPU tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_relay_gpu.py tests/test_entry_gpu.py tests/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5b_pytest.log 2>&1; rc=$?
tail -40 gpurun_out/r5b_pytest.log
exit $rc
