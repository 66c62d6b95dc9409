#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9v; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9v/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9v/pytest.log; exit $rc
