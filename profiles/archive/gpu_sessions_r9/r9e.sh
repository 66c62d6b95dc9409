#!/bin/bash
# ws kernel (native f32 math) anatomy + numerics; bench ladder on the peer vehicle
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9e; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
bash dev/gpu/r9d.sh; fatal $? r9d
timeout -k 10 600 python -u -m pytest tests/test_wgrad_opt_gpu.py tests/test_peer_gpu.py -x -q --timeout 300 --timeout-method thread -k "ws_ or ladder or captured_syncbn or captured_accelerate or captured_cnn" > gpurun_out/r9e/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r9e/pytest.log; fatal $rc pytest
echo done
