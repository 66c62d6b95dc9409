#!/bin/bash
# Full GPU suite + smoke() after the fused tensor-sharded optimizer.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9al; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r9al/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r9al/gpu_suite.log; grep -E "FAILED|Error" gpurun_out/r9al/gpu_suite.log | head -5; fatal $rc suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r9al/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r9al/smoke.log; fatal $rc smoke
echo done
