#!/bin/bash
# Full GPU suite + smoke() at this round's tree (what the driver runs at round end).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9t; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r9t/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r9t/gpu_suite.log; grep -E "FAIL|Error" gpurun_out/r9t/gpu_suite.log | head -5; fatal $rc suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r9t/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r9t/smoke.log; fatal $rc smoke
echo done
