#!/bin/bash
# (1) hypothesis check: another thread's event query during a global-mode capture; (2) the new
# regression test; (3) the full GPU suite + smoke() at this tree.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ah; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
PYTHONPATH=. timeout -k 10 120 python -u dev/micro/capture_thread_query.py > gpurun_out/r9ah/thread_query.log 2>&1; rc=$?; tail -2 gpurun_out/r9ah/thread_query.log; fatal $rc thread_query
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r9ah/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r9ah/gpu_suite.log; grep -E "FAILED|Error" gpurun_out/r9ah/gpu_suite.log | head -5; fatal $rc suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r9ah/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r9ah/smoke.log; fatal $rc smoke
echo done
