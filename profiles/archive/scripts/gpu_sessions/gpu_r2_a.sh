#!/bin/bash
# Round-2 GPU check: new sync/optimizer tests first, then the whole GPU suite, then the bench.
# Stops at the first crash / timeout (exit 124, 134, 137, 139); plain test failures continue.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_sync_gpu.py -v --timeout 200 --timeout-method thread \
  > gpurun_out/r2a_sync_gpu.log 2>&1
rc=$?; echo "sync_gpu rc=$rc"; tail -3 gpurun_out/r2a_sync_gpu.log; fatal $rc sync_gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  --deselect tests/test_sync_gpu.py > gpurun_out/r2a_gpu_all.log 2>&1
rc=$?; echo "gpu_all rc=$rc"; tail -5 gpurun_out/r2a_gpu_all.log; fatal $rc gpu_all
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/r2a_bench.json 2> gpurun_out/r2a_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2a_bench.json; fatal $rc bench
