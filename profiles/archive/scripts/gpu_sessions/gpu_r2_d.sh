#!/bin/bash
# BN final-reduction / residual-join / counter fusions: CNN tests, full GPU suite, CNN benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2d_all.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/r2d_all.log | head -10; tail -2 gpurun_out/r2d_all.log; fatal $rc all
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --no-diag > gpurun_out/r2d_r50.json 2> gpurun_out/r2d_r50.err
rc=$?; cat gpurun_out/r2d_r50.json; fatal $rc r50
timeout -k 10 300 python bench.py --model alexnet --steps 50 --warmup 10 --no-diag > gpurun_out/r2d_alex.json 2> gpurun_out/r2d_alex.err
rc=$?; cat gpurun_out/r2d_alex.json; fatal $rc alex
