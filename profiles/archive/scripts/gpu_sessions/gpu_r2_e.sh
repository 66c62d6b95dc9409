#!/bin/bash
# Channels-last conv weights read/written in place (no per-step permutes): tests, CNN benches,
# AlexNet / ResNet-50 kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2e_all.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2e_all.log | head -10; tail -2 gpurun_out/r2e_all.log; fatal $rc all
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --no-diag > gpurun_out/r2e_r50.json 2> gpurun_out/r2e_r50.err
rc=$?; cat gpurun_out/r2e_r50.json; fatal $rc r50
timeout -k 10 300 python bench.py --model alexnet --steps 50 --warmup 10 --no-diag > gpurun_out/r2e_alex.json 2> gpurun_out/r2e_alex.err
rc=$?; cat gpurun_out/r2e_alex.json; fatal $rc alex
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alex_e -o alex -- python3 bench.py --model alexnet --steps 10 --warmup 3 --no-diag > gpurun_out/prof_alex_e.log 2>&1
fatal $? profalex
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_e -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_e.log 2>&1
fatal $? profr50
