#!/bin/bash
# Shared residual-input gradient (fork / SharedGrad): CNN tests, ResNet-50 bench + kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2f_cnn.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2f_cnn.log | head -10; tail -2 gpurun_out/r2f_cnn.log; fatal $rc cnn
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --no-diag > gpurun_out/r2f_r50.json 2> gpurun_out/r2f_r50.err
rc=$?; cat gpurun_out/r2f_r50.json; fatal $rc r50
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_f -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_f.log 2>&1
fatal $? profr50
