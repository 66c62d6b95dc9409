#!/bin/bash
# Kernel stats: ResNet-50 and AlexNet with the conv plan table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_o -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_o.log 2>&1
fatal $? r50
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alex_o -o alex -- python3 bench.py --model alexnet --steps 10 --warmup 3 --no-diag > gpurun_out/prof_alex_o.log 2>&1
fatal $? alex
