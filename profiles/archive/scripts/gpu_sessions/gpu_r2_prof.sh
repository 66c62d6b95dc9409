#!/bin/bash
# Kernel-trace profiles at the current tree: toy MLP (kernel + HIP API order, to attribute
# memsets/copies), AlexNet and ResNet-50 per-kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/prof_mlp -o mlp -- python3 bench.py --steps 6 --warmup 4 --no-diag > gpurun_out/prof_mlp.log 2>&1
fatal $? mlp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alex -o alex -- python3 bench.py --model alexnet --steps 10 --warmup 3 --no-diag > gpurun_out/prof_alex.log 2>&1
fatal $? alex
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50 -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50.log 2>&1
fatal $? r50
find gpurun_out/prof_mlp gpurun_out/prof_alex gpurun_out/prof_r50 -name "*.csv" | head -20
