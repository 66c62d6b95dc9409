#!/bin/bash
# Fresh CNN kernel tables at this round's tree (ResNet-50 / AlexNet dp1, B = 128, 224^2).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ai; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r9ai/r50 -o kt -- python3 bench.py --model resnet50 --steps 10 --warmup 3 --no-diag --device-warmup-ms 0 > gpurun_out/r9ai/r50.json 2> gpurun_out/r9ai/r50.err; fatal $? r50
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r9ai/alex -o kt -- python3 bench.py --model alexnet --steps 20 --warmup 5 --no-diag --device-warmup-ms 0 > gpurun_out/r9ai/alex.json 2> gpurun_out/r9ai/alex.err; fatal $? alex
find gpurun_out/r9ai -name "*kernel_stats.csv" | head; echo done
