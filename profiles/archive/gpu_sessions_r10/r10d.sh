#!/bin/bash
# Head + loss launch micro-benchmark (fused vs unfused), with a kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10d; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 200 python scripts/bench_head.py > gpurun_out/r10d/head.jsonl 2> gpurun_out/r10d/head.err; fatal $? head
cat gpurun_out/r10d/head.jsonl
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r10d/kt -o kt -- python3 scripts/bench_head.py --iters 100 > gpurun_out/r10d/kt.log 2>&1; fatal $? kt
S=$(find gpurun_out/r10d/kt -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 $S | head -20
echo done
