#!/bin/bash
# AlexNet dp1: planes GEMM one-group (3) vs two-group (4, default) kernel, interleaved x2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ae; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2; do
for c in 3 4; do
timeout -k 10 300 python scripts/archive/run_with_variant.py --planes $c,0,0 -- bench.py --model alexnet --steps 20 --warmup 5 --no-diag > gpurun_out/r9ae/c${c}_$i.json 2>/dev/null; fatal $? c$c
python3 -c 'import json,sys; print(sys.argv[1][-12:], json.load(open(sys.argv[1]))["ms_per_step"])' gpurun_out/r9ae/c${c}_$i.json
done
done
echo done
