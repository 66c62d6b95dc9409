#!/bin/bash
# Tensor-sharded per-rank step at W = 2 (rank 0's shard shapes on one GPU): proxy timing and a
# kernel trace, to see where it loses 13 us against dp1 (TP_RANK_US).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9aj; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u scripts/tp_rank_proxy.py 2 > gpurun_out/r9aj/proxy.jsonl 2> gpurun_out/r9aj/proxy.err; rc=$?; cat gpurun_out/r9aj/proxy.jsonl; fatal $rc proxy
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9aj/kt -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 2 > gpurun_out/r9aj/kt.log 2>&1; fatal $? kt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r9aj/bench_d1.json 2> gpurun_out/r9aj/bench_d1.err; rc=$?; tail -c 300 gpurun_out/r9aj/bench_d1.json; fatal $rc bench
echo done
