#!/bin/bash
# head_ce with sharded tickets + early dx weight loads: numerics, micro-benchmark, dp1 A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10e; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_head_ce_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r10e/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10e/tests.log; grep -E "FAILED|Error" gpurun_out/r10e/tests.log | head -5; fatal $rc tests
timeout -k 10 200 python scripts/bench_head.py > gpurun_out/r10e/head.jsonl 2> gpurun_out/r10e/head.err; fatal $? head
cat gpurun_out/r10e/head.jsonl
for i in 1 2; do
for h in fused separate; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --head-loss $h --no-diag > gpurun_out/r10e/d${i}_$h.json 2> gpurun_out/r10e/d${i}_$h.err; fatal $? bench$i$h
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["final_loss"])' gpurun_out/r10e/d${i}_$h.json
done; done
echo done
