#!/bin/bash
# graph steps per replay: 2 vs 4 (driver-shaped, interleaved), trajectory test
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9j; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_bench_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r9j/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9j/pytest.log; fatal $rc pytest
for i in 1 2 3; do
for g in 2 4; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g --no-diag > gpurun_out/r9j/g${g}_$i.json 2>/dev/null; fatal $? g$g
done
python3 -c 'import json,sys; print(*[(f[-12:], json.load(open(f))["ms_per_step"]) for f in sys.argv[1:]])' gpurun_out/r9j/g2_$i.json gpurun_out/r9j/g4_$i.json
done
echo done
