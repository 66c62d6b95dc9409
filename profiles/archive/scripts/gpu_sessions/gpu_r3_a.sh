#!/bin/bash
# Session re-entry check at HEAD: GPU suite, smoke, default bench, then kernel traces of the
# multi-GPU schedule rehearsed on one GPU (collectives kept, captured step) for the overlap report.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3a_pytest_gpu.log; fatal $rc pytest
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/r3a_smoke.log 2>&1; fatal $? smoke
tail -1 gpurun_out/r3a_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err; fatal $? bench
cat gpurun_out/r3a_bench.json
cd /tmp
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r3a_ov_mlp" -o mlp -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph --steps 6 --warmup 4 --no-diag > "$GRAFT_REPO_ROOT/gpurun_out/r3a_ov_mlp.log" 2>&1
fatal $? ov_mlp
TDP_FORCE_COLLECTIVE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r3a_ov_r50" -o r50 -- python3 "$GRAFT_REPO_ROOT/bench.py" --model resnet50 --graph --steps 4 --warmup 3 --no-diag > "$GRAFT_REPO_ROOT/gpurun_out/r3a_ov_r50.log" 2>&1
fatal $? ov_r50
cd "$GRAFT_REPO_ROOT"
find gpurun_out/r3a_ov_mlp gpurun_out/r3a_ov_r50 -name "*.csv"
