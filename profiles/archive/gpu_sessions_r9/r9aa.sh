#!/bin/bash
# fc2's weight gradient on an aux stream beside fc1's backward; dH1 gated in its epilogue.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9aa; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 700 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9aa/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9aa/pytest.log; grep -E "FAIL|Error" gpurun_out/r9aa/pytest.log | head -5; fatal $rc pytest
timeout -k 10 300 python -u scripts/tp_rank_proxy.py > gpurun_out/r9aa/proxy.jsonl 2> gpurun_out/r9aa/proxy.err; rc=$?; grep W gpurun_out/r9aa/proxy.jsonl; fatal $rc proxy
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9aa/kt -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 8 > gpurun_out/r9aa/kt.log 2>&1; fatal $? kt
T=$(find gpurun_out/r9aa/kt -name '*kernel_trace.csv' | head -1)
python3 scripts/step_timeline.py $T ce_fwd 2 > gpurun_out/r9aa/tp8_timeline.md; cat gpurun_out/r9aa/tp8_timeline.md
echo done
