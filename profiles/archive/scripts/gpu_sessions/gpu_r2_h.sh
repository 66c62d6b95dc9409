#!/bin/bash
# Row-vector (LDS-staged) GEMM output stores: full GPU suite, conv per-layer A/B, MLP / ResNet benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r2h_all.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2h_all.log | head -10; tail -2 gpurun_out/r2h_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_conv.py resnet50 128 > gpurun_out/r2h_conv_on.jsonl 2> gpurun_out/r2h_conv.err
fatal $? conv_on
TDP_GEMM_NO_CVEC=1 timeout -k 10 300 python scripts/bench_conv.py resnet50 128 > gpurun_out/r2h_conv_off.jsonl 2>> gpurun_out/r2h_conv.err
fatal $? conv_off
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-diag > gpurun_out/r2h_mlp.json 2> gpurun_out/r2h_mlp.err
rc=$?; cat gpurun_out/r2h_mlp.json; fatal $rc mlp
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --no-diag > gpurun_out/r2h_r50.json 2> gpurun_out/r2h_r50.err
rc=$?; cat gpurun_out/r2h_r50.json; fatal $rc r50
timeout -k 10 300 python bench.py --model alexnet --steps 50 --warmup 10 --no-diag > gpurun_out/r2h_alex.json 2> gpurun_out/r2h_alex.err
rc=$?; cat gpurun_out/r2h_alex.json; fatal $rc alex
