#!/bin/bash
# After the FastParams zero-init fix: GPU suite without the persistent-GEMM tests (verbose log),
# then ResNet-50 with the conv-epilogue BN statistics.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x -k "not persistent" --timeout 120 --timeout-method thread > gpurun_out/r2r_all.log 2>&1
rc=$?; grep -E "FAILED|Error|Fault" gpurun_out/r2r_all.log | head -10; tail -2 gpurun_out/r2r_all.log; fatal $rc tests
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --no-diag > gpurun_out/r2r_r50_$i.json 2>gpurun_out/r2r_r50.err; fatal $? r50
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2r_r50_$i.json
done
