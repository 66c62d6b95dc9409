#!/bin/bash
# 1024-thread BN reductions: BN/CNN tests, ResNet-50 bench x2 + kernel stats, MLP+SyncBN bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cnn_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r2k_t.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2k_t.log | head -10; tail -2 gpurun_out/r2k_t.log; fatal $rc tests
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-diag > gpurun_out/r2k_r50_$i.json 2>/dev/null; fatal $? r50
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2k_r50_$i.json
done
timeout -k 10 200 python bench.py --syncbn --steps 200 --warmup 20 --no-diag > gpurun_out/r2k_mlp_syncbn.json 2>/dev/null; fatal $? syncbn
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2k_mlp_syncbn.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_k -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_k.log 2>&1
fatal $? prof
