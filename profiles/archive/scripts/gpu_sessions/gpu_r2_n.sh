#!/bin/bash
# Conv plan table: CNN tests, ResNet-50 / AlexNet with and without the table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r2n_t.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2n_t.log | head -10; tail -2 gpurun_out/r2n_t.log; fatal $rc tests
for db in default 0; do
  for m in resnet50 alexnet; do
    TDP_CONV_PLAN_DB=$([ $db = 0 ] && echo 0 || echo "") timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --no-diag > gpurun_out/r2n_${m}_$db.json 2>/dev/null; fatal $? $m$db
    echo "$m db=$db $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2n_${m}_$db.json)"
  done
done
