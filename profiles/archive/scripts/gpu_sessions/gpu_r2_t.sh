#!/bin/bash
# Plan table v2 (BN statistics priced in): ResNet-50 / AlexNet benches, ResNet-50 kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for m in resnet50 alexnet resnet50 alexnet; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --no-diag > gpurun_out/r2t_$m.json 2>/dev/null; fatal $? $m
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2t_$m.json)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_t -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_t.log 2>&1
fatal $? prof
