#!/bin/bash
# What the first steps of a short window still time: window length, dataset size, warm-up mode.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for args in "--steps 10 --warmup 5" "--steps 20 --warmup 5" "--steps 40 --warmup 5" "--steps 80 --warmup 5" "--steps 20 --warmup 5 --dataset 1280" "--steps 80 --warmup 5 --dataset 1280" "--steps 20 --warmup 5 --warmup-mode scratch" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --dataset 1280"; do
  timeout -k 10 300 python bench.py $args --no-diag > gpurun_out/r4q.json 2>/dev/null; fatal $? "bench $args"
  echo "[$args] $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4q.json)"
done
