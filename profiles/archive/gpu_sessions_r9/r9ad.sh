#!/bin/bash
# CNN configs at this round's tree (dp1): ResNet-50 and AlexNet, 20 steps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ad; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for m in resnet50 alexnet; do
timeout -k 10 500 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r9ad/$m.json 2> gpurun_out/r9ad/$m.err; fatal $? $m
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1][-14:], d["ms_per_step"], d["value"])' gpurun_out/r9ad/$m.json
done
echo done
