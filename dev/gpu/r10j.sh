#!/bin/bash
# Round-6 tree, every BASELINE config at dp1 next to stock torch DDP (same box, interleaved).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10j; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py --no-diag "$@" > gpurun_out/r10j/$name.json 2> gpurun_out/r10j/$name.err; fatal $? $name
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["value"])' gpurun_out/r10j/$name.json
}
run mlp_tdp 300 --steps 100 --warmup 20
run mlp_torch 300 --steps 100 --warmup 20 --impl torch
run mlp_adam_tdp 300 --steps 100 --warmup 20 --optim adam
run mlp_adam_torch 300 --steps 100 --warmup 20 --optim adam --impl torch
run mlp_syncbn_tdp 300 --steps 100 --warmup 20 --syncbn
run mlp_syncbn_torch 300 --steps 100 --warmup 20 --syncbn --impl torch
run mlp_accel_tdp 300 --steps 100 --warmup 20 --api accelerate
run r50_tdp 400 --model resnet50 --steps 20 --warmup 5
run r50_torch 400 --model resnet50 --steps 20 --warmup 5 --impl torch
run alex_tdp 300 --model alexnet --steps 20 --warmup 5
run alex_torch 300 --model alexnet --steps 20 --warmup 5 --impl torch
echo done
