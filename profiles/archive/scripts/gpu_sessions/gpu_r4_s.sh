#!/bin/bash
# Optimizer-epilogue variants re-checked under split-bf16 GEMM products (toy MLP, SGD and Adam).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2; do
  for v in "TDP_OPT_VARIANT=24" "TDP_OPT_VARIANT=8" "TDP_OPT_VARIANT=16" "TDP_OPT_PERSIST=0" "TDP_OPT_WGS=1" "TDP_OPT_EPILOGUE=0"; do
    env $v timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r4s.json 2>/dev/null; fatal $? "bench $v"
    echo "$r sgd $v $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4s.json)"
  done
  for v in "TDP_OPT_ADAM_VARIANT=24" "TDP_OPT_ADAM_VARIANT=8" "TDP_OPT_ADAM_VARIANT=16" "TDP_OPT_PERSIST=0"; do
    env $v timeout -k 10 300 python bench.py --optim adam --steps 60 --warmup 10 --no-diag > gpurun_out/r4s.json 2>/dev/null; fatal $? "bench adam $v"
    echo "$r adam $v $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4s.json)"
  done
done
