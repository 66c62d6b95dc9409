#!/bin/bash
# Scratch-replica device warm-up vs dummy GEMMs, driver-shaped windows (20 timed / 5 warm-up).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2; do for w in scratch gemm; do for m in toy_mlp alexnet resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --warmup-mode $w --no-diag > gpurun_out/r4p.json 2>gpurun_out/r4p.err; fatal $? "bench $m $w"
  echo "$r $w $m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4p.json)"
done; done; done
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-diag > gpurun_out/r4p.json 2>/dev/null; fatal $? long
echo "long toy_mlp $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4p.json)"
timeout -k 10 300 python bench.py --syncbn --steps 20 --warmup 5 > gpurun_out/r4p_syncbn.json 2>/dev/null; fatal $? syncbn
timeout -k 10 300 python bench.py --api accelerate --steps 20 --warmup 5 > gpurun_out/r4p_acc.json 2>/dev/null; fatal $? acc
for f in r4p_syncbn r4p_acc; do echo "$f $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/$f.json)"; done
