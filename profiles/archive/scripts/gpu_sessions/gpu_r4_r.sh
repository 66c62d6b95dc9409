#!/bin/bash
# Driver-shaped runs (20 timed / 5 warm-up) with the default (auto = scratch replica) warm-up vs GEMMs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2 3; do for w in auto gemm; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --warmup-mode $w > gpurun_out/r4r_$w$r.json 2>/dev/null; fatal $? "bench $w"
  echo "$r $w $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' gpurun_out/r4r_$w$r.json)"
done; done
