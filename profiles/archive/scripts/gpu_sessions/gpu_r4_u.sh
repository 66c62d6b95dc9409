#!/bin/bash
# Driver-shaped toy MLP: scratch-replica warm-up length 200 vs 600 ms, same box.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2 3; do for ms in 200 600; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --device-warmup-ms $ms --no-diag > gpurun_out/r4u.json 2>/dev/null; fatal $? "bench $ms"
  echo "$r $ms $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4u.json)"
done; done
