#!/bin/bash
# Parameter-store policy under the paired launch: SGD 24 vs 88 (3 interleaved pairs) and Adam
# 24 vs 88 (3 pairs), 100-step windows, one box.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10p; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
V=scripts/run_with_variant.py
show() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"])' $1; }
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 300 python $V --sgd $v -- bench.py --steps 100 --warmup 20 --no-diag > gpurun_out/r10p/sgd${i}_$v.json 2> gpurun_out/r10p/sgd${i}_$v.err; fatal $? sgd$i$v; show gpurun_out/r10p/sgd${i}_$v.json
done; done
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 300 python $V --adam $v -- bench.py --optim adam --steps 100 --warmup 20 --no-diag > gpurun_out/r10p/adam${i}_$v.json 2> gpurun_out/r10p/adam${i}_$v.err; fatal $? adam$i$v; show gpurun_out/r10p/adam${i}_$v.json
done; done
echo done
