#!/bin/bash
# Eager vs hipGraph-replayed toy-MLP step at world size 1 (current kernels, SGD epilogue default).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r22; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/eager.json 2>> $O/eager.err && \
  timeout -k 10 120 python bench.py --steps 500 --warmup 30 --graph >> $O/graph.json 2>> $O/graph.err || exit $?
done
timeout -k 10 120 python bench.py --steps 500 --warmup 30 --graph --optim adam >> $O/graph_adam.json 2>> $O/graph_adam.err && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 --optim adam >> $O/eager_adam.json 2>> $O/eager_adam.err
rc=$?
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"final_loss": [0-9.e-]*' $f | tr '\n' ' ')"; done
exit $rc
