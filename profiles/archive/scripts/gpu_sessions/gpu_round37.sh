#!/bin/bash
# Final state: default bench, AlexNet + ResNet-50 with the round's last build.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r37; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python bench.py > $O/mlp_default.json 2> $O/mlp_default.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 > $O/alex.json 2> $O/alex.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > $O/r50.json 2> $O/r50.err
rc=$?
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.e-]*' $f)"; done
exit $rc
