#!/bin/bash
# Re-measure the CNN configs (AlexNet = the reference's model, ResNet-50 = BASELINE config 5) and the
# stock torch DDP path on the same box; toy MLP + SyncBN and the Accelerate-facade configs.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r25; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 > $O/alex.json 2> $O/alex.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 --impl torch > $O/alex_torch.json 2> $O/alex_torch.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > $O/r50.json 2> $O/r50.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 --impl torch > $O/r50_torch.json 2> $O/r50_torch.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --syncbn > $O/mlp_syncbn.json 2> $O/mlp_syncbn.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --syncbn --impl torch > $O/mlp_syncbn_torch.json 2> $O/mlp_syncbn_torch.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --api accelerate > $O/mlp_accel.json 2> $O/mlp_accel.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --optim adam --impl torch > $O/adam_torch.json 2> $O/adam_torch.err
rc=$?
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f)"; done
exit $rc
