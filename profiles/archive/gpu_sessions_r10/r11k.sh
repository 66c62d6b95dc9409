#!/bin/bash
# final tree, N > 1 bench path on the peer vehicle (W rank processes time-sharing ONE GPU over the
# capturable peer collectives): toy MLP W = 2 / 4, SyncBN W = 2 / 4, Accelerate W = 2, ResNet-50 W = 2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11k; export TMPDIR=/tmp
run() { tag=$1; shift; TDP_GPU_PEER=1 timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r11k/$tag.json 2> gpurun_out/r11k/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/r11k/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r11k/$tag.json')); c=d['config']; print('$tag', d['n_gpus'], d['ms_per_step'], c['parallelism'], c.get('rung'), c.get('replicas_identical', c.get('replicas')))"; }
run mlp2 --gpus 2 --steps 20 --warmup 5 && run mlp4 --gpus 4 --steps 20 --warmup 5 && run sbn2 --gpus 2 --syncbn --steps 20 --warmup 5 && run sbn4 --gpus 4 --syncbn --steps 20 --warmup 5 && run acc2 --gpus 2 --api accelerate --steps 20 --warmup 5 && run rn2 --gpus 2 --model resnet50 --steps 5 --warmup 2 && echo done
