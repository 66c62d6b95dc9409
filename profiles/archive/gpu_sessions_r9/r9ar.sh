#!/bin/bash
# Plumbing of the tensor rungs at N = 2 (peer vehicle) for BASELINE config 3 (SyncBN) and Adam.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ar; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for extra in "--syncbn" "--optim adam"; do
  tag=$(echo $extra | tr -d ' -')
  TDP_GPU_PEER=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 6 --warmup 3 --mlp-dims 1024,512,512 --dataset 1024 --batch 32 --device-warmup-ms 0 --no-diag --parallel tensor $extra > gpurun_out/r9ar/$tag.json 2> gpurun_out/r9ar/$tag.err; rc=$?
  python -c "import json,sys; r=json.loads(open('gpurun_out/r9ar/$tag.json').read().strip().splitlines()[-1]); c=r['config']; print('$tag', r['value'], c['rung'], c['optimizer'], c['sync']['captured'], c['sync']['replicas_identical'], c['fallbacks'])"; fatal $rc $tag
done
echo done
