#!/bin/bash
# MLP+SyncBN with / without the BN ReLU mask (A/B), kernel stats of both.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2; do
  for m in 1 0; do
    TDP_BN_MASK=$m timeout -k 10 200 python bench.py --syncbn --steps 300 --warmup 30 --no-diag > gpurun_out/r2m_sbn_$m.json 2>/dev/null; fatal $? sbn
    echo "mask=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2m_sbn_$m.json)"
  done
done
for m in 1 0; do
  TDP_BN_MASK=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sbn_$m -o sbn -- python3 bench.py --syncbn --steps 50 --warmup 10 --no-diag > gpurun_out/prof_sbn_$m.log 2>&1
  fatal $? prof$m
done
