#!/bin/bash
# BN reduction occupancy sweep (TDP_BN_WG_PER_CU) on ResNet-50; kernel stats at the default.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for w in 1 2 4 8 1 4; do
  TDP_BN_WG_PER_CU=$w timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-diag > gpurun_out/r2j_r50_$w.json 2>/dev/null; fatal $? r50_$w
  echo "wg/cu=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2j_r50_$w.json)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_j -o r50 -- python3 bench.py --model resnet50 --steps 6 --warmup 2 --no-diag > gpurun_out/prof_r50_j.log 2>&1
fatal $? prof
