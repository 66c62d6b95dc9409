#!/bin/bash
# W = 4 / 8 peer-vehicle bench at the headline dims: which rank fails and why (r9af: rank 2 left
# the DDP rung early at W = 4 after the tensor variants).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ag; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for n in 4 8; do mode=auto
  TDP_GPU_PEER=1 TDP_PEER_TIMEOUT_S=60 timeout -k 10 300 python -u bench.py --gpus $n --steps 10 --warmup 3 --parallel $mode --no-diag > gpurun_out/r9ag/w${n}_$mode.json 2> gpurun_out/r9ag/w${n}_$mode.err; rc=$?
  tail -c 400 gpurun_out/r9ag/w${n}_$mode.json; echo; grep -A30 "raised" gpurun_out/r9ag/w${n}_$mode.err | head -40; fatal $rc w${n}_$mode
done
echo done
