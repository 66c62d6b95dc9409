#!/bin/bash
# Driver-shaped bench (20 steps / 5 warm-up) with and without the device clock warm-up, and the
# stock torch DDP comparison under the same protocol.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for w in 200 0 200 0 200; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --device-warmup-ms $w > gpurun_out/r3d_tdp_$w.json 2>/dev/null; fatal $? "tdp $w"
  echo "tdp warm=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3d_tdp_$w.json)"
done
for w in 200 0; do
  timeout -k 10 200 python bench.py --impl torch --steps 20 --warmup 5 --device-warmup-ms $w > gpurun_out/r3d_torch_$w.json 2>/dev/null; fatal $? "torch $w"
  echo "torch warm=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3d_torch_$w.json)"
done
timeout -k 10 200 python bench.py --impl torch --steps 100 --warmup 20 > gpurun_out/r3d_torch_long.json 2>/dev/null; fatal $? "torch long"
echo "torch long $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3d_torch_long.json)"
