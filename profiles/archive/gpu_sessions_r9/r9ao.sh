#!/bin/bash
# Final-tree checks: driver-shaped dp1 bench (diagnostics on), and the 2-rank peer-vehicle bench
# at the headline dims with --parallel auto (plumbing: fused tensor rungs chosen / recorded).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ao; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r9ao/d1.json 2> gpurun_out/r9ao/d1.err; rc=$?; tail -c 700 gpurun_out/r9ao/d1.json; echo; fatal $rc d1
TDP_GPU_PEER=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-diag > gpurun_out/r9ao/peer2.json 2> gpurun_out/r9ao/peer2.err; rc=$?; tail -c 500 gpurun_out/r9ao/peer2.json; echo; fatal $rc peer2
echo done
