#!/bin/bash
# W = 8 rehearsal of the tensor-sharded path on ONE GPU (peer vehicle, 8 ranks): captured parity
# tests at W = 8, then bench.py at the headline dims with --parallel auto at 2 / 4 / 8 ranks.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9af; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r9af/tp_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r9af/tp_tests.log; fatal $rc tp_tests
for n in 2 4 8; do
  TDP_GPU_PEER=1 timeout -k 10 420 python -u bench.py --gpus $n --steps 10 --warmup 3 --parallel auto --no-diag > gpurun_out/r9af/peer_auto_w$n.json 2> gpurun_out/r9af/peer_auto_w$n.err; rc=$?
  tail -c 600 gpurun_out/r9af/peer_auto_w$n.json; echo; tail -3 gpurun_out/r9af/peer_auto_w$n.err; fatal $rc bench_w$n
done
echo done
