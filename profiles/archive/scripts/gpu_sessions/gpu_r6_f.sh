#!/bin/bash
# Planes GEMM bottleneck experiments (TDP_PLANES_EXP: 1 no MFMA, 2 no B DMA, 4 no A DMA).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for cfg in 2,0 3,0; do for e in 0 1 2 4 3 5 6 7; do
TDP_PLANES_CFG=$cfg TDP_PLANES_EXP=$e timeout -k 10 200 python -u scripts/bench_gemm_planes.py > gpurun_out/r6f_bench.log 2>&1; rc=$?; echo "cfg $cfg exp $e"; grep -v amdgpu.ids gpurun_out/r6f_bench.log | cut -c1-75; fatal $rc bench
done; done
echo done
