#!/bin/bash
# Planes GEMM: B prefetch distance A/B (TDP_PLANES_CFG=2,PF), numerics under each.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for cfg in 2,2 2,1; do
TDP_PLANES_CFG=$cfg timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r6d_pytest.log; fatal $rc "pytest $cfg"
done
for r in 1 2; do for cfg in 2,0 2,1 2,2 2,3 3,0; do
TDP_PLANES_CFG=$cfg timeout -k 10 200 python -u scripts/bench_gemm_planes.py > gpurun_out/r6d_bench.log 2>&1; rc=$?; echo "cfg $cfg"; grep -v amdgpu.ids gpurun_out/r6d_bench.log | cut -c1-120; fatal $rc bench
done; done
echo done
