#!/bin/bash
# Planes GEMM: 2 vs 3 stages, kernel-level split of GEMM vs reduce (rocprofv3 stats).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r6b_pytest.log; fatal $rc pytest
TDP_PLANES_CFG=3,1 timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b_pytest3.log 2>&1
rc=$?; tail -2 gpurun_out/r6b_pytest3.log; fatal $rc pytest3
for st in 2 3; do
TDP_PLANES_CFG=$st,1 timeout -k 10 200 python -u scripts/bench_gemm_planes.py > gpurun_out/r6b_bench$st.log 2>&1; rc=$?; echo "stages $st"; cat gpurun_out/r6b_bench$st.log; fatal $rc bench
done
TDP_PLANES_CFG=2,1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof -o prof -- python scripts/bench_gemm_planes.py > gpurun_out/r6b_prof.log 2>&1; fatal $? rocprof
find gpurun_out/r6b_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/r6b_kernel_stats.csv
head -20 gpurun_out/r6b_kernel_stats.csv | cut -c1-200
echo done
