#!/bin/bash
# Round 4: non-finite-safe split in the planes producers -- planes / emu / kernel / MLP tests,
# headline bench (the producers' select must cost nothing).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8l; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_gemm_emu_gpu.py tests/test_kernels_gpu.py tests/test_sync_gpu.py tests/test_cnn_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8l/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r8l/pytest.log; fatal $rc pytest
for r in 1 2; do timeout -k 10 300 python bench.py --no-diag > gpurun_out/r8l/b$r.json 2>/dev/null; fatal $? b; python3 -c 'import json; d=json.load(open("gpurun_out/r8l/b'$r'.json")); print("bench", d["ms_per_step"], d["config"]["final_loss"])'; done
echo done
