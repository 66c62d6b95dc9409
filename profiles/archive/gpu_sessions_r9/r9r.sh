#!/bin/bash
# After the linear / planes changes: TP + planes + linear GPU tests, driver-shaped dp1 bench with
# diagnostics (now incl. the tensor-sharded per-rank compute), x2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9r; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py tests/test_gemm_planes_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9r/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9r/pytest.log; fatal $rc pytest
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r9r/d$i.json 2> gpurun_out/r9r/d$i.err; rc=$?; tail -2 gpurun_out/r9r/d$i.err; fatal $rc bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(d["ms_per_step"], {k: g.get(k) for k in ("rehearsal_ms","tensor_rank_compute_ms","tensor_predicted_step_ms","tensor_predicted_eff")})' gpurun_out/r9r/d$i.json
done
echo done
