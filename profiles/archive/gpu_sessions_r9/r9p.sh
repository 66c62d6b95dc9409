#!/bin/bash
# Tensor-sharded step with the chunked fc2 overlap and the planes path up to 1024 rows: GPU tests,
# per-rank proxy; peer-vehicle bench (2 ranks on one GPU, full dims) with --parallel auto.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9p; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py tests/test_gemm_planes_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9p/pytest.log 2>&1; rc=$?; grep -E "FAIL|passed|failed" gpurun_out/r9p/pytest.log | tail -8; fatal $rc pytest
timeout -k 10 300 python -u scripts/tp_rank_proxy.py > gpurun_out/r9p/proxy.jsonl 2> gpurun_out/r9p/proxy.err; rc=$?; grep W gpurun_out/r9p/proxy.jsonl; fatal $rc proxy
TDP_GPU_PEER=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-diag > gpurun_out/r9p/peer_auto.json 2> gpurun_out/r9p/peer_auto.err; rc=$?; tail -3 gpurun_out/r9p/peer_auto.err; fatal $rc peer_auto
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(d["ms_per_step"], c["rung"], c["selection"], c["fallbacks"], c["sync"]["captured"])' gpurun_out/r9p/peer_auto.json
echo done
