#!/bin/bash
# Round 4: the one-process Accelerate facade with the hidden world-1 DDP (fused optimizer in the
# GEMM epilogues): GPU tests, entry-point tests, bench --api accelerate vs the native DDP step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8e; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d["config"]["optimizer"])' $1; }
timeout -k 10 600 python -u -m pytest tests/test_accelerate_gpu.py tests/test_entry_gpu.py tests/test_sync_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r8e/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r8e/pytest.log; fatal $rc pytest
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag --api accelerate > gpurun_out/r8e/accel_r$r.json 2>gpurun_out/r8e/accel_r$r.err; fatal $? accel; echo "accelerate r$r $(ms gpurun_out/r8e/accel_r$r.json)"
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r8e/ddp_r$r.json 2>gpurun_out/r8e/ddp_r$r.err; fatal $? ddp; echo "ddp r$r $(ms gpurun_out/r8e/ddp_r$r.json)"
done
timeout -k 10 300 python bench.py --no-diag --api accelerate --impl torch > gpurun_out/r8e/accel_torch.json 2>gpurun_out/r8e/accel_torch.err; fatal $? accel_torch; echo "accelerate torch $(ms gpurun_out/r8e/accel_torch.json)"
echo done
