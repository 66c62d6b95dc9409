#!/bin/bash
# Round 4: factored g gathers issued before the layer's input-gradient GEMM (overlap it):
# multi-rank parity on the peer vehicle (captured + eager + ragged), relay, DDP / factor GPU
# tests, rehearsal and headline bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8k; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=15
timeout -k 10 900 python -u -m pytest tests/test_peer_gpu.py tests/test_relay_gpu.py tests/test_factor_gpu.py tests/test_ddp_gpu.py tests/test_entry_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8k/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r8k/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d.get("diagnostics",{}).get("rehearsal_ms"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8k/d$r.json 2>gpurun_out/r8k/d$r.err; fatal $? d; echo "driver-shaped + rehearsal r$r $(ms gpurun_out/r8k/d$r.json)"
done
TDP_GPU_PEER=1 timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 --no-diag > gpurun_out/r8k/peer2.json 2>gpurun_out/r8k/peer2.err; fatal $? peer2; echo "peer W=2 on one GPU $(ms gpurun_out/r8k/peer2.json)"
echo done
