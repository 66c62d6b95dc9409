#!/bin/bash
# Round 4: the previous layer's g gather issued one layer early (from the consumer's backward,
# after its gated input-gradient GEMM) and the factored job waiting on exactly its gathers:
# captured bitwise A/B, multi-rank parity on the peer vehicle, rehearsal A/B, peer benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8o; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=15
timeout -k 10 900 python -u -m pytest tests/test_factor_gpu.py tests/test_peer_gpu.py tests/test_relay_gpu.py tests/test_ddp_gpu.py tests/test_entry_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8o/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r8o/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d.get("diagnostics",{}).get("rehearsal_ms"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8o/d$r.json 2>gpurun_out/r8o/d$r.err; fatal $? d; echo "early g: driver-shaped + rehearsal r$r $(ms gpurun_out/r8o/d$r.json)"
timeout -k 10 300 python scripts/run_with_variant.py --no-early-g -- bench.py --steps 20 --warmup 5 > gpurun_out/r8o/n$r.json 2>gpurun_out/r8o/n$r.err; fatal $? n; echo "no early g: driver-shaped + rehearsal r$r $(ms gpurun_out/r8o/n$r.json)"
done
for w in 2 4; do
TDP_GPU_PEER=1 timeout -k 10 300 python bench.py --gpus $w --steps 30 --warmup 5 --no-diag > gpurun_out/r8o/peer$w.json 2>gpurun_out/r8o/peer$w.err; fatal $? peer$w; echo "peer W=$w on one GPU $(ms gpurun_out/r8o/peer$w.json)"
done
echo done
