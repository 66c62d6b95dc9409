#!/bin/bash
# Round 4: peer-memory vehicle -- collectives, captured multi-rank step with real peers, stall
# timeouts, RCCL watchdog; bench self-launch through the vehicle (captured W=2, full toy MLP).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8b; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=10
timeout -k 10 900 python -u -m pytest tests/test_peer_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r8b/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r8b/pytest.log | tail -25; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(d["n_gpus"], d["ms_per_step"], d["value"], c.get("final_loss"), c["sync"]["captured"], c["sync"]["replicas_identical"], c["sync"]["modes"]["fc1.weight"], c["sync"].get("factor_tuning"), d.get("diagnostics"))' $1; }
TDP_GPU_PEER=1 timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/r8b/w2.json 2>gpurun_out/r8b/w2.err; fatal $? w2; echo "peer W=2 headline dims: $(ms gpurun_out/r8b/w2.json)"
echo done
