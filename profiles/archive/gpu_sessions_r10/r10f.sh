#!/bin/bash
# The N > 1 default (DDP ladder, dp{N}) at the headline dims on the peer vehicle (W ranks on ONE
# GPU): W = 2 / 4 / 8, with diagnostics -- a plumbing rehearsal of the driver's scaling run, not
# a multi-GPU number.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10f; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for n in 2 4 8; do
  TDP_GPU_PEER=1 TDP_PEER_TIMEOUT_S=60 timeout -k 10 400 python -u bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/r10f/w${n}.json 2> gpurun_out/r10f/w${n}.err; rc=$?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(sys.argv[1], d["ms_per_step"], c["parallelism"], c["rung"], c["fallbacks"], c["sync"]["replicas_identical"], c["sync"]["captured"], c["sync"]["modes"].get("fc1.weight"), {k: d.get("diagnostics",{}).get(k) for k in ("comm_ms","compute_ms","overlap_pct","predicted_step_ms")})' gpurun_out/r10f/w${n}.json; grep -A30 "raised" gpurun_out/r10f/w${n}.err | head -40; fatal $rc w$n
done
echo done
