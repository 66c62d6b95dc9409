#!/bin/bash
# Round 4: full GPU suite after the head_bwd race fix and the one-process Accelerate path,
# smoke, driver-shaped bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8h; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=15
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r8h/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r8h/pytest.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r8h/smoke.log 2>&1; fatal $? smoke; tail -1 gpurun_out/r8h/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8h/d.json 2>gpurun_out/r8h/d.err; fatal $? bench
python3 -c 'import json; d=json.load(open("gpurun_out/r8h/d.json")); print(d["ms_per_step"], d["value"], d["vs_baseline"], d.get("diagnostics",{}).get("rehearsal_ms"))'
echo done
