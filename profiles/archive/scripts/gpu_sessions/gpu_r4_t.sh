#!/bin/bash
# Final tree: GPU suite, smoke, driver-shaped bench, default bench, kernel stats of the default MLP step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4t_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4t_pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4t_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r4t_smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4t_driver_shaped.json 2> gpurun_out/r4t_driver_shaped.err; fatal $? bench_driver
tail -1 gpurun_out/r4t_driver_shaped.json
timeout -k 10 300 python bench.py > gpurun_out/r4t_default.json 2>/dev/null; fatal $? bench_default
echo "default $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d.get("diagnostics"))' gpurun_out/r4t_default.json)"
