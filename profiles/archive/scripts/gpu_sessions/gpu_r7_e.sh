#!/bin/bash
# Final-tree verification for the round: GPU suite, smoke, driver-shaped headline, kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7e; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r7e/pytest.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r7e/smoke.log 2>&1; fatal $? smoke; tail -1 gpurun_out/r7e/smoke.log
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"))' $1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7e/d.json 2>gpurun_out/r7e/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r7e/d.json)"
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7e/b.json 2>/dev/null; fatal $? b; echo "default 100 steps $(ms gpurun_out/r7e/b.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r7e/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r7e/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r7e/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7e/mlp_kernels.md
python3 scripts/step_timeline.py $(find gpurun_out/r7e/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7e/mlp_timeline.md
cat gpurun_out/r7e/mlp_timeline.md
echo done
