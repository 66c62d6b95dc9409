#!/bin/bash
# Bias / head optimizer epilogues: GPU suite, kernel table, bench; rehearsal kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6o; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6o/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6o/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6o/b.json 2>/dev/null; fatal $? b; echo "default r$r $(ms gpurun_out/r6o/b.json)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r6o/d.json 2>/dev/null; fatal $? d; echo "driver-shaped $(ms gpurun_out/r6o/d.json)"
timeout -k 10 300 python bench.py --optim adam --no-diag > gpurun_out/r6o/adam.json 2>/dev/null; fatal $? adam; echo "adam $(ms gpurun_out/r6o/adam.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6o/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6o/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6o/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6o/mlp_kernels.md
cat gpurun_out/r6o/mlp_kernels.md
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6o/reh.json 2>/dev/null; fatal $? reh; echo "rehearsal $(ms gpurun_out/r6o/reh.json)"
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6o/prof2 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6o/prof2.log 2>&1; fatal $? prof2
python3 scripts/step_kernels.py $(find gpurun_out/r6o/prof2 -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6o/rehearsal_kernels.md
cat gpurun_out/r6o/rehearsal_kernels.md
echo done
