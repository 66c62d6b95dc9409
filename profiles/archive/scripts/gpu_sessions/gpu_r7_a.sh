#!/bin/bash
# Re-entry verification of the restored tree: GPU suite, smoke, default / driver-shaped benches,
# rehearsal (multi-GPU schedule at W=1) with and without the captured fork marker + kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7a; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7a/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r7a/pytest.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r7a/smoke.log 2>&1; fatal $? smoke; tail -2 gpurun_out/r7a/smoke.log
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7a/d.json 2>gpurun_out/r7a/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r7a/d.json)"
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7a/b.json 2>/dev/null; fatal $? b; echo "default r$r $(ms gpurun_out/r7a/b.json)"
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7a/reh.json 2>/dev/null; fatal $? reh; echo "rehearsal r$r $(ms gpurun_out/r7a/reh.json)"
TDP_GRAPH_FORK_MARKER=0 TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7a/reh0.json 2>/dev/null; fatal $? reh0; echo "rehearsal nomarker r$r $(ms gpurun_out/r7a/reh0.json)"
done
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7a/prof2 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r7a/prof2.log 2>&1; fatal $? prof2
python3 scripts/step_kernels.py $(find gpurun_out/r7a/prof2 -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7a/rehearsal_kernels.md
cat gpurun_out/r7a/rehearsal_kernels.md
echo done
