#!/bin/bash
# Full GPU suite + smoke on the planes / head-fused tree, default bench (captured dp1), kernel
# table of the captured step, CNN eager vs graph.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6k; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6k/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6k/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r6k/smoke.log; fatal $rc smoke
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"]["impl"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/r6k/default.json 2>gpurun_out/r6k/default.err; fatal $? default; echo "default r$r $(ms gpurun_out/r6k/default.json)"
TDP_HEAD_FUSED=0 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6k/nohead.json 2>/dev/null; fatal $? nohead; echo "nohead r$r $(ms gpurun_out/r6k/nohead.json)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r6k/driver.json 2>/dev/null; fatal $? driver; echo "driver-shaped r$r $(ms gpurun_out/r6k/driver.json)"
done
python3 -c 'import json; d=json.load(open("gpurun_out/r6k/default.json")); print(d["diagnostics"])'
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6k/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6k/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6k/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6k/mlp_kernels.md
cat gpurun_out/r6k/mlp_kernels.md
for m in alexnet resnet50; do for mode in "" "--graph"; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag $mode > gpurun_out/r6k/$m$mode.json 2>/dev/null; fatal $? "$m $mode"; echo "$m $mode $(ms gpurun_out/r6k/$m$mode.json)"
done; done
echo done
