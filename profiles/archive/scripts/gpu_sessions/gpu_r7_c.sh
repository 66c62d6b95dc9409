#!/bin/bash
# Full GPU suite + smoke on the current tree; driver-shaped headline; config benches (SyncBN, Adam,
# Accelerate facade); CNNs captured vs eager at dp1.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7c; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7c/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r7c/pytest.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r7c/smoke.log 2>&1; fatal $? smoke; tail -1 gpurun_out/r7c/smoke.log
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"))' $1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7c/d.json 2>gpurun_out/r7c/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r7c/d.json)"
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7c/b.json 2>/dev/null; fatal $? b; echo "default 100 steps $(ms gpurun_out/r7c/b.json)"
timeout -k 10 300 python bench.py --syncbn --no-diag > gpurun_out/r7c/sbn.json 2>/dev/null; fatal $? sbn; echo "syncbn $(ms gpurun_out/r7c/sbn.json)"
timeout -k 10 300 python bench.py --optim adam --no-diag > gpurun_out/r7c/adam.json 2>/dev/null; fatal $? adam; echo "adam $(ms gpurun_out/r7c/adam.json)"
timeout -k 10 300 python bench.py --api accelerate --no-diag > gpurun_out/r7c/acc.json 2>/dev/null; fatal $? acc; echo "accelerate $(ms gpurun_out/r7c/acc.json)"
for m in resnet50 alexnet; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r7c/$m.json 2>/dev/null; fatal $? $m; echo "$m eager $(ms gpurun_out/r7c/$m.json)"
timeout -k 10 300 python bench.py --model $m --graph --steps 20 --warmup 5 --no-diag > gpurun_out/r7c/${m}_g.json 2>gpurun_out/r7c/${m}_g.err; fatal $? ${m}_g; echo "$m graph $(ms gpurun_out/r7c/${m}_g.json)"
done

timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7c/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r7c/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r7c/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7c/mlp_kernels.md
python3 scripts/step_timeline.py $(find gpurun_out/r7c/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7c/mlp_timeline.md
cat gpurun_out/r7c/mlp_timeline.md
echo done
