#!/bin/bash
# Round 4: two training steps per hipGraph replay in bench.py (--graph-steps 2) vs one:
# identical final loss (same kernels, same order), time per step, captured-step tests, the
# multi-rank bench on the peer vehicle.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8n; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d["config"].get("graph_steps"))' $1; }
for r in 1 2; do
for g in 1 2; do
timeout -k 10 300 python bench.py --no-diag --graph-steps $g > gpurun_out/r8n/g${g}_r$r.json 2>gpurun_out/r8n/g${g}_r$r.err; fatal $? g$g; echo "graph-steps $g r$r $(ms gpurun_out/r8n/g${g}_r$r.json)"
done; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8n/d.json 2>gpurun_out/r8n/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r8n/d.json)"
timeout -k 10 300 python bench.py --steps 21 --warmup 4 --no-diag --dataset 3200 > gpurun_out/r8n/odd.json 2>gpurun_out/r8n/odd.err; fatal $? odd; echo "odd steps / short epochs $(ms gpurun_out/r8n/odd.json)"
timeout -k 10 300 python bench.py --steps 21 --warmup 4 --no-diag --dataset 3200 --graph-steps 1 > gpurun_out/r8n/odd1.json 2>gpurun_out/r8n/odd1.err; fatal $? odd1; echo "odd steps / short epochs, 1 per graph $(ms gpurun_out/r8n/odd1.json)"
echo done
