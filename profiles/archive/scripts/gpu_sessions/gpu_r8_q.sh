#!/bin/bash
# Round 4: headline bench repeats at the final tree (box-to-box spread check).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8q; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["vs_baseline"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r8q/d$r.json 2>gpurun_out/r8q/d$r.err; fatal $? d$r; echo "driver-shaped r$r $(ms gpurun_out/r8q/d$r.json)"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-diag > gpurun_out/r8q/l.json 2>gpurun_out/r8q/l.err; fatal $? l; echo "100 steps $(ms gpurun_out/r8q/l.json)"
echo done
