#!/bin/bash
# Round 5 first contact: driver-shaped bench x2 and the dp1 kernel trace / timeline at the
# round-4 tree (baseline for this round's changes).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9a; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r9a/d$i.json 2>gpurun_out/r9a/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d.get("diagnostics",{}).get("rehearsal_ms"))' gpurun_out/r9a/d$i.json
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9a/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r9a/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r9a/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9a/dp1_kernels.md
python3 scripts/step_timeline.py $T ce_fwd 40 > gpurun_out/r9a/dp1_timeline.md
cat gpurun_out/r9a/dp1_kernels.md
echo done
