#!/bin/bash
# Final-tree evidence: dp1 kernel table / timeline, driver-shaped dp1 bench x2 with diagnostics.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9z; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9z/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r9z/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r9z/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9z/dp1_kernels.md
python3 scripts/step_timeline.py $T ce_fwd 40 > gpurun_out/r9z/dp1_timeline.md
cat gpurun_out/r9z/dp1_kernels.md
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r9z/d$i.json 2> gpurun_out/r9z/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(d["ms_per_step"], {k: g.get(k) for k in ("rehearsal_ms","tensor_rank_compute_ms","tensor_predicted_eff")})' gpurun_out/r9z/d$i.json
done
echo done
