#!/bin/bash
# Validation of the tree with the paired launch: full GPU tier, smoke, driver-shaped bench x2,
# peer-vehicle dp2 record, dp1 kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10q; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r10q/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r10q/gpu_suite.log; grep -E "FAILED|Error" gpurun_out/r10q/gpu_suite.log | head -5; fatal $rc suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r10q/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r10q/smoke.log; fatal $rc smoke
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r10q/d$i.json 2> gpurun_out/r10q/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], d["value"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r10q/d$i.json
done
TDP_GPU_PEER=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-diag > gpurun_out/r10q/peer2.json 2> gpurun_out/r10q/peer2.err; fatal $? peer2
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["parallelism"], d["config"].get("rung"))' gpurun_out/r10q/peer2.json
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10q/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10q/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r10q/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10q/dp1_kernels.md; cat gpurun_out/r10q/dp1_kernels.md
echo done
