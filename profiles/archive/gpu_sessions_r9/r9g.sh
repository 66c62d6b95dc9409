#!/bin/bash
# lockstep wgrad+optimizer kernel: numerics, bench A/B vs the persistent kernel, kernel trace
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9g; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_wgrad_lockstep_gpu.py tests/test_ddp_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r9g/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r9g/pytest.log; fatal $rc pytest
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r9g/on$i.json 2>gpurun_out/r9g/on$i.err; fatal $? on$i
TDP_WGRAD_LOCKSTEP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r9g/off$i.json 2>gpurun_out/r9g/off$i.err; fatal $? off$i
python3 -c 'import json,sys; [print(f, json.load(open(f))["ms_per_step"], json.load(open(f))["config"]["final_loss"]) for f in sys.argv[1:]]' gpurun_out/r9g/on$i.json gpurun_out/r9g/off$i.json
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9g/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r9g/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r9g/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9g/dp1_kernels.md
head -8 gpurun_out/r9g/dp1_kernels.md
echo done
