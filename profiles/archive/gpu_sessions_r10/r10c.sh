#!/bin/bash
# head_ce with the row's input-gradient columns over 2 workgroups: numerics + dp1 kernel table + A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10c; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_head_ce_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r10c/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10c/tests.log; grep -E "FAILED|Error" gpurun_out/r10c/tests.log | head -5; fatal $rc tests
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10c/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10c/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r10c/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T head_ce 40 > gpurun_out/r10c/dp1_kernels.md; cat gpurun_out/r10c/dp1_kernels.md
for i in 1 2; do
for h in fused separate; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --head-loss $h --no-diag > gpurun_out/r10c/d${i}_$h.json 2> gpurun_out/r10c/d${i}_$h.err; fatal $? bench$i$h
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["final_loss"])' gpurun_out/r10c/d${i}_$h.json
done; done
echo done
