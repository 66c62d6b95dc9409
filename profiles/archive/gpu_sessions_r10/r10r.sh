#!/bin/bash
# Prefetched gather: bit-identity tests, A/B of the dp1 step (prefetch off / on, interleaved),
# kernel trace of the prefetched step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10r; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r10r/bench_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r10r/bench_tests.log; fatal $rc tests
for i in 1 2 3; do
for pf in off on; do
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-diag --prefetch $pf > gpurun_out/r10r/ab_${pf}_$i.json 2> gpurun_out/r10r/ab_${pf}_$i.err; fatal $? ab$pf$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["prefetch"], d["config"]["final_loss"])' gpurun_out/r10r/ab_${pf}_$i.json
done; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r10r/d1.json 2> gpurun_out/r10r/d1.err; fatal $? d1
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], d["value"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r10r/d1.json
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10r/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10r/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r10r/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10r/dp1_kernels.md; cat gpurun_out/r10r/dp1_kernels.md
echo done
