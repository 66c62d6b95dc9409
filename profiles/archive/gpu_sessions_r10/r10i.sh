#!/bin/bash
# In-place factored g gathers (the consumer's input-gradient GEMM writes g into its gather slot):
# the W-rank DDP paths (peer / relay vehicles, factored jobs, sync modes), the rehearsal's kernel
# table and the driver-shaped bench with its rehearsal diagnostic.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10i; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests/test_peer_gpu.py tests/test_factor_gpu.py tests/test_ddp_gpu.py tests/test_sync_gpu.py tests/test_relay_gpu.py tests/test_bench_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r10i/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10i/tests.log; grep -E "FAILED|Error" gpurun_out/r10i/tests.log | head -5; fatal $rc tests
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10i/reh -o kt -- python3 scripts/rehearsal_probe.py --steps 60 > gpurun_out/r10i/reh.log 2>&1; fatal $? reh
T=$(find gpurun_out/r10i/reh -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10i/reh_kernels.md; cat gpurun_out/r10i/reh_kernels.md
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r10i/d$i.json 2> gpurun_out/r10i/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r10i/d$i.json
done
TDP_GPU_PEER=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r10i/peer2.json 2> gpurun_out/r10i/peer2.err; fatal $? peer2
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(d["ms_per_step"], c["parallelism"], c["rung"], c["sync"]["replicas_identical"], c["sync"]["modes"].get("fc1.weight"))' gpurun_out/r10i/peer2.json
echo done
