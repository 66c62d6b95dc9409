#!/bin/bash
# Linear split-K reduce fused into the following BatchNorm1d's launch: tests (bitwise vs separate
# launches, BN kernels, DDP / peer SyncBN), SyncBN-config A/B, kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11c; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests/test_ddp_gpu.py tests/test_gemm_planes_gpu.py tests/test_peer_gpu.py tests/test_tensor_parallel_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r11c/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r11c/tests.log; grep -E "FAILED|Error" gpurun_out/r11c/tests.log | head; fatal $rc tests
for i in 1 2 3; do
timeout -k 10 300 python scripts/run_with_variant.py --no-linear-bn -- bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r11c/sep_$i.json 2> gpurun_out/r11c/sep_$i.err; fatal $? sep
timeout -k 10 300 python bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r11c/fused_$i.json 2> gpurun_out/r11c/fused_$i.err; fatal $? fused
python3 -c 'import json,sys; [print(f, json.load(open(f))["ms_per_step"], json.load(open(f))["config"]["final_loss"]) for f in sys.argv[1:]]' gpurun_out/r11c/sep_$i.json gpurun_out/r11c/fused_$i.json
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r11c/sbn -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r11c/sbn.log 2>&1; fatal $? sbn
T=$(find gpurun_out/r11c/sbn -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r11c/syncbn_kernels.md; cat gpurun_out/r11c/syncbn_kernels.md
echo done
