#!/bin/bash
# One-launch one-rank BatchNorm1d: kernel / module tests, SyncBN-config A/B; then the final
# same-box refresh: dp1 kernel table, every BASELINE config at dp1 next to stock torch DDP, the
# SyncBN-config kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10x; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_gemm_planes_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r10x/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r10x/tests.log; grep -E "FAILED|Error" gpurun_out/r10x/tests.log | head; fatal $rc tests
for i in 1 2; do
timeout -k 10 300 python scripts/run_with_variant.py --no-local1d -- bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10x/sbn_off_$i.json 2> gpurun_out/r10x/sbn_off_$i.err; fatal $? sbnoff
timeout -k 10 300 python bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10x/sbn_on_$i.json 2> gpurun_out/r10x/sbn_on_$i.err; fatal $? sbnon
python3 -c 'import json,sys; [print(f, json.load(open(f))["ms_per_step"], json.load(open(f))["config"]["final_loss"]) for f in sys.argv[1:]]' gpurun_out/r10x/sbn_off_$i.json gpurun_out/r10x/sbn_on_$i.json
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10x/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10x/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r10x/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10x/dp1_kernels.md; cat gpurun_out/r10x/dp1_kernels.md
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py --no-diag "$@" > gpurun_out/r10x/$name.json 2> gpurun_out/r10x/$name.err; fatal $? $name
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["value"])' gpurun_out/r10x/$name.json
}
run d1 300 --steps 20 --warmup 5
run d2 300 --steps 20 --warmup 5
run mlp_tdp 300 --steps 100 --warmup 20
run mlp_torch 300 --steps 100 --warmup 20 --impl torch
run mlp_adam_tdp 300 --steps 100 --warmup 20 --optim adam
run mlp_adam_torch 300 --steps 100 --warmup 20 --optim adam --impl torch
run mlp_syncbn_tdp 300 --steps 100 --warmup 20 --syncbn
run mlp_syncbn_torch 300 --steps 100 --warmup 20 --syncbn --impl torch
run mlp_accel_tdp 300 --steps 100 --warmup 20 --api accelerate
run r50_tdp 400 --model resnet50 --steps 20 --warmup 5
run r50_torch 400 --model resnet50 --steps 20 --warmup 5 --impl torch
run alex_tdp 300 --model alexnet --steps 20 --warmup 5
run alex_torch 300 --model alexnet --steps 20 --warmup 5 --impl torch
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10x/sbn -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r10x/sbn.log 2>&1; fatal $? sbn
T=$(find gpurun_out/r10x/sbn -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10x/syncbn_kernels.md; cat gpurun_out/r10x/syncbn_kernels.md
echo done
