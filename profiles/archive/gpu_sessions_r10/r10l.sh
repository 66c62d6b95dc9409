#!/bin/bash
# planes split-K reduce with all partial loads in flight: planes tests + dp1 kernel table; then
# every BASELINE config at dp1 next to stock torch DDP (same box).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10l; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_bench_gpu.py tests/test_head_ce_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r10l/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r10l/tests.log; fatal $rc tests
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10l/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10l/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r10l/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10l/dp1_kernels.md; cat gpurun_out/r10l/dp1_kernels.md
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py --no-diag "$@" > gpurun_out/r10l/$name.json 2> gpurun_out/r10l/$name.err; fatal $? $name
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["value"])' gpurun_out/r10l/$name.json
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
echo done
