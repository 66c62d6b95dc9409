#!/bin/bash
# split-bf16 GEMM v2 (MFMA/VALU interleave, 2 waves/EU): numerics, micro-benchmark, model benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_emu_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_emu.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_emu.log; fatal $rc emu_tests
timeout -k 10 300 python -u scripts/bench_gemm_emu.py > gpurun_out/r4c_gemm_emu.jsonl 2>&1
rc=$?; cat gpurun_out/r4c_gemm_emu.jsonl | cut -c1-400; fatal $rc gemm_bench
for m in toy_mlp alexnet resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r4c_${m}.json 2>/dev/null; fatal $? "bench $m"
  echo "$m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' gpurun_out/r4c_${m}.json)"
done
