#!/bin/bash
# split-bf16 fp32 GEMM: numerics vs fp64, micro-benchmark vs native f32 MFMA, model benches, GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_emu_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4b_emu.log 2>&1
rc=$?; tail -25 gpurun_out/r4b_emu.log; fatal $rc emu_tests
timeout -k 10 300 python -u scripts/bench_gemm_emu.py > gpurun_out/r4b_gemm_emu.jsonl 2>&1
rc=$?; cat gpurun_out/r4b_gemm_emu.jsonl; fatal $rc gemm_bench
for e in 1 0; do for m in toy_mlp alexnet resnet50; do
  TDP_GEMM_EMU=$e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r4b_${m}_emu$e.json 2>/dev/null; fatal $? "bench $m $e"
  echo "$m emu=$e $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' gpurun_out/r4b_${m}_emu$e.json)"
done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r4b_pytest.log; fatal $rc pytest
