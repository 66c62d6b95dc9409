#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_cnn_gpu.py -x -q > gpurun_out/pytest_cnn.log 2>&1 && \
timeout -k 10 600 python scripts/bench_conv.py resnet50 128 > gpurun_out/convbench_r50.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bench_r50_tdp.json 2> gpurun_out/bench_r50_tdp.err && \
timeout -k 10 300 python bench.py --model alexnet --steps 10 --warmup 3 > gpurun_out/bench_alex_tdp.json 2> gpurun_out/bench_alex_tdp.err
rc=$?
tail -2 gpurun_out/pytest_cnn.log; tail -1 gpurun_out/bench_r50_tdp.json; tail -1 gpurun_out/bench_alex_tdp.json
exit $rc
