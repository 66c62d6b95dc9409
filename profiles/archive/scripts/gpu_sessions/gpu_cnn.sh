#!/bin/bash
# CNN iteration: conv/pool kernel numerics, then AlexNet / ResNet-50 step time tdp vs stock torch.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-128}
timeout -k 10 600 python -m pytest tests/test_cnn_gpu.py -x -q > gpurun_out/pytest_cnn.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --batch $B --eager > gpurun_out/bench_r50_tdp_eager.json 2> gpurun_out/bench_r50_tdp_eager.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --batch $B --impl torch > gpurun_out/bench_r50_torch.json 2> gpurun_out/bench_r50_torch.err && \
timeout -k 10 300 python bench.py --model alexnet --steps 10 --warmup 3 --batch $B --eager > gpurun_out/bench_alex_tdp_eager.json 2> gpurun_out/bench_alex_tdp_eager.err && \
timeout -k 10 300 python bench.py --model alexnet --steps 10 --warmup 3 --batch $B --impl torch > gpurun_out/bench_alex_torch.json 2> gpurun_out/bench_alex_torch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 2 --batch $B --eager > gpurun_out/prof_r50.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50_torch -o run -- python3 bench.py --model resnet50 --impl torch --steps 5 --warmup 2 --batch $B > gpurun_out/prof_r50_torch.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_cnn.log; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench_r50*.json gpurun_out/bench_alex*.json 2>/dev/null
exit $rc
