#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_conv.py resnet50 128 > gpurun_out/convbench_r50.log 2>&1 && \
timeout -k 10 300 python scripts/bench_conv.py alexnet 128 > gpurun_out/convbench_alex.log 2>&1
