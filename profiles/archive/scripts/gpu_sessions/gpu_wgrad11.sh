#!/bin/bash
# Weight-gradient plan sweep (AlexNet + ResNet-50 conv shapes), CNN numerics, AlexNet per-layer.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/w11; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/sweep_wgrad.py alexnet 128 > $O/sweep_alexnet.jsonl 2> $O/sweep_alexnet.err && \
timeout -k 10 300 python scripts/bench_conv.py alexnet 128 > $O/conv_alexnet.jsonl 2> $O/conv_alexnet.err && \
timeout -k 10 500 python scripts/sweep_wgrad.py resnet50 128 > $O/sweep_r50.jsonl 2> $O/sweep_r50.err
rc=$?
tail -3 $O/pytest.log
grep best $O/sweep_alexnet.jsonl; tail -1 $O/conv_alexnet.jsonl; grep best $O/sweep_r50.jsonl
exit $rc
