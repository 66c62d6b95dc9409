#!/bin/bash
# Weight-gradient planner v2 (FN=2 when it does not pad, split-K target per CU): numerics, target sweep, AlexNet per-layer + step.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/w12; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/sweep_wgrad.py alexnet 128 targets > $O/tg_alexnet.jsonl 2> $O/tg_alexnet.err && \
timeout -k 10 300 python scripts/sweep_wgrad.py resnet50 128 targets > $O/tg_r50.jsonl 2> $O/tg_r50.err && \
timeout -k 10 300 python scripts/bench_conv.py alexnet 128 > $O/conv_alexnet.jsonl 2> $O/conv_alexnet.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 30 --warmup 5 > $O/alex.json 2> $O/alex.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.json 2> $O/r50.err
rc=$?
tail -3 $O/pytest.log
cat $O/tg_alexnet.jsonl $O/tg_r50.jsonl | cut -c1-250; tail -1 $O/conv_alexnet.jsonl; cat $O/alex.json $O/r50.json
exit $rc
