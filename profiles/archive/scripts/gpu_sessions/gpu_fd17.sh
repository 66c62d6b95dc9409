#!/bin/bash
# Forward / input-gradient plan sweep (AlexNet, ResNet-50 shapes).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/fd17; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python scripts/sweep_conv_fd.py alexnet 128 > $O/fd_alexnet.jsonl 2> $O/fd_alexnet.err && \
timeout -k 10 400 python scripts/sweep_conv_fd.py resnet50 128 > $O/fd_r50.jsonl 2> $O/fd_r50.err
rc=$?
cat $O/fd_alexnet.jsonl $O/fd_r50.jsonl
exit $rc
