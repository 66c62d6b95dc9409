#!/bin/bash
# Flat Adam kernel (2 float4 per stream in flight, non-temporal): GPU suite + the r35 Adam rehearsal.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r36; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r36/pytest.log 2>&1 || exit $?
tail -n 1 gpurun_out/r36/pytest.log
TDP_RUN=r36 bash scripts/gpu_round35.sh
