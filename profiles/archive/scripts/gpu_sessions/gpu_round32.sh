#!/bin/bash
# LDS-staged Adam epilogue (TDP_OPT_ADAM_VARIANT 16 / 24) vs the register epilogue (0): fused-optimizer
# tests per variant, Adam bench x2 each.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r32; mkdir -p $O; export TMPDIR=/tmp
for v in 16 24; do
  TDP_OPT_ADAM_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_v$v.log 2>&1 || exit $?
done
for v in 0 16 24 0 16 24; do
  TDP_OPT_ADAM_VARIANT=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --optim adam >> $O/adam_v$v.json 2>> $O/adam_v$v.err || exit $?
done
for f in $O/pytest_v*.log; do echo "$f: $(tail -n 1 $f)"; done
for v in 0 16 24; do echo "v$v: $(grep -o '"ms_per_step": [0-9.]*' $O/adam_v$v.json | tr '\n' ' ') $(grep -o '"final_loss": [0-9.e-]*' $O/adam_v$v.json | tr '\n' ' ')"; done
