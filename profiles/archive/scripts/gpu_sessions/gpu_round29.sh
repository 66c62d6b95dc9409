#!/bin/bash
# LDS-staged SGD epilogue (TDP_OPT_VARIANT 16 / 24 = +non-temporal) vs the default (8): numerics
# through the fused-optimizer + kernel tests, headline bench x2 each, epilogue micro-benchmark.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r29; mkdir -p $O; export TMPDIR=/tmp
for v in 16 24; do
  TDP_OPT_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_v$v.log 2>&1 || exit $?
done
for v in 8 16 24 8 16 24; do
  TDP_OPT_VARIANT=$v timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp_v$v.json 2>> $O/mlp_v$v.err || exit $?
done
for v in 8 16 24; do
  TDP_OPT_VARIANT=$v timeout -k 10 150 python scripts/bench_opt_epilogue.py > $O/epi_v$v.jsonl 2> $O/epi_v$v.err || exit $?
done
for f in $O/pytest_v*.log; do echo "$f: $(tail -n 1 $f)"; done
for v in 8 16 24; do echo "v$v: $(grep -o '"ms_per_step": [0-9.]*' $O/mlp_v$v.json | tr '\n' ' ') $(grep -o '"final_loss": [0-9.e-]*' $O/mlp_v$v.json | tr '\n' ' ')"; grep '"fn": 2' $O/epi_v$v.jsonl | cut -c1-140; done
