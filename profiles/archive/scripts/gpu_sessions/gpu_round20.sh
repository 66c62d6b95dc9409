#!/bin/bash
# SGD optimizer-epilogue variants (TDP_OPT_VARIANT: 4 = whole-tile batch, 8 = non-temporal, 12 = both):
# numerics through the fused-optimizer tests, then headline bench + epilogue microbench per variant.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r20; mkdir -p $O; export TMPDIR=/tmp
for v in 4 8 12; do
  TDP_OPT_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_v$v.log 2>&1 || exit $?
done
for v in 0 4 8 12 0 4 8 12; do
  TDP_OPT_VARIANT=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 >> $O/mlp_v$v.json 2> $O/mlp_v$v.err || exit $?
done
for v in 0 4 8 12; do
  TDP_OPT_VARIANT=$v timeout -k 10 120 python scripts/bench_opt_epilogue.py > $O/epi_v$v.jsonl 2> $O/epi_v$v.err || exit $?
done
tail -1 $O/pytest_v*.log
for v in 0 4 8 12; do echo "v$v: $(grep -o '"ms_per_step": [0-9.]*' $O/mlp_v$v.json | tr '\n' ' ')"; grep '"fn": 2' $O/epi_v$v.jsonl; done
