#!/bin/bash
# 4-way unrolled non-temporal flat SGD (the world > 1 sharded update): kernel + optimizer tests, the
# epilogue micro-benchmark's sgd_us column (flat SGD over fc1 / fc2), headline bench.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r34; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 150 python scripts/bench_opt_epilogue.py > $O/epi.jsonl 2> $O/epi.err && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 > $O/mlp.json 2> $O/mlp.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/mlp_coll.json 2> $O/mlp_coll.err
rc=$?
tail -n 1 $O/pytest.log
grep '"fn": 2' $O/epi.jsonl | cut -c1-120
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
exit $rc
