#!/bin/bash
# Baseline for the flat Adam kernel change: multi-GPU-schedule rehearsal with Adam (per-bucket update).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${TDP_RUN:-r35}; mkdir -p $O; export TMPDIR=/tmp
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 --optim adam >> $O/adam_coll.json 2>> $O/adam_coll.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 --optim adam >> $O/adam_coll.json 2>> $O/adam_coll.err
rc=$?
echo "$(grep -o '"ms_per_step": [0-9.]*' $O/adam_coll.json | tr '\n' ' ')"
exit $rc
