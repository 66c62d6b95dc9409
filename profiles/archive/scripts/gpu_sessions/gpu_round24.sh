#!/bin/bash
# Lean optimizer step/zero_grad wrappers: GPU tests, headline bench x2, kernel trace of the step.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r24; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp.json 2>> $O/mlp.err && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp.json 2>> $O/mlp.err && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 --optim adam >> $O/adam.json 2>> $O/adam.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 > $O/prof_mlp.log 2>&1
rc=$?
tail -n 1 $O/pytest.log
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
