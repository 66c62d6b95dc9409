#!/bin/bash
# One-launch batch gather: GPU suite, smoke, headline bench x2, AlexNet, kernel stats.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r27; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp.json 2>> $O/mlp.err && \
timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp.json 2>> $O/mlp.err && \
timeout -k 10 120 python bench.py >> $O/mlp_default.json 2>> $O/mlp_default.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 > $O/alex.json 2> $O/alex.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 > $O/prof_mlp.log 2>&1
rc=$?
tail -n 1 $O/pytest.log; tail -n 1 $O/smoke.log
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
grep -i gather $O/prof_mlp/run_kernel_stats.csv | cut -c1-160
exit $rc
