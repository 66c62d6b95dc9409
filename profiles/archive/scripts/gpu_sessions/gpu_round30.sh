#!/bin/bash
# LDS-staged SGD epilogue as the default: full GPU suite, smoke, bench default, variants 16/24 x3, kernel stats.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r30; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 python bench.py > $O/mlp_default.json 2> $O/mlp_default.err || exit $?
for v in 16 24 16 24 16 24; do
  TDP_OPT_VARIANT=$v timeout -k 10 120 python bench.py --steps 500 --warmup 30 >> $O/mlp_v$v.json 2>> $O/mlp_v$v.err || exit $?
done
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/mlp_coll.json 2> $O/mlp_coll.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 > $O/prof_mlp.log 2>&1
rc=$?
tail -n 1 $O/pytest.log; tail -n 1 $O/smoke.log
for f in $O/*.json; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
