#!/bin/bash
# Re-entry verification: full GPU test suite, smoke(), headline bench, rocprof stats of the headline step.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r19; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 python bench.py > $O/mlp_default.json 2> $O/mlp_default.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/mlp.json 2> $O/mlp.err && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --impl torch > $O/mlp_torch.json 2> $O/mlp_torch.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/mlp_coll.json 2> $O/mlp_coll.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 > $O/prof_mlp.log 2>&1
rc=$?
tail -3 $O/pytest.log
cat $O/smoke.log | tail -2
for f in $O/*.json; do echo "$f: $(tail -1 $f)"; done
exit $rc
