#!/bin/bash
# Parameter-store policy (kOptPT) round 2: variant tests (SGD + Adam), SGD default (now 88) vs 24
# and Adam 88 vs 24, interleaved 100-step windows on one box; driver-shaped default bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10n; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
V=scripts/run_with_variant.py
show() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"])' $1; }
timeout -k 10 400 python -u -m pytest tests/test_sync_gpu.py -k epilogue_variants -q --timeout 200 --timeout-method thread > gpurun_out/r10n/variants.log 2>&1; rc=$?; tail -2 gpurun_out/r10n/variants.log; fatal $rc variants
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 300 python $V --sgd $v -- bench.py --steps 100 --warmup 20 --no-diag > gpurun_out/r10n/sgd${i}_$v.json 2> gpurun_out/r10n/sgd${i}_$v.err; fatal $? sgd$i$v; show gpurun_out/r10n/sgd${i}_$v.json
done; done
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 300 python $V --adam $v -- bench.py --optim adam --steps 100 --warmup 20 --no-diag > gpurun_out/r10n/adam${i}_$v.json 2> gpurun_out/r10n/adam${i}_$v.err; fatal $? adam$i$v; show gpurun_out/r10n/adam${i}_$v.json
done; done
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r10n/d$i.json 2> gpurun_out/r10n/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], d["value"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r10n/d$i.json
done
echo done
