#!/bin/bash
# Full GPU tests + smoke, headline bench (stdout must be ONE JSON line), Accelerate-API bench,
# stock torch, eager side-stream join variants (1-rank collective rehearsal), AlexNet per-layer.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r9
export TMPDIR=/tmp
O=gpurun_out/r9
B="python bench.py --steps 200 --warmup 30"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 $B > $O/default.json 2> $O/default.err && \
timeout -k 10 120 $B --api accelerate > $O/accel.json 2> $O/accel.err && \
timeout -k 10 120 $B --impl torch > $O/torch.json 2> $O/torch.err && \
TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=hostjoin timeout -k 10 120 $B --fused-opt off > $O/coll_hostjoin.json 2> $O/coll_hostjoin.err && \
TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=nojoin timeout -k 10 120 $B --fused-opt off > $O/coll_nojoin.json 2> $O/coll_nojoin.err && \
TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=side TDP_BENCH_STREAM=1 timeout -k 10 120 $B --fused-opt off > $O/coll_side_ownstream.json 2> $O/coll_side_ownstream.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 $B --fused-opt off > $O/coll_compute.json 2> $O/coll_compute.err && \
timeout -k 10 300 python scripts/bench_conv.py alexnet 128 > $O/conv_alexnet.jsonl 2> $O/conv_alexnet.err
rc=$?
tail -3 $O/pytest.log
for f in $O/*.json; do echo "$f: lines=$(wc -l < $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["final_loss"])' 2>/dev/null)"; done
tail -1 $O/conv_alexnet.jsonl
exit $rc
