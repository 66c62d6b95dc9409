#!/bin/bash
# Stream-hop penalty experiments for the eager multi-GPU schedule (rehearsed at world size 1).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDP_FORCE_COLLECTIVE=1
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 200 --warmup 30 "$@" > gpurun_out/mode2_$name.json 2> gpurun_out/mode2_$name.err; }
run eager_coll --eager && \
TDP_COMM_PRIORITY=normal run eager_coll_normprio --eager && \
TDP_COMM_STREAM=compute run eager_coll_inline --eager && \
TDP_COMM_STREAM=compute run eager_coll_inline_fused --eager --fused-opt on && \
TDP_COMM_PRIORITY=normal run eager_coll_normprio_fused --eager --fused-opt on && \
TDP_COMM_PRIORITY=normal run graph_coll_normprio_fused --fused-opt on && \
TDP_COMM_STREAM=compute run graph_coll_inline --fused-opt off
rc=$?
for f in gpurun_out/mode2_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
