#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDP_FORCE_COLLECTIVE=1
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 200 --warmup 30 "$@" > gpurun_out/mode3_$name.json 2> gpurun_out/mode3_$name.err; }
runr() { local name=$1; shift; timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 "$@" > gpurun_out/mode3_$name.json 2> gpurun_out/mode3_$name.err; }
TDP_COMM_STREAM=hostsync run eager_coll_hostsync --eager && \
TDP_COMM_STREAM=hostsync run eager_coll_hostsync_fused --eager --fused-opt on && \
runr r50_eager_coll --eager && TDP_COMM_STREAM=compute runr r50_eager_coll_inline --eager && \
TDP_COMM_STREAM=hostsync runr r50_eager_coll_hostsync --eager && runr r50_graph_coll && \
TDP_FORCE_COLLECTIVE=0 runr r50_eager_nocoll --eager
rc=$?
for f in gpurun_out/mode3_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
