#!/bin/bash
# Execution-mode sweep on one MI355X after the "eager collectives on the compute stream" change:
# the 1-rank collective rehearsal (TDP_FORCE_COLLECTIVE=1) per stream mode / bucket size / fused
# optimizer, AlexNet native vs stock, and kernel traces (with timestamps, for idle-gap analysis)
# of the default eager step and of the rehearsal.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/m6
export TMPDIR=/tmp
O=gpurun_out/m6
B="python bench.py --steps 200 --warmup 30"
timeout -k 10 120 $B > $O/eager.json 2> $O/eager.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 $B > $O/coll_compute.json 2> $O/coll_compute.err && \
TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=side timeout -k 10 120 $B > $O/coll_side.json 2> $O/coll_side.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 $B --bucket-mb 256 > $O/coll_compute_b256.json 2> $O/coll_compute_b256.err && \
TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=side timeout -k 10 120 $B --bucket-mb 64 > $O/coll_side_b64.json 2> $O/coll_side_b64.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 $B --fused-opt on > $O/coll_compute_fused.json 2> $O/coll_compute_fused.err && \
timeout -k 10 120 $B --fused-opt on > $O/fused.json 2> $O/fused.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 120 $B --graph > $O/coll_graph.json 2> $O/coll_graph.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 20 --warmup 5 > $O/alex_tdp.json 2> $O/alex_tdp.err && \
timeout -k 10 200 python bench.py --model alexnet --impl torch --steps 20 --warmup 5 > $O/alex_torch.json 2> $O/alex_torch.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_eager -o run -- python3 bench.py --steps 30 --warmup 10 > $O/prof_eager.log 2>&1 && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_coll -o run -- python3 bench.py --steps 30 --warmup 10 > $O/prof_coll.log 2>&1
rc=$?
for f in $O/*.json; do echo "$f: $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null)"; done
exit $rc
