#!/bin/bash
# Why does an eager side comm stream cost ~1 ms/step? Stream priority variants + kernel and HIP
# runtime traces of the side-stream rehearsal (GPU idle gaps vs host-side blocking calls).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/s7
export TMPDIR=/tmp
O=gpurun_out/s7
B="python bench.py --steps 200 --warmup 30"
export TDP_FORCE_COLLECTIVE=1 TDP_COMM_STREAM=side
TDP_COMM_PRIORITY=normal timeout -k 10 120 $B > $O/side_normal.json 2> $O/side_normal.err && \
TDP_COMM_PRIORITY=blocking timeout -k 10 120 $B > $O/side_blocking.json 2> $O/side_blocking.err && \
timeout -k 10 120 $B --fused-opt on > $O/side_fused.json 2> $O/side_fused.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof_side -o run -- python3 bench.py --steps 20 --warmup 10 > $O/prof_side.log 2>&1
rc=$?
for f in $O/*.json; do echo "$f: $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null)"; done
exit $rc
