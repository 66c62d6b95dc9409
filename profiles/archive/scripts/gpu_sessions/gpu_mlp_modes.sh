#!/bin/bash
# Toy-MLP step time under every execution mode on one GPU (graph/eager x fused/unfused x
# real RCCL all-reduce), plus a kernel trace of the eager rehearsal of the multi-GPU schedule.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 200 --warmup 30 "$@" > gpurun_out/mode_$name.json 2> gpurun_out/mode_$name.err; }
run graph && run eager --eager && run graph_fused --fused-opt on && run eager_fused --eager --fused-opt on && \
TDP_FORCE_COLLECTIVE=1 run graph_coll && TDP_FORCE_COLLECTIVE=1 run eager_coll --eager && \
TDP_FORCE_COLLECTIVE=1 run graph_coll_fused --fused-opt on && TDP_FORCE_COLLECTIVE=1 run eager_coll_fused --eager --fused-opt on && \
run torch --impl torch && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eager_coll_fused -o run -- python3 bench.py --steps 30 --warmup 10 --eager --fused-opt on > gpurun_out/prof_eager_coll_fused.log 2>&1
rc=$?
for f in gpurun_out/mode_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
