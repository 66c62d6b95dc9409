#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDP_FORCE_COLLECTIVE=1
export GPU_MAX_HW_QUEUES=2
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 200 --warmup 30 "$@" > gpurun_out/mode5_$name.json 2> gpurun_out/mode5_$name.err; }
runr() { local name=$1; shift; timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 "$@" > gpurun_out/mode5_$name.json 2> gpurun_out/mode5_$name.err; }
TDP_COMM_STREAM=side run side && run auto && TDP_COMM_STREAM=side run side_fused --fused-opt on && \
run graph --graph && run graph_fused --graph --fused-opt on && \
TDP_FORCE_COLLECTIVE=0 run nocoll && \
TDP_COMM_STREAM=side runr r50_side && runr r50_auto && \
TDP_COMM_STREAM=side timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_side_hwq2 -o run -- python3 bench.py --steps 30 --warmup 10 --fused-opt on > gpurun_out/prof_side_hwq2.log 2>&1
rc=$?
for f in gpurun_out/mode5_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
