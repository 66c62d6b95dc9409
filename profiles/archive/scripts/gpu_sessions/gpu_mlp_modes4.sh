#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDP_FORCE_COLLECTIVE=1
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 200 --warmup 30 "$@" > gpurun_out/mode4_$name.json 2> gpurun_out/mode4_$name.err; }
TDP_COMM_STREAM=side run side && \
TDP_COMM_STREAM=side TDP_COMM_PRIORITY=blocking run side_blocking && \
TDP_COMM_STREAM=side GPU_MAX_HW_QUEUES=1 run side_hwq1 && \
TDP_COMM_STREAM=side GPU_MAX_HW_QUEUES=2 run side_hwq2 && \
GPU_MAX_HW_QUEUES=1 run inline_hwq1 && \
TDP_FORCE_COLLECTIVE=0 run torch --impl torch && \
TDP_FORCE_COLLECTIVE=0 GPU_MAX_HW_QUEUES=1 run torch_hwq1 --impl torch && \
TDP_FORCE_COLLECTIVE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_torch_mlp -o run -- python3 bench.py --impl torch --steps 30 --warmup 10 > gpurun_out/prof_torch_mlp.log 2>&1
rc=$?
for f in gpurun_out/mode4_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
