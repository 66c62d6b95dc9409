#!/bin/bash
# Full GPU test suite + flagship bench (graph and eager) + rehearsal of the multi-GPU comm path.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 300 python bench.py --eager > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py > gpurun_out/bench_coll_graph.json 2> gpurun_out/bench_coll_graph.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --eager > gpurun_out/bench_coll_eager.json 2> gpurun_out/bench_coll_eager.err && \
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --eager > gpurun_out/bench_r50_coll_eager.json 2> gpurun_out/bench_r50_coll_eager.err
rc=$?
tail -2 gpurun_out/pytest_gpu.log
for f in gpurun_out/bench_default.json gpurun_out/bench_eager.json gpurun_out/bench_coll_*.json gpurun_out/bench_r50_coll_eager.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
