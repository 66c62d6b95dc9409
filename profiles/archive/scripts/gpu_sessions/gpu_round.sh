#!/bin/bash
# One gpurun call: GPU tests, smoke, benches (native vs stock torch), rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained so the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-100}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps $STEPS --warmup 20 > gpurun_out/bench_tdp.json 2> gpurun_out/bench_tdp.err && \
timeout -k 10 300 python bench.py --impl torch --steps $STEPS --warmup 20 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tdp -o run -- python3 bench.py --steps 30 --warmup 10 > gpurun_out/prof_tdp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_torch -o run -- python3 bench.py --impl torch --steps 30 --warmup 10 > gpurun_out/prof_torch.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench_tdp.json gpurun_out/bench_torch.json 2>/dev/null
exit $rc
