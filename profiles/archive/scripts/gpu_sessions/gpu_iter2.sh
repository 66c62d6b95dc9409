#!/bin/bash
# Iteration: CNN numerics, ResNet-50 graph/eager timing + kernel profile, MLP eager host profile.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-128}
timeout -k 10 600 python -m pytest tests/test_cnn_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_cnn.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --batch $B > gpurun_out/bench_r50_tdp.json 2> gpurun_out/bench_r50_tdp.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 2 --batch $B --eager > gpurun_out/prof_r50.log 2>&1 && \
timeout -k 10 300 python -m cProfile -o gpurun_out/eager.prof bench.py --eager --steps 300 --warmup 20 > gpurun_out/eager_prof_bench.json 2>&1 && \
python - > gpurun_out/eager_prof.txt <<'PY'
import pstats
s = pstats.Stats("gpurun_out/eager.prof")
s.sort_stats("tottime").print_stats(40)
s.sort_stats("cumtime").print_stats(50)
PY
rc=$?
tail -3 gpurun_out/pytest_cnn.log; cat gpurun_out/bench_r50_tdp.json 2>/dev/null | tail -1
exit $rc
