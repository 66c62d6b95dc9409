#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/eager.prof bench.py --eager --steps 300 --warmup 20 > gpurun_out/eager_prof_bench.json 2>&1 && \
python - > gpurun_out/eager_prof.txt <<'PY'
import pstats
s = pstats.Stats("gpurun_out/eager.prof")
s.sort_stats("tottime").print_stats(45)
s.sort_stats("cumtime").print_stats(60)
PY
