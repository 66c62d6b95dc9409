#!/bin/bash
# Host-side (Python) cost of the eager toy-MLP step: cProfile of bench.py, top functions by self time.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r21; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 python -m cProfile -o $O/bench.prof bench.py --steps 1000 --warmup 30 > $O/mlp.json 2> $O/mlp.err && \
python -c "
import pstats
s = pstats.Stats('$O/bench.prof')
s.sort_stats('tottime').print_stats(45)
s.sort_stats('cumulative').print_stats(60)
" > $O/pstats.txt 2>&1
