#!/bin/bash
# graph steps per replay: 4 (default) vs 8, driver-shaped, interleaved x3.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9w; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2 3; do
for g in 4 8; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g --no-diag > gpurun_out/r9w/g${g}_$i.json 2>/dev/null; fatal $? g$g
done
python3 -c 'import json,sys; print(*[(f[-10:], json.load(open(f))["ms_per_step"]) for f in sys.argv[1:]])' gpurun_out/r9w/g4_$i.json gpurun_out/r9w/g8_$i.json
done
echo done
