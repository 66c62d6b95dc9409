#!/bin/bash
# Is the driver's short bench (20 steps after 5 warm-up) slower than long runs, and why?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for sw in "20 5" "20 5" "20 100" "100 5" "100 20" "400 5" "20 5"; do
  set -- $sw
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-diag > gpurun_out/r3c_$1_$2.json 2>/dev/null; fatal $? "bench $sw"
  echo "steps=$1 warmup=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3c_$1_$2.json)"
done
timeout -k 10 200 python scripts/step_timeline.py > gpurun_out/r3c_timeline.txt 2>&1; fatal $? timeline
cat gpurun_out/r3c_timeline.txt
