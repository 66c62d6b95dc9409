#!/bin/bash
# Driver-shaped (20 timed / 5 warm-up) vs long runs: what the short window still times.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2; do for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --device-warmup-ms 1000" "--steps 20 --warmup 40" "--steps 100 --warmup 20"; do
  timeout -k 10 300 python bench.py $args --no-diag > gpurun_out/r4o.json 2>/dev/null; fatal $? "bench $args"
  echo "$r [$args] $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4o.json)"
done; done
timeout -k 10 300 python scripts/step_timeline.py > gpurun_out/r4o_timeline.log 2>&1; tail -30 gpurun_out/r4o_timeline.log
