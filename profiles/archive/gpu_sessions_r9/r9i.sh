#!/bin/bash
# rehearsal anatomy: dp1 vs rehearsal vs rehearsal without one-rank collectives (kernel traces)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9i; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for v in dp1:0:0 reh:1:0 sched:1:1; do
  IFS=: read name fc sk <<< "$v"
  TDP_FORCE_COLLECTIVE=$fc TDP_SKIP_COLLECTIVES=$sk timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9i/$name -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r9i/$name.log 2>&1; fatal $? $name
  T=$(find gpurun_out/r9i/$name -name '*kernel_trace.csv' | head -1)
  python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9i/${name}_kernels.md
  python3 scripts/step_timeline.py $T ce_fwd 40 > gpurun_out/r9i/${name}_timeline.md
  echo "== $name"; head -16 gpurun_out/r9i/${name}_kernels.md
done
echo done
