#!/bin/bash
# Kernel table of the tensor-sharded step's per-rank compute at W = 8 (proxy, one GPU).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9n; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9n/kt -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 8 > gpurun_out/r9n/kt.log 2>&1; fatal $? kt
T=$(find gpurun_out/r9n/kt -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9n/tp8_kernels.md
cat gpurun_out/r9n/tp8_kernels.md
python3 scripts/step_timeline.py $T ce_fwd 2 > gpurun_out/r9n/tp8_timeline.md; head -60 gpurun_out/r9n/tp8_timeline.md
echo done
