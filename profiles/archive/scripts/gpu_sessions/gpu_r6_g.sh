#!/bin/bash
# Kernel-level times of the planes GEMM bottleneck experiments (TDP_PLANES_EXP).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6g; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for e in 0 1 4 6 7; do
TDP_PLANES_EXP=$e timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6g/e$e -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6g/e$e.log 2>&1
fatal $? "exp $e"
done
echo ok
