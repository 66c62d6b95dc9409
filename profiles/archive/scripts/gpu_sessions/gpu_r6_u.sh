#!/bin/bash
# Bound experiment: the weight-gradient + SGD epilogue GEMMs with no VALU split at all
# (TDP_GEMM_EXP=3, timing only, numerically wrong) vs the real split.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6u; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for e in 0 3; do
TDP_GEMM_EXP=$e timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6u/p$e -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6u/p$e.log 2>&1; fatal $? p$e
python3 scripts/step_kernels.py $(find gpurun_out/r6u/p$e -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6u/k$e.md
echo "exp $e"; head -5 gpurun_out/r6u/k$e.md
done
echo done
