#!/bin/bash
# Planes GEMM skeleton / split-count experiments (kernel trace per setting).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6h; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
run() { tag=$1; shift; env "$@" timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6h/$tag -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6h/$tag.log 2>&1; fatal $? $tag; }
run e7 TDP_PLANES_EXP=7
run e15 TDP_PLANES_EXP=15
run e8 TDP_PLANES_EXP=8
run s4 TDP_PLANES_SPLITS=4
run s8 TDP_PLANES_SPLITS=8
run s8e7 TDP_PLANES_SPLITS=8 TDP_PLANES_EXP=7
run c3s4 TDP_PLANES_CFG=3,0 TDP_PLANES_SPLITS=4
run c3s8 TDP_PLANES_CFG=3,0 TDP_PLANES_SPLITS=8
echo ok
