#!/bin/bash
# Bound experiment on the CNNs: conv GEMMs with no A split (EXP=1), no B split (EXP=2), none (3).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6v; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' $1; }
for m in resnet50 alexnet; do for e in 0 1 2 3; do
TDP_GEMM_EXP=$e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r6v/$m$e.json 2>/dev/null; fatal $? $m$e
echo "$m exp $e $(ms gpurun_out/r6v/$m$e.json)"
done; done
echo done
