#!/bin/bash
# Kernel table of the multi-GPU schedule rehearsed on one GPU (TDP_FORCE_COLLECTIVE=1: RCCL
# collectives kept, factored Linear sync, captured step).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6n; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"]["sync"])' $1; }
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6n/b.json 2>gpurun_out/r6n/b.err; fatal $? b; echo "rehearsal $(ms gpurun_out/r6n/b.json)"
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6n/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6n/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6n/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6n/kernels.md
cat gpurun_out/r6n/kernels.md
echo done
