#!/bin/bash
# Kernel table of the current captured toy-MLP step + AlexNet / ResNet-50 sanity benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6m; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6m/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6m/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6m/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6m/mlp_kernels.md
cat gpurun_out/r6m/mlp_kernels.md
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' $1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r6m/d.json 2>/dev/null; fatal $? d; echo "driver-shaped $(ms gpurun_out/r6m/d.json)"
timeout -k 10 300 python bench.py --model alexnet --steps 20 --warmup 5 --no-diag > gpurun_out/r6m/a.json 2>/dev/null; fatal $? a; echo "alexnet $(ms gpurun_out/r6m/a.json)"
TDP_PLANES=0 timeout -k 10 300 python bench.py --model alexnet --steps 20 --warmup 5 --no-diag > gpurun_out/r6m/a0.json 2>/dev/null; fatal $? a0; echo "alexnet planes off $(ms gpurun_out/r6m/a0.json)"
echo done
