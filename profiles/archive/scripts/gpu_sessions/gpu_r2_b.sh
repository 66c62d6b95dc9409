#!/bin/bash
# Bench diagnostics: world-1 rehearsal, forced multi-GPU diagnostics branch, graph mode, Adam.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py -q -k commbench --timeout 120 --timeout-method thread > gpurun_out/r2b_commbench.log 2>&1
rc=$?; tail -2 gpurun_out/r2b_commbench.log; fatal $rc commbench
for cfg in "default:" "graph:--graph" "adam:--optim adam" "adam_graph:--optim adam --graph"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 $args > gpurun_out/r2b_$name.json 2> gpurun_out/r2b_$name.err
  rc=$?; echo "$name rc=$rc"; cat gpurun_out/r2b_$name.json; fatal $rc $name
done
TDP_DIAG_MULTI=1 timeout -k 10 180 python bench.py --steps 100 --warmup 20 --graph > gpurun_out/r2b_diagmulti.json 2> gpurun_out/r2b_diagmulti.err
rc=$?; echo "diagmulti rc=$rc"; cat gpurun_out/r2b_diagmulti.json; fatal $rc diagmulti
timeout -k 10 120 python scripts/rccl_sweep.py --max-mib 64 --iters 5 > gpurun_out/r2b_sweep_w1.jsonl 2> gpurun_out/r2b_sweep.err
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/r2b_sweep_w1.jsonl
