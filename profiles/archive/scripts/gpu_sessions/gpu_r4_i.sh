#!/bin/bash
# Replicated factored update: GPU tests + one-GPU rehearsal of the multi-GPU schedule, both modes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_factor_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4i_factor.log 2>&1
rc=$?; tail -4 gpurun_out/r4i_factor.log; fatal $rc factor_tests
for e in 0 1; do for o in sgd adam; do
  TDP_FACTOR_REPLICATE=$e timeout -k 10 300 python bench.py --optim $o > gpurun_out/r4i_${o}_rep$e.json 2>/dev/null; fatal $? "bench $o $e"
  echo "rep=$e $o $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d.get("diagnostics"))' gpurun_out/r4i_${o}_rep$e.json)"
done; done
