#!/bin/bash
# Factored Linear-weight synchronisation: GPU tests, full GPU suite, one-GPU rehearsal benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_factor_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3e_factor.log 2>&1
rc=$?; tail -8 gpurun_out/r3e_factor.log; fatal $rc factor_tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3e_pytest.log; fatal $rc pytest
for e in TDP_FACTOR_SYNC=1 TDP_FACTOR_SYNC=0; do for m in toy_mlp alexnet; do
  env $e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r3e_${m}_$e.json 2>/dev/null; fatal $? "bench $m $e"
  echo "$m $e $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["diagnostics"])' gpurun_out/r3e_${m}_$e.json)"
done; done
