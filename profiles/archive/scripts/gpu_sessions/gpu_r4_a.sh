#!/bin/bash
# Re-entry verification: full GPU suite, smoke, default bench, per-model benches, kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4a_pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r4a_smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py > gpurun_out/r4a_default.json 2> gpurun_out/r4a_default.err; fatal $? bench_default
tail -1 gpurun_out/r4a_default.json
for m in alexnet resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r4a_$m.json 2> gpurun_out/r4a_$m.err; fatal $? "bench $m"
  echo "$m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' gpurun_out/r4a_$m.json)"
done
timeout -k 10 300 python bench.py --model alexnet --optim adam --steps 20 --warmup 5 > gpurun_out/r4a_alexnet_adam.json 2> /dev/null; fatal $? "bench alexnet adam"
echo "alexnet adam $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' gpurun_out/r4a_alexnet_adam.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4a_prof_r50 -o r50 -- python3 bench.py --model resnet50 --steps 10 --warmup 3 --no-diag > gpurun_out/r4a_prof_r50.log 2>&1; fatal $? prof_r50
echo done
