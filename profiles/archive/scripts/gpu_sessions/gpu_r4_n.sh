#!/bin/bash
# Round-2 end-of-session verification of the final tree: GPU suite, smoke, driver-shaped benches, MLP kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4n_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4n_pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r4n_smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4n_driver_shaped.json 2> gpurun_out/r4n_driver_shaped.err; fatal $? bench_driver
tail -1 gpurun_out/r4n_driver_shaped.json
timeout -k 10 300 python bench.py > gpurun_out/r4n_default.json 2>/dev/null; fatal $? bench_default
for cfg in "toy_mlp:--optim adam" "toy_mlp:--syncbn" "toy_mlp:--api accelerate" "alexnet:--steps 20 --warmup 5" "alexnet:--optim adam --steps 20 --warmup 5" "resnet50:--steps 20 --warmup 5"; do
  m=${cfg%%:*}; extra=${cfg#*:}; tag=$(echo "$m $extra" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python bench.py --model $m $extra > gpurun_out/r4n_$tag.json 2>/dev/null; fatal $? "bench $tag"
done
for f in gpurun_out/r4n_default.json gpurun_out/r4n_toy_mlp*.json gpurun_out/r4n_alexnet*.json gpurun_out/r4n_resnet50*.json; do
  echo "$f $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d.get("diagnostics"))' $f)"; done
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4n_prof_mlp" -o mlp -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-diag > "$R/gpurun_out/r4n_prof_mlp.log" 2>&1; fatal $? prof_mlp
echo done
