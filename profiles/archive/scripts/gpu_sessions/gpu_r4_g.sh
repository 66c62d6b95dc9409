#!/bin/bash
# 128-wide tiles for skinny-M GEMMs under split-bf16: benches + GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for cfg in "toy_mlp:" "toy_mlp:--optim adam" "toy_mlp:--syncbn" "alexnet:--steps 20 --warmup 5" "alexnet:--optim adam --steps 20 --warmup 5"; do
  m=${cfg%%:*}; extra=${cfg#*:}; tag=$(echo "$m $extra" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python bench.py --model $m $extra > gpurun_out/r4g_$tag.json 2>/dev/null; fatal $? "bench $tag"
  echo "$tag $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"]["final_loss"], d.get("diagnostics"))' gpurun_out/r4g_$tag.json)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_pytest.log; fatal $rc pytest
