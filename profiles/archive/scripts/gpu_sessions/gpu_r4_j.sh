#!/bin/bash
# Fused CE forward+gradient: kernel tests, MLP benches (SGD / Adam / SyncBN), AlexNet.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_k.log 2>&1
rc=$?; tail -2 gpurun_out/r4j_k.log; fatal $rc kernel_tests
for cfg in "toy_mlp:" "toy_mlp:--optim adam" "toy_mlp:--syncbn" "alexnet:--steps 20 --warmup 5"; do
  m=${cfg%%:*}; extra=${cfg#*:}; tag=$(echo "$m $extra" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python bench.py --model $m $extra > gpurun_out/r4j_$tag.json 2>/dev/null; fatal $? "bench $tag"
  echo "$tag $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"]["final_loss"], d.get("diagnostics"))' gpurun_out/r4j_$tag.json)"
done
