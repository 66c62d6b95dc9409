#!/bin/bash
# Full GPU suite + smoke on the current tree; comm-CU reservation A/B; rehearsal vs dp1;
# AlexNet / ResNet-50 / Adam / SyncBN / Accelerate benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5i_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5i_pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5i_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r5i_smoke.log; fatal $rc smoke
for r in 1 2; do for c in 0 8 16; do
  timeout -k 10 200 python bench.py --comm-cus $c --no-diag > gpurun_out/r5i_cus$c.json 2>/dev/null; fatal $? "cus $c"
  echo "comm_cus $c round $r $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r5i_cus$c.json)"
done; done
timeout -k 10 300 python bench.py > gpurun_out/r5i_default.json 2>/dev/null; fatal $? default
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("default", d["ms_per_step"], d["diagnostics"])' gpurun_out/r5i_default.json
for cfg in "toy_mlp:--optim adam" "toy_mlp:--syncbn" "toy_mlp:--api accelerate" "alexnet:--steps 20 --warmup 5" "resnet50:--steps 20 --warmup 5"; do
  m=${cfg%%:*}; extra=${cfg#*:}; tag=$(echo "$m $extra" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python bench.py --model $m $extra --no-diag > gpurun_out/r5i_$tag.json 2>/dev/null; fatal $? "bench $tag"
  echo "$tag $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' gpurun_out/r5i_$tag.json)"
done
echo done
