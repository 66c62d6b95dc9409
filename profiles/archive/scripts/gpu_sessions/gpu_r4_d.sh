#!/bin/bash
# Re-tune the conv plan table under split-bf16 GEMM products, then re-bench the CNNs with it.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u scripts/tune_conv_plans.py gpurun_out/r4d_plans.json resnet50:128 alexnet:128 > gpurun_out/r4d_tune.jsonl 2> gpurun_out/r4d_tune.err
rc=$?; tail -2 gpurun_out/r4d_tune.jsonl | cut -c1-300; fatal $rc tune
cp gpurun_out/r4d_plans.json tutorial_torch_distributed_data_parallel_amd/perfdb/gfx950_conv_plans.json
for m in alexnet resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r4d_${m}.json 2>/dev/null; fatal $? "bench $m"
  echo "$m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' gpurun_out/r4d_${m}.json)"
done
