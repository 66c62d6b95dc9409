#!/bin/bash
# Kernel-stat profiles (toy MLP, AlexNet, ResNet-50) of the split-bf16 build, stock-torch MLP row, GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4e_prof_mlp" -o mlp -- python3 "$R/bench.py" --steps 50 --warmup 10 --device-warmup-ms 0 --no-diag > "$R/gpurun_out/r4e_prof_mlp.log" 2>&1; fatal $? prof_mlp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4e_prof_alexnet" -o alexnet -- python3 "$R/bench.py" --model alexnet --steps 10 --warmup 3 --device-warmup-ms 0 --no-diag > "$R/gpurun_out/r4e_prof_alexnet.log" 2>&1; fatal $? prof_alexnet
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4e_prof_r50" -o r50 -- python3 "$R/bench.py" --model resnet50 --steps 10 --warmup 3 --device-warmup-ms 0 --no-diag > "$R/gpurun_out/r4e_prof_r50.log" 2>&1; fatal $? prof_r50
timeout -k 10 300 python bench.py --impl torch > gpurun_out/r4e_mlp_torch.json 2>/dev/null; fatal $? torch_mlp
timeout -k 10 300 python bench.py > gpurun_out/r4e_mlp.json 2>/dev/null; fatal $? mlp
timeout -k 10 300 python bench.py --optim adam > gpurun_out/r4e_mlp_adam.json 2>/dev/null; fatal $? mlp_adam
timeout -k 10 300 python bench.py --syncbn > gpurun_out/r4e_mlp_syncbn.json 2>/dev/null; fatal $? mlp_syncbn
for f in r4e_mlp_torch r4e_mlp r4e_mlp_adam r4e_mlp_syncbn; do echo "$f $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d.get("diagnostics"))' gpurun_out/$f.json)"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_pytest.log; fatal $rc pytest
