#!/bin/bash
# Padded channels_last input + native flatten: full GPU suite, AlexNet / ResNet benches, AlexNet trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r2p_all.log 2>&1
rc=$?; grep -E "^FAILED|Error" gpurun_out/r2p_all.log | head -10; tail -2 gpurun_out/r2p_all.log; fatal $rc tests
for m in alexnet resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --no-diag > gpurun_out/r2p_$m.json 2>/dev/null; fatal $? $m
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2p_$m.json)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alex_p -o alex -- python3 bench.py --model alexnet --steps 10 --warmup 3 --no-diag > gpurun_out/prof_alex_p.log 2>&1
fatal $? alex
