#!/bin/bash
# Per-layer ResNet-50 conv timings; MLP headline bench + kernel stats (seeded backward).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r2g_mlp.json 2> gpurun_out/r2g_mlp.err
rc=$?; cat gpurun_out/r2g_mlp.json; fatal $rc mlp
timeout -k 10 300 python scripts/bench_conv.py resnet50 128 > gpurun_out/r2g_conv_r50.jsonl 2> gpurun_out/r2g_conv.err
fatal $? conv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp_g -o mlp -- python3 bench.py --steps 50 --warmup 10 --no-diag > gpurun_out/prof_mlp_g.log 2>&1
fatal $? profmlp
