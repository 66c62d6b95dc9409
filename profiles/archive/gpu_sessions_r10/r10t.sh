#!/bin/bash
# BN partial-statistics merge in 64-tile chunks: BN / CNN tests, ResNet-50 and AlexNet dp1 eager
# and captured, ResNet-50 kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10t; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r10t/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10t/tests.log; fatal $rc tests
show() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(sys.argv[1], d["ms_per_step"], c["sync"]["captured"] if c.get("sync") else None, c["final_loss"])' $1; }
for i in 1 2; do
for m in resnet50 alexnet; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r10t/${m}_e_$i.json 2> gpurun_out/r10t/${m}_e_$i.err; fatal $? ${m}e
show gpurun_out/r10t/${m}_e_$i.json
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag --graph > gpurun_out/r10t/${m}_g_$i.json 2> gpurun_out/r10t/${m}_g_$i.err; fatal $? ${m}g
show gpurun_out/r10t/${m}_g_$i.json
done; done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r10t/r50 -o kt -- python3 bench.py --model resnet50 --steps 10 --warmup 3 --no-diag > gpurun_out/r10t/r50prof.log 2>&1; fatal $? prof
echo done
