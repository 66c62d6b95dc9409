#!/bin/bash
# aux-stream conv weight gradient: bitwise test, ResNet-50 / AlexNet A/B (eager and captured);
# prefetch released at the head: toy-MLP A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10s; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py -k aux -v --timeout 200 --timeout-method thread > gpurun_out/r10s/aux_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r10s/aux_tests.log; fatal $rc tests
show() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(sys.argv[1], d["ms_per_step"], c.get("prefetch"), c.get("aux_wgrad"), c["sync"]["captured"] if c.get("sync") else None, c["final_loss"])' $1; }
for i in 1 2; do
for v in off on; do
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-diag --aux-wgrad $v > gpurun_out/r10s/r50_e_${v}_$i.json 2> gpurun_out/r10s/r50_e_${v}_$i.err; fatal $? r50e$v
show gpurun_out/r10s/r50_e_${v}_$i.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-diag --graph --aux-wgrad $v > gpurun_out/r10s/r50_g_${v}_$i.json 2> gpurun_out/r10s/r50_g_${v}_$i.err; fatal $? r50g$v
show gpurun_out/r10s/r50_g_${v}_$i.json
done; done
for v in off on; do
timeout -k 10 300 python bench.py --model alexnet --steps 20 --warmup 5 --no-diag --aux-wgrad $v > gpurun_out/r10s/alex_e_${v}.json 2> gpurun_out/r10s/alex_e_${v}.err; fatal $? alex$v
show gpurun_out/r10s/alex_e_${v}.json
done
for i in 1 2 3; do
for pf in "--prefetch off" "--prefetch on --prefetch-at head"; do
tag=$(echo $pf | tr -d ' -'); 
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-diag $pf > gpurun_out/r10s/mlp_${tag}_$i.json 2> gpurun_out/r10s/mlp_${tag}_$i.err; fatal $? mlp$tag
show gpurun_out/r10s/mlp_${tag}_$i.json
done; done
echo done
