#!/bin/bash
# Steps per replay: driver-shaped dp1 bench at --graph-steps 4 / 5 / 10 / 20, interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10v; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2 3; do
for g in 4 5 10 20; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag --graph-steps $g > gpurun_out/r10v/g${g}_$i.json 2> gpurun_out/r10v/g${g}_$i.err; fatal $? g$g
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["graph_steps"], d["config"]["final_loss"])' gpurun_out/r10v/g${g}_$i.json
done; done
for i in 1 2; do
for g in 4 10; do
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-diag --graph-steps $g > gpurun_out/r10v/l${g}_$i.json 2> gpurun_out/r10v/l${g}_$i.err; fatal $? l$g
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"], d["config"]["graph_steps"], d["config"]["final_loss"])' gpurun_out/r10v/l${g}_$i.json
done; done
echo done
