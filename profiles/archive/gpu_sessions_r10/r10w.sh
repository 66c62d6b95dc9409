#!/bin/bash
# First bench on a fresh box: does a longer device warm-up remove the first-run penalty?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10w; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
n=0
for w in 2000 200 2000 200 1000; do
n=$((n+1))
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag --device-warmup-ms $w > gpurun_out/r10w/r${n}_w$w.json 2> gpurun_out/r10w/r${n}_w$w.err; fatal $? r$n
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"])' gpurun_out/r10w/r${n}_w$w.json
done
echo done
