#!/bin/bash
# Tile-width A/B on N=128 convs; MLP cvec A/B; captured multi-GPU-schedule rehearsal kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python scripts/ab_fn.py > gpurun_out/ab_fn.jsonl 2> gpurun_out/ab_fn.err
fatal $? abfn
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-diag > gpurun_out/r2i_mlp_on$i.json 2>/dev/null; fatal $? mlpon
  TDP_GEMM_NO_CVEC=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-diag > gpurun_out/r2i_mlp_off$i.json 2>/dev/null; fatal $? mlpoff
done
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/r2i_mlp_*.json
TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_overlap -o ov -- python3 bench.py --graph --steps 20 --warmup 5 --no-diag > gpurun_out/prof_overlap.log 2>&1
fatal $? overlap
tail -1 gpurun_out/prof_overlap.log
