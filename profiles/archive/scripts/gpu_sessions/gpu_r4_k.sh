#!/bin/bash
# Same-box A/B of the fused CE gradient (TDP_CE_FUSED_GRAD=0 off), toy MLP with and without SyncBN.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2; do for e in 0 1; do for extra in "" "--syncbn"; do
  TDP_CE_FUSED_GRAD=$e timeout -k 10 300 python bench.py $extra --no-diag > gpurun_out/r4k.json 2>/dev/null; fatal $? "bench $e $extra"
  echo "$r fused=$e $extra $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4k.json)"
done; done; done
