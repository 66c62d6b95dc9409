#!/bin/bash
# A/B on one box: skinny-M GEMM tile width (FN=2 default under split-bf16 vs TDP_GEMM_SKINNY_FN1=1).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for r in 1 2; do for e in TDP_GEMM_SKINNY_FN1=1 TDP_NONE=1; do for o in sgd adam; do
  env $e timeout -k 10 300 python bench.py --optim $o --no-diag > gpurun_out/r4h_${o}_$e_$r.json 2>/dev/null; fatal $? "bench $o $e"
  echo "$r $e $o $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4h_${o}_$e_$r.json)"
done; done; done
