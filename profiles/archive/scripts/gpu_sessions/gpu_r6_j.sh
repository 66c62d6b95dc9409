#!/bin/bash
# dp1 toy-MLP: eager vs captured step, planes on/off, 2 vs 3 stages; interleaved rounds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6j; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"]["impl"])' $1; }
for r in 1 2 3; do
for v in "eager TDP_PLANES=1 --" "graph TDP_PLANES=1 -- --graph" "eager_c3 TDP_PLANES_CFG=3,0 --" "graph_c3 TDP_PLANES_CFG=3,0 -- --graph" "eager_off TDP_PLANES=0 --" "graph_off TDP_PLANES=0 -- --graph"; do
  set -- $v; tag=$1; shift; envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-diag "$@" > gpurun_out/r6j/$tag.json 2>gpurun_out/r6j/$tag.err; fatal $? $tag
  echo "$tag r$r $(ms gpurun_out/r6j/$tag.json)"
done; done
echo done
