#!/bin/bash
# A/B: 256-row tiles (FM=4) for 64-wide conv plans under split-bf16 products (TDP_GEMM_BM=256).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for e in 0 256; do
  TDP_GEMM_BM=$e timeout -k 10 300 python -u scripts/bench_conv.py alexnet 128 > gpurun_out/r4m_conv_alexnet_bm$e.jsonl 2>&1; fatal $? "conv alexnet $e"
  TDP_GEMM_BM=$e timeout -k 10 300 python -u scripts/bench_conv.py resnet50 128 > gpurun_out/r4m_conv_r50_bm$e.jsonl 2>&1; fatal $? "conv r50 $e"
  tail -1 gpurun_out/r4m_conv_alexnet_bm$e.jsonl; tail -1 gpurun_out/r4m_conv_r50_bm$e.jsonl
done
for r in 1 2; do for e in 0 256; do for m in alexnet resnet50; do
  TDP_GEMM_BM=$e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r4m.json 2>/dev/null; fatal $? "bench $m $e"
  echo "$r bm=$e $m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4m.json)"
done; done; done
