#!/bin/bash
# A/B: static wave priority for every other workgroup slot in the split-bf16 GEMM (TDP_GEMM_EMU_PRIO=1).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for e in 0 1; do
  TDP_GEMM_EMU_PRIO=$e timeout -k 10 300 python -u scripts/bench_gemm_emu.py > gpurun_out/r4l_gemm_prio$e.jsonl 2>&1; fatal $? "gemm $e"
  python3 -c 'import json,sys; [print(sys.argv[2], k, v["emu_us"]) for l in open(sys.argv[1]) if l.startswith("{") for k, v in json.loads(l).items()]' gpurun_out/r4l_gemm_prio$e.jsonl $e
done
for r in 1 2; do for e in 0 1; do for m in toy_mlp resnet50; do
  TDP_GEMM_EMU_PRIO=$e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r4l.json 2>/dev/null; fatal $? "bench $m $e"
  echo "$r prio=$e $m $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r4l.json)"
done; done; done
