#!/bin/bash
# Round 4: same-box stock comparisons for the BASELINE.md table at 1 GPU (the multi-GPU rows are
# the driver's): toy MLP + SyncBatchNorm, toy MLP via Accelerator.prepare, Adam, ResNet-50,
# AlexNet -- tdp and stock torch DDP + torch.optim interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8d; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"))' $1; }
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py --no-diag "$@" > gpurun_out/r8d/$n.json 2> gpurun_out/r8d/$n.err; fatal $? $n
  echo "$n $(ms gpurun_out/r8d/$n.json)"
}
# SGD epilogue: default (24 = LDS + non-temporal) vs 28 (+ one batch per tile), interleaved
timeout -k 10 200 python -u -m pytest tests/test_sync_gpu.py -x -q --timeout 120 --timeout-method thread -k "epilogue_variants and 28" > gpurun_out/r8d/variant28_test.log 2>&1; fatal $? variant28_test; tail -1 gpurun_out/r8d/variant28_test.log
timeout -k 10 240 python scripts/diag_adam_capture.py --runs 6 > gpurun_out/r8d/diag_adam_capture.jsonl 2>gpurun_out/r8d/diag_adam_capture.err; fatal $? diag_adam
python3 -c "import json; [print(r['seed'], r['fused'], r['loss_max_diff'], {k: (v['max'], v['n_over_1e-5']) for k, v in r['params'].items() if v['max'] > 0}) for r in map(json.loads, open('gpurun_out/r8d/diag_adam_capture.jsonl'))]"
for r in 1 2 3; do
for v in 24 28; do
timeout -k 10 300 python scripts/run_with_variant.py --sgd $v -- bench.py --no-diag > gpurun_out/r8d/epi_v${v}_r$r.json 2>gpurun_out/r8d/epi_v${v}_r$r.err; fatal $? epi_$v; echo "epilogue variant $v r$r $(ms gpurun_out/r8d/epi_v${v}_r$r.json)"
done; done
for r in 1 2; do
for v in 24 28; do
timeout -k 10 300 python scripts/run_with_variant.py --adam $v -- bench.py --no-diag --optim adam > gpurun_out/r8d/adam_v${v}_r$r.json 2>gpurun_out/r8d/adam_v${v}_r$r.err; fatal $? adam_$v; echo "adam epilogue variant $v r$r $(ms gpurun_out/r8d/adam_v${v}_r$r.json)"
done; done
run mlp_syncbn_tdp 300 --syncbn
run mlp_syncbn_torch 300 --syncbn --impl torch
run mlp_accel_tdp 300 --api accelerate
run mlp_accel_torch 300 --api accelerate --impl torch
run mlp_adam_tdp 300 --optim adam
run mlp_adam_torch 300 --optim adam --impl torch
run r50_tdp 400 --model resnet50 --steps 20 --warmup 5
run r50_torch 400 --model resnet50 --steps 20 --warmup 5 --impl torch
run alexnet_tdp 300 --model alexnet --steps 20 --warmup 5
run alexnet_torch 300 --model alexnet --steps 20 --warmup 5 --impl torch
echo done
