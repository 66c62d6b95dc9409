#!/bin/bash
# SyncBatchNorm halves of the whole-column BN kernels (measured with them opt-in: --sync1d then): kernel tests, the peer-vehicle SyncBN /
# DDP tests; peer-vehicle SyncBN bench at W = 2 / 4, split kernels vs whole-column (torchrun,
# N ranks on ONE GPU: plumbing + kernel counts, not a multi-GPU number).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11b; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_peer_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r11b/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r11b/tests.log; grep -E "FAILED|Error" gpurun_out/r11b/tests.log | head; fatal $rc tests
export TDP_GPU_PEER=1 HSA_ENABLE_IPC_MODE_LEGACY=0
for W in 2 4; do
for i in 1 2; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29611 scripts/run_with_variant.py --no-sync1d -- bench.py --gpus $W --syncbn --steps 30 --warmup 5 --no-diag > gpurun_out/r11b/w${W}_split_$i.json 2> gpurun_out/r11b/w${W}_split_$i.err; fatal $? split$W
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29612 scripts/run_with_variant.py -- bench.py --gpus $W --syncbn --steps 30 --warmup 5 --no-diag > gpurun_out/r11b/w${W}_col_$i.json 2> gpurun_out/r11b/w${W}_col_$i.err; fatal $? col$W
python3 -c 'import json,sys; [print(f, d["ms_per_step"], d["config"]["parallelism"], d["config"]["rung"], d["config"]["sync"]["replicas_identical"], d["config"]["final_loss"]) for f in sys.argv[1:] for d in [json.loads([l for l in open(f) if l.strip().startswith("{")][-1])]]' gpurun_out/r11b/w${W}_split_$i.json gpurun_out/r11b/w${W}_col_$i.json
done; done
echo done
