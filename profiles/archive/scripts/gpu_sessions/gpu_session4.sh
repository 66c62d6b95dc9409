#!/bin/bash
# Re-validate HEAD on a fresh MI355X: GPU tests, smoke, MLP + ResNet-50 benches (native vs stock
# torch), then a 2-ranks-on-one-GPU RCCL probe (last: its failure only tells whether RCCL allows it).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_tdp.json 2> gpurun_out/bench_tdp.err && \
timeout -k 10 300 python bench.py --impl torch --steps 200 --warmup 30 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_r50_tdp.json 2> gpurun_out/bench_r50_tdp.err && \
timeout -k 10 300 python bench.py --model resnet50 --impl torch --steps 20 --warmup 5 > gpurun_out/bench_r50_torch.json 2> gpurun_out/bench_r50_torch.err && \
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_2on1.json 2> gpurun_out/bench_2on1.err
rc=$?
tail -3 gpurun_out/pytest_gpu.log
for f in gpurun_out/bench_*.json; do echo "$f: $(tail -1 $f)"; done
exit $rc
