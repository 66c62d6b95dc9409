#!/bin/bash
# W = 8 plumbing of the tensor-sharded step on ONE GPU (peer vehicle, 8 ranks): captured parity
# at W = 8, and bench --gpus 8 --parallel tensor at the full toy-MLP dims (node batch 1024 rows:
# the cursor gather at 1024 rows, G-step graphs, chunked variant). Not a performance number.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9u; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=60
timeout -k 10 300 python -u -c "
import functools, sys
sys.path.insert(0, 'tests')
import tp_workers as TW
from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn
spawn(functools.partial(TW.captured_parity, chunks=1), 8, args=('/tmp',), grace=5.0)
spawn(functools.partial(TW.captured_parity, chunks=2), 8, args=('/tmp',), grace=5.0)
print('w8 parity ok')
" > gpurun_out/r9u/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r9u/parity.log; fatal $rc parity
TDP_GPU_PEER=1 timeout -k 10 500 python bench.py --gpus 8 --steps 8 --warmup 3 --parallel tensor --select-steps 4 > gpurun_out/r9u/peer8.json 2> gpurun_out/r9u/peer8.err; rc=$?; tail -3 gpurun_out/r9u/peer8.err; fatal $rc peer8
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(d["ms_per_step"], c["rung"], c["selection"], c["graph_steps"], c["sync"], c["final_loss"])' gpurun_out/r9u/peer8.json
echo done
