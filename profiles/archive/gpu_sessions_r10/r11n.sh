#!/bin/bash
# where the AccumulateGrad stream-mismatch warning comes from at W > 1 (peer vehicle, W = 2):
# the warning raised as an error shows the phase that first runs backward on another stream
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11n; export TMPDIR=/tmp
TDP_GPU_PEER=1 PYTHONWARNINGS="error::UserWarning:torch.autograd.graph" timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r11n/mlp2.json 2> gpurun_out/r11n/mlp2.err; echo "rc=$?"
grep -n -B2 -A30 "Traceback" gpurun_out/r11n/mlp2.err | head -80
echo done
