#!/bin/bash
# Round 4: head_bwd with 16-column workgroups on the in-place (fused) path -- tests + profile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8j; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_sync_gpu.py tests/test_accelerate_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8j/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r8j/pytest.log; fatal $rc pytest
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8j/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r8j/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r8j/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r8j/dp1_kernels.md
head -12 gpurun_out/r8j/dp1_kernels.md
for r in 1 2; do timeout -k 10 300 python bench.py --no-diag > gpurun_out/r8j/b$r.json 2>/dev/null; fatal $? b; python3 -c 'import json; d=json.load(open("gpurun_out/r8j/b'$r'.json")); print("bench", d["ms_per_step"], d["config"]["final_loss"])'; done
echo done
