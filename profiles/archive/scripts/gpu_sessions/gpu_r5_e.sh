#!/bin/bash
# ReLU-gated input gradients + GEMM range tests; MLP bench and kernel profile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_emu_gpu.py tests/test_ddp_gpu.py tests/test_sync_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5e_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r5e_pytest.log; fatal $rc pytest
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-diag > gpurun_out/r5e_driver.json 2>/dev/null; fatal $? bench_driver
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r5e_default.json 2>/dev/null; fatal $? bench_default
for f in gpurun_out/r5e_driver.json gpurun_out/r5e_default.json; do echo "$f $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' $f)"; done
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5e_prof" -o mlp -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-diag > "$R/gpurun_out/r5e_prof.log" 2>&1; fatal $? prof
ls -R gpurun_out/r5e_prof | head
