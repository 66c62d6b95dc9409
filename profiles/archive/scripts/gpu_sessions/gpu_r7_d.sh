#!/bin/bash
# Head logits in the fc2 reduce (1024-thread row workgroups) vs the separate head forward:
# targeted tests, interleaved A/B, step timeline.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7d; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7d/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r7d/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2 3; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7d/b.json 2>/dev/null; fatal $? b; echo "head-in-reduce r$r $(ms gpurun_out/r7d/b.json)"
TDP_HEAD_IN_REDUCE=0 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7d/b0.json 2>/dev/null; fatal $? b0; echo "separate head r$r $(ms gpurun_out/r7d/b0.json)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7d/d.json 2>gpurun_out/r7d/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r7d/d.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7d/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r7d/prof.log 2>&1; fatal $? prof
python3 scripts/step_timeline.py $(find gpurun_out/r7d/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7d/mlp_timeline.md
python3 scripts/step_kernels.py $(find gpurun_out/r7d/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7d/mlp_kernels.md
cat gpurun_out/r7d/mlp_timeline.md
echo done
