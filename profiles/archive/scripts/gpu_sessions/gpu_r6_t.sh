#!/bin/bash
# Single-split BatchNorm1d moments for small tensors: BN tests, SyncBN bench + kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6t; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_kernels_gpu.py tests/test_sync_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6t/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r6t/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --syncbn --no-diag > gpurun_out/r6t/sbn.json 2>/dev/null; fatal $? sbn; echo "syncbn r$r $(ms gpurun_out/r6t/sbn.json)"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6t/sbnprof -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r6t/sbnprof.log 2>&1; fatal $? sbnprof
python3 scripts/step_kernels.py $(find gpurun_out/r6t/sbnprof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6t/syncbn_kernels.md
head -22 gpurun_out/r6t/syncbn_kernels.md
echo done
