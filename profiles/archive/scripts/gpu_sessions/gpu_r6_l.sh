#!/bin/bash
# Cross-tile pipelined 3-stage planes GEMM: numerics, kernel times, step time.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6l; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6l/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r6l/pytest.log; fatal $rc pytest
for c in 3,0 2,0; do
TDP_PLANES_CFG=$c timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6l/kt$c -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6l/kt$c.log 2>&1; fatal $? kt$c
done
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' $1; }
for r in 1 2; do for c in 3,0 2,0; do
TDP_PLANES_CFG=$c timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6l/b.json 2>/dev/null; fatal $? bench; echo "cfg $c r$r $(ms gpurun_out/r6l/b.json)"
done; done
echo done
