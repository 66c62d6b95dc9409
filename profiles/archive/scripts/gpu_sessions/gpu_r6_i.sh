#!/bin/bash
# Planes path in the toy-MLP step: tests, driver-shaped and 100-step benches with planes on/off
# and priority on/off, then a kernel trace of the default step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6i; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_ddp_gpu.py tests/test_factor_gpu.py tests/test_sync_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6i/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r6i/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
for v in "planes1 TDP_PLANES=1" "planes0 TDP_PLANES=0" "prio0 TDP_PLANES_PRIO=0" "c3 TDP_PLANES_CFG=3,0"; do
  set -- $v; tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-diag > gpurun_out/r6i/$tag.json 2>/dev/null; fatal $? $tag
  echo "$tag r$r 100-step $(ms gpurun_out/r6i/$tag.json)"
done; done
for v in "planes1 TDP_PLANES=1" "planes0 TDP_PLANES=0"; do
  set -- $v; tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r6i/d_$tag.json 2>/dev/null; fatal $? d_$tag
  echo "$tag driver-shaped $(ms gpurun_out/r6i/d_$tag.json)"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6i/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6i/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6i/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6i/mlp_kernels.md
cat gpurun_out/r6i/mlp_kernels.md
echo done
