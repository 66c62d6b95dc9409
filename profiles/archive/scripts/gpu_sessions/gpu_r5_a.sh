#!/bin/bash
# Round-3 first contact: GPU suite + driver-shaped bench on the round-2 tree.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r5a_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || exit $?
cat gpurun_out/r5a_bench.json
