#!/bin/bash
# BN affine update with its operands prefetched: tests; SyncBN config A/B (split kernels / one
# launch without the in-place update / with it), interleaved; kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10z; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_gemm_planes_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r10z/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r10z/tests.log; grep -E "FAILED|Error" gpurun_out/r10z/tests.log | head; fatal $rc tests
for i in 1 2 3; do
timeout -k 10 300 python scripts/run_with_variant.py --no-local1d -- bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10z/split_$i.json 2> gpurun_out/r10z/split_$i.err; fatal $? split
timeout -k 10 300 python scripts/run_with_variant.py --no-bn-update -- bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10z/noupd_$i.json 2> gpurun_out/r10z/noupd_$i.err; fatal $? noupd
timeout -k 10 300 python bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10z/upd_$i.json 2> gpurun_out/r10z/upd_$i.err; fatal $? upd
python3 -c 'import json,sys; [print(f, json.load(open(f))["ms_per_step"], json.load(open(f))["config"]["final_loss"]) for f in sys.argv[1:]]' gpurun_out/r10z/split_$i.json gpurun_out/r10z/noupd_$i.json gpurun_out/r10z/upd_$i.json
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10z/sbn -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r10z/sbn.log 2>&1; fatal $? sbn
T=$(find gpurun_out/r10z/sbn -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10z/syncbn_kernels.md; cat gpurun_out/r10z/syncbn_kernels.md
echo done
