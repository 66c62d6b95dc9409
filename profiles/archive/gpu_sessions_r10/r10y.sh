#!/bin/bash
# BN affine parameters updated inside the one-launch BN backward (world size 1, fused optimizer):
# epilogue / DDP / BN tests, SyncBN-config A/B and kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10y; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_sync_gpu.py tests/test_gemm_planes_gpu.py tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r10y/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r10y/tests.log; grep -E "FAILED|Error" gpurun_out/r10y/tests.log | head; fatal $rc tests
for i in 1 2; do
timeout -k 10 300 python scripts/run_with_variant.py --no-local1d -- bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10y/sbn_off_$i.json 2> gpurun_out/r10y/sbn_off_$i.err; fatal $? sbnoff
timeout -k 10 300 python bench.py --syncbn --steps 100 --warmup 20 --no-diag > gpurun_out/r10y/sbn_on_$i.json 2> gpurun_out/r10y/sbn_on_$i.err; fatal $? sbnon
timeout -k 10 300 python bench.py --syncbn --optim adam --steps 100 --warmup 20 --no-diag > gpurun_out/r10y/sbn_adam_$i.json 2> gpurun_out/r10y/sbn_adam_$i.err; fatal $? sbnadam
python3 -c 'import json,sys; [print(f, json.load(open(f))["ms_per_step"], json.load(open(f))["config"]["final_loss"]) for f in sys.argv[1:]]' gpurun_out/r10y/sbn_off_$i.json gpurun_out/r10y/sbn_on_$i.json gpurun_out/r10y/sbn_adam_$i.json
done
timeout -k 10 300 python bench.py --syncbn --steps 20 --warmup 5 > gpurun_out/r10y/sbn_diag.json 2> gpurun_out/r10y/sbn_diag.err; fatal $? sbndiag
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["diagnostics"])' gpurun_out/r10y/sbn_diag.json
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10y/sbn -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r10y/sbn.log 2>&1; fatal $? sbn
T=$(find gpurun_out/r10y/sbn -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10y/syncbn_kernels.md; cat gpurun_out/r10y/syncbn_kernels.md
echo done
