#!/bin/bash
# Paired weight-gradient + optimizer launch: bitwise tests, optimizer-path GPU tests, A/B of
# bench.py with the pair on (default) / off (interleaved, 100-step windows), kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10o; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
V=scripts/run_with_variant.py
show() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"])' $1; }
timeout -k 10 600 python -u -m pytest tests/test_sync_gpu.py tests/test_ddp_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/r10o/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10o/tests.log; grep -E "FAILED|Error" gpurun_out/r10o/tests.log | head -5; fatal $rc tests
for i in 1 2 3; do for v in off on; do
F=""; [ $v = off ] && F="--no-pair-wgrad"
timeout -k 10 300 python $V $F -- bench.py --steps 100 --warmup 20 --no-diag > gpurun_out/r10o/ab${i}_$v.json 2> gpurun_out/r10o/ab${i}_$v.err; fatal $? ab$i$v; show gpurun_out/r10o/ab${i}_$v.json
done; done
for i in 1 2; do for v in off on; do
F=""; [ $v = off ] && F="--no-pair-wgrad"
timeout -k 10 300 python $V $F -- bench.py --optim adam --steps 100 --warmup 20 --no-diag > gpurun_out/r10o/adam${i}_$v.json 2> gpurun_out/r10o/adam${i}_$v.err; fatal $? adam$i$v; show gpurun_out/r10o/adam${i}_$v.json
done; done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10o/k -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10o/k.log 2>&1; fatal $? k
T=$(find gpurun_out/r10o/k -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10o/kernels.md; cat gpurun_out/r10o/kernels.md
echo done
