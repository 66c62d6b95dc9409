#!/bin/bash
# Round 4 first session: DDP GPU tests (capture bookkeeping), fork form A/B on the one-GPU
# rehearsal of the multi-GPU step (defer / marker / inline), rehearsal kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8a; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_factor_gpu.py tests/test_sync_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r8a/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r8a/pytest.log
for i in 1 2 3; do timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py -q -k test_captured_adam_with_lr_change --timeout 120 --timeout-method thread > gpurun_out/r8a/adam_$i.log 2>&1; echo "adam rerun $i rc=$?"; grep -E "Greatest|passed|failed" gpurun_out/r8a/adam_$i.log; done
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d["config"]["sync"]["captured"])' $1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8a/d.json 2>gpurun_out/r8a/d.err; fatal $? d; echo "driver-shaped $(ms gpurun_out/r8a/d.json)"
for r in 1 2; do
for f in defer marker inline; do
TDP_GRAPH_FORK=$f TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r8a/reh_$f.json 2>gpurun_out/r8a/reh_$f.err; fatal $? reh_$f; echo "rehearsal $f r$r $(ms gpurun_out/r8a/reh_$f.json)"
done
done
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8a/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r8a/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r8a/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r8a/rehearsal_kernels.md
python3 scripts/step_timeline.py $(find gpurun_out/r8a/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r8a/rehearsal_timeline.md
cat gpurun_out/r8a/rehearsal_kernels.md
echo done
