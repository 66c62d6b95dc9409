#!/bin/bash
# BN local merge + BN planes: GPU suite, SyncBN / default / ResNet-50 benches, SyncBN kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6s; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6s/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6s/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --syncbn --no-diag > gpurun_out/r6s/sbn.json 2>/dev/null; fatal $? sbn; echo "syncbn r$r $(ms gpurun_out/r6s/sbn.json)"
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6s/b.json 2>/dev/null; fatal $? b; echo "default r$r $(ms gpurun_out/r6s/b.json)"
done
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-diag > gpurun_out/r6s/r50.json 2>/dev/null; fatal $? r50; echo "resnet50 $(ms gpurun_out/r6s/r50.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6s/sbnprof -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r6s/sbnprof.log 2>&1; fatal $? sbnprof
python3 scripts/step_kernels.py $(find gpurun_out/r6s/sbnprof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6s/syncbn_kernels.md
cat gpurun_out/r6s/syncbn_kernels.md
echo done
