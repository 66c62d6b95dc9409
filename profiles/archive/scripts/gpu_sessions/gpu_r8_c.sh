#!/bin/bash
# Round 4: full GPU suite on the current tree, smoke, headline benches (driver-shaped + default),
# one-GPU rehearsal, entry-point (scripts/train_ddp.py) rocprofv3 trace with the bucket
# collectives forced at W=1 + overlap report, stock torch comparison for bench_baseline.json.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8c; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=15
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r8c/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r8c/pytest.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r8c/smoke.log 2>&1; fatal $? smoke; tail -1 gpurun_out/r8c/smoke.log
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"), d.get("diagnostics",{}).get("rehearsal_ms"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r8c/d$r.json 2>gpurun_out/r8c/d$r.err; fatal $? d; echo "driver-shaped r$r $(ms gpurun_out/r8c/d$r.json)"
timeout -k 10 300 python bench.py --impl torch --steps 20 --warmup 5 > gpurun_out/r8c/t$r.json 2>gpurun_out/r8c/t$r.err; fatal $? t; echo "stock torch driver-shaped r$r $(ms gpurun_out/r8c/t$r.json)"
done
timeout -k 10 300 python bench.py > gpurun_out/r8c/b.json 2>/dev/null; fatal $? b; echo "default 100 steps $(ms gpurun_out/r8c/b.json)"
timeout -k 10 300 python bench.py --impl torch > gpurun_out/r8c/bt.json 2>/dev/null; fatal $? bt; echo "stock default 100 steps $(ms gpurun_out/r8c/bt.json)"
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8c/prof_ddp -o kt -- python3 scripts/train_ddp.py --settings_file scripts/profile_train_ddp.yaml > gpurun_out/r8c/prof_ddp.log 2>&1; fatal $? prof_ddp
tail -2 gpurun_out/r8c/prof_ddp.log
T=$(find gpurun_out/r8c/prof_ddp -name '*kernel_trace.csv' | head -1)
python3 scripts/overlap_report.py $T --by-queue --step-marker gather --last-steps 4 --title "scripts/train_ddp.py captured step, collectives forced at W=1" > gpurun_out/r8c/train_ddp_overlap.md
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r8c/train_ddp_kernels.md
head -12 gpurun_out/r8c/train_ddp_overlap.md
rm -f $T.bak
echo done
