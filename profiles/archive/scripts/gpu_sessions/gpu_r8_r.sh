#!/bin/bash
# Round 4: kernel traces of the one-GPU rehearsal of the multi-GPU step (TDP_FORCE_COLLECTIVE=1)
# with and without the early g gather: order of the comm-queue gathers against the parameter
# all-gather, and the overlap report.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8r; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for v in early late; do
A=""; [ $v = late ] && A="--no-early-g"
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8r/$v -o kt -- python3 scripts/run_with_variant.py $A -- bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r8r/$v.log 2>&1; fatal $? $v
T=$(find gpurun_out/r8r/$v -name '*kernel_trace.csv' | head -1)
python3 scripts/step_timeline.py $T ce_fwd 40 > gpurun_out/r8r/${v}_timeline.md
python3 scripts/overlap_report.py $T --by-queue --step-marker ce_fwd --last-steps 4 --title "rehearsal ($v g gather), side = the comm queue" > gpurun_out/r8r/${v}_overlap.md
head -8 gpurun_out/r8r/${v}_overlap.md
tail -1 gpurun_out/r8r/$v.log
done
echo done
