#!/bin/bash
# Rehearsal of the W > 1 DDP schedule on the current tree: kernel tables and timelines, with and
# without the one-rank collectives, next to dp1.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11d; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for v in "reh:" "sched:--skip-collectives" "dp1:--dp1"; do
n=${v%%:*}; f=${v#*:}
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r11d/$n -o kt -- python3 scripts/rehearsal_probe.py --steps 100 $f > gpurun_out/r11d/$n.log 2>&1; fatal $? $n
tail -1 gpurun_out/r11d/$n.log
T=$(find gpurun_out/r11d/$n -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r11d/${n}_kernels.md; cat gpurun_out/r11d/${n}_kernels.md
python3 scripts/step_timeline.py $T ce_fwd > gpurun_out/r11d/${n}_timeline.md 2>&1 || true
done
echo done
