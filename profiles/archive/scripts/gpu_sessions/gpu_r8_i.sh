#!/bin/bash
# Round 4 closing profiles: dp1 headline step kernel table + timeline on the final tree, and the
# one-GPU rehearsal of the multi-GPU step (TDP_FORCE_COLLECTIVE=1) with its comm-queue overlap.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8i; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8i/dp1 -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r8i/dp1.log 2>&1; fatal $? dp1
T=$(find gpurun_out/r8i/dp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r8i/dp1_kernels.md
python3 scripts/step_timeline.py $T ce_fwd 40 > gpurun_out/r8i/dp1_timeline.md
head -14 gpurun_out/r8i/dp1_kernels.md
TDP_FORCE_COLLECTIVE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r8i/reh -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r8i/reh.log 2>&1; fatal $? reh
T=$(find gpurun_out/r8i/reh -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r8i/reh_kernels.md
python3 scripts/overlap_report.py $T --by-queue --step-marker ce_fwd --last-steps 4 --title "bench.py rehearsal of the multi-GPU step (TDP_FORCE_COLLECTIVE=1), side = the comm queue" > gpurun_out/r8i/reh_overlap.md
head -14 gpurun_out/r8i/reh_kernels.md
head -6 gpurun_out/r8i/reh_overlap.md
echo done
