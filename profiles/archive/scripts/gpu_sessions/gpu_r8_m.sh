#!/bin/bash
# Round 4: PMC counters of the dp1 headline step's kernels (eager step: one dispatch per kernel),
# one counter group per run, --kernel-trace only beside --pmc.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8m; cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
B="bench.py --eager --steps 8 --warmup 3 --no-diag --device-warmup-ms 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r8m/p1 -o p1 -- python3 $B > gpurun_out/r8m/p1.log 2>&1; fatal $? p1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r8m/p2 -o p2 -- python3 $B > gpurun_out/r8m/p2.log 2>&1; fatal $? p2
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r8m/p3 -o p3 -- python3 $B > gpurun_out/r8m/p3.log 2>&1; fatal $? p3
python3 scripts/pmc_summary.py "dp1 toy-MLP step kernels, PMC (eager step, 11 steps)" gpurun_out/r8m/p1 gpurun_out/r8m/p2 gpurun_out/r8m/p3 > gpurun_out/r8m/pmc.md
cat gpurun_out/r8m/pmc.md
echo done
