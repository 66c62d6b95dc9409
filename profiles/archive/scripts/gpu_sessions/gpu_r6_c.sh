#!/bin/bash
# PMC passes + kernel stats of the planes GEMM (fc1 forward shape) vs the fast GEMM.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6c; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c/kt -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6c/kt.log 2>&1
fatal $? kt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/r6c/p1 -o p1 -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6c/p1.log 2>&1
fatal $? p1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES --output-format csv -d gpurun_out/r6c/p2 -o p2 -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6c/p2.log 2>&1
fatal $? p2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d gpurun_out/r6c/p3 -o p3 -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6c/p3.log 2>&1
fatal $? p3
find gpurun_out/r6c -name '*.csv' | sort
echo ok
