#!/bin/bash
# PMC passes over representative conv GEMMs (one counter group per run).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc; cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 scripts/conv_pmc_probe.py > gpurun_out/pmc/p1.log 2>&1
fatal $? p1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 scripts/conv_pmc_probe.py > gpurun_out/pmc/p2.log 2>&1
fatal $? p2
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/kt -o kt -- python3 scripts/conv_pmc_probe.py > gpurun_out/pmc/kt.log 2>&1
fatal $? kt
