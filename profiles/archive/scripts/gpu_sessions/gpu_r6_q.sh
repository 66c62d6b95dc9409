#!/bin/bash
# Pipelined 3-stage planes GEMM: compute-only (TDP_PLANES_EXP=6: no DMA) vs full, kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6q; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for e in 0 6 2 4; do
TDP_PLANES_EXP=$e timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6q/e$e -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6q/e$e.log 2>&1; fatal $? e$e
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/r6q/p1 -o p1 -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6q/p1.log 2>&1; fatal $? p1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES --output-format csv -d gpurun_out/r6q/p2 -o p2 -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6q/p2.log 2>&1; fatal $? p2

ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"]["impl"])' $1; }
timeout -k 10 300 python bench.py --syncbn --no-diag > gpurun_out/r6q/sbn.json 2>/dev/null; fatal $? sbn; echo "syncbn $(ms gpurun_out/r6q/sbn.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6q/sbnprof -o kt -- python3 bench.py --syncbn --steps 60 --warmup 10 --no-diag > gpurun_out/r6q/sbnprof.log 2>&1; fatal $? sbnprof
python3 scripts/step_kernels.py $(find gpurun_out/r6q/sbnprof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6q/syncbn_kernels.md
cat gpurun_out/r6q/syncbn_kernels.md
echo ok
