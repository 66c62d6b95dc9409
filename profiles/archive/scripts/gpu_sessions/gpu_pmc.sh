#!/bin/bash
# PMC counters for the GEMM microbenchmark (own run: --pmc with --kernel-trace only).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
PMC=${PMC:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"}
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d gpurun_out/pmc1 -o run -- python3 scripts/bench_gemm.py > gpurun_out/pmc1.log 2>&1
rc=$?
PMC2=${PMC2:-"SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"}
[ $rc -eq 0 ] && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC2 --output-format csv -d gpurun_out/pmc2 -o run -- python3 scripts/bench_gemm.py > gpurun_out/pmc2.log 2>&1
rc=$?
exit $rc
