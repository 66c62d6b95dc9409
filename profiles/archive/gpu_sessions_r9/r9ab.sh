#!/bin/bash
# PMC: MFMA busy / VALU and MFMA instruction counts of the two split-bf16 GEMM kernels at 4096^3.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ab; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r9ab/p1 -o pmc -- python3 dev/micro/emu8_pmc_probe.py > gpurun_out/r9ab/p1.log 2>&1; fatal $? p1
F=$(find gpurun_out/r9ab/p1 -name '*counter_collection.csv' | head -1)
python3 - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in d.items()})
PY
echo done
