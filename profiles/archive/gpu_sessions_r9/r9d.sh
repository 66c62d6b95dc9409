#!/bin/bash
# ws kernel anatomy: full / math only (stream skips HBM) / stream only (math skips its K loop) /
# old persistent kernel, fc1 and fc2 shapes, kernel trace per variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9d; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for v in full:0:1 math:2:1 stream:1:1 old:0:0; do
  IFS=: read name exp ws <<< "$v"
  TDP_WS_EXP=$exp TDP_WGRAD_WS=$ws timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r9d/$name -o kt -- python3 dev/micro/ws_probe.py 30 > gpurun_out/r9d/$name.log 2>&1; fatal $? $name
  S=$(find gpurun_out/r9d/$name -name '*kernel_stats.csv' | head -1)
  echo "== $name"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$S')):
    n=r['Name']
    if 'wgrad' in n or 'gemm_f32_fast' in n: print(n[:60], r['Calls'], round(float(r['AverageNs'])/1000,1), round(float(r['MinNs'])/1000,1), round(float(r['MaxNs'])/1000,1))
"
done
T=$(find gpurun_out/r9d/full -name '*kernel_trace.csv' | head -1)
python3 -c "
import csv
rows=[r for r in csv.DictReader(open('$T')) if 'wgrad' in r['Kernel_Name']]
print([round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000,1) for r in rows])
"
echo done
