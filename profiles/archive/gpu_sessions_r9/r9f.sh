#!/bin/bash
# ws kernel interference: full / math without operand loads / math-only without loads
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9f; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for v in full:0 noload:4 noload_math:6 stream:1 math:2; do
  IFS=: read name exp <<< "$v"
  TDP_WS_EXP=$exp TDP_WGRAD_WS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9f/$name -o kt -- python3 dev/micro/ws_probe.py 30 > gpurun_out/r9f/$name.log 2>&1; fatal $? $name
  T=$(find gpurun_out/r9f/$name -name '*kernel_trace.csv' | head -1)
  python3 -c "
import csv, statistics as st
rows=[r for r in csv.DictReader(open('$T')) if 'wgrad' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000 for r in rows]
print('$name', 'fc1 median', round(st.median(d[5:30]),1), 'fc2 median', round(st.median(d[35:60]),1))
"
done
echo done
