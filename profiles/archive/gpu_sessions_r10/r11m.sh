#!/bin/bash
# Final validation of the round-6 tree (after the archive move and the last rebuild)
# Final validation of the round-6 tree (after the archive move and the last rebuild)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11m; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r11m/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r11m/gpu_suite.log; grep -E "FAILED|Error" gpurun_out/r11m/gpu_suite.log | head -5; fatal $rc suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r11m/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r11m/smoke.log; fatal $rc smoke
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r11m/d$i.json 2> gpurun_out/r11m/d$i.err; fatal $? bench$i
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], d["value"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r11m/d$i.json
done
timeout -k 10 400 python bench.py --syncbn --steps 20 --warmup 5 > gpurun_out/r11m/syncbn.json 2> gpurun_out/r11m/syncbn.err; fatal $? syncbn
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d[\"ms_per_step\"], d.get(\"diagnostics\"))" gpurun_out/r11m/syncbn.json
for m in resnet50 alexnet; do
timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r11m/$m.json 2> gpurun_out/r11m/$m.err; fatal $? $m
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(sys.argv[1], d["ms_per_step"], d["config"]["sync"]["captured"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1")})' gpurun_out/r11m/$m.json
done
echo done
