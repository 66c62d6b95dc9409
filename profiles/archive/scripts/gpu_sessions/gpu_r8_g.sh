#!/bin/bash
# Round 4: head_bwd read/update race fix (the fused head backward at world size 1 read W for dx
# in some workgroups while others updated W in place): determinism diagnostics, the affected
# tests, the headline bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8g; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"], d["config"].get("final_loss"))' $1; }
timeout -k 10 200 python scripts/diag_accel_hidden.py > gpurun_out/r8g/diag.jsonl 2> gpurun_out/r8g/diag.err; fatal $? diag
grep '^{' gpurun_out/r8g/diag.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    r = json.loads(l); print(r['vs'], r['epilogue_gemms'], [max(s.values()) for s in r['max_diff_per_step']])"
timeout -k 10 600 python -u -m pytest tests/test_accelerate_gpu.py tests/test_sync_gpu.py tests/test_ddp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8g/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r8g/pytest.log; fatal $rc pytest
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r8g/b$r.json 2>gpurun_out/r8g/b$r.err; fatal $? bench; echo "bench r$r $(ms gpurun_out/r8g/b$r.json)"
timeout -k 10 300 python bench.py --no-diag --api accelerate > gpurun_out/r8g/a$r.json 2>gpurun_out/r8g/a$r.err; fatal $? accel; echo "accelerate r$r $(ms gpurun_out/r8g/a$r.json)"
done
echo done
