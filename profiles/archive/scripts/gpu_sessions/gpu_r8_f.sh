#!/bin/bash
# Round 4: why the one-process Accelerate step differs from the native DDP step (diagnostic).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r8f; export TMPDIR=/tmp
timeout -k 10 200 python scripts/diag_accel_hidden.py > gpurun_out/r8f/diag.jsonl 2> gpurun_out/r8f/diag.err; rc=$?
grep '^{' gpurun_out/r8f/diag.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    r = json.loads(l); print(r['vs'], r['epilogue_gemms'], [max(s.values()) for s in r['max_diff_per_step']])"
tail -3 gpurun_out/r8f/diag.err
exit $rc
