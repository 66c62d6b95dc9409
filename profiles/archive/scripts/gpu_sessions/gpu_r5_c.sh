#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/diag/relay_debug.py 2 > gpurun_out/r5c_debug.log 2>&1; rc=$?
grep -v "Gloo\|socket.cpp\|amdgpu.ids" gpurun_out/r5c_debug.log | tail -60
exit $rc
