#!/bin/bash
# Diagnostic: tensor-sharded gradient accumulation variants against the torch oracle (W = 2).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9an; export TMPDIR=/tmp
timeout -k 10 200 python -u -c "
import functools, sys
sys.path.insert(0, 'tests')
import tp_workers as TW
from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn
spawn(TW.accumulation_diag, 2, args=('gpurun_out/r9an',), grace=5.0)
" > gpurun_out/r9an/diag.log 2>&1; rc=$?; grep -v "Gloo\|socket" gpurun_out/r9an/diag.log | tail -40; exit $rc
