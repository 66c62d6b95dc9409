#!/bin/bash
# Split-K / tile sweep of the tensor-sharded step's GEMMs at W = 8.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9q; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_tp_gemms.py > gpurun_out/r9q/sweep.jsonl 2> gpurun_out/r9q/sweep.err; rc=$?
cat gpurun_out/r9q/sweep.jsonl; tail -3 gpurun_out/r9q/sweep.err; exit $rc
