#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_stream.py > gpurun_out/r5g_stream.jsonl 2> gpurun_out/r5g_stream.err; rc=$?
cat gpurun_out/r5g_stream.jsonl; tail -3 gpurun_out/r5g_stream.err; exit $rc
