#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ac; export TMPDIR=/tmp
timeout -k 10 400 python -u dev/micro/emu8_variants.py > gpurun_out/r9ac/variants.jsonl 2> gpurun_out/r9ac/variants.err; rc=$?; cat gpurun_out/r9ac/variants.jsonl; tail -2 gpurun_out/r9ac/variants.err; exit $rc
