#!/bin/bash
# AlexNet convolution plan sweep (every pass, every (FN, split-K) candidate): is conv2's
# 70 TF/s a plan choice?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10g; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -u scripts/tune_conv_plans.py gpurun_out/r10g/alex_plans.json alexnet:128 > gpurun_out/r10g/alex.jsonl 2> gpurun_out/r10g/alex.err; rc=$?; cat gpurun_out/r10g/alex.jsonl; tail -5 gpurun_out/r10g/alex.err; fatal $rc tune
echo done
