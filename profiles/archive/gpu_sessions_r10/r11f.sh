#!/bin/bash
# dp1 step and its multi-GPU rehearsal: captured graphs dumped as DOT (node kinds, branches)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11f; export TMPDIR=/tmp
DUMP_DIR=gpurun_out/r11f/graphs timeout -k 10 400 python -u dev/gpu/graph_dump.py -- --steps 20 --warmup 5 > gpurun_out/r11f/d1.json 2> gpurun_out/r11f/d1.err && tail -3 gpurun_out/r11f/d1.err && ls -la gpurun_out/r11f/graphs && echo done
