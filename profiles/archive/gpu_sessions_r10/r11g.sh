#!/bin/bash
# HIP graph-runtime settings against the dp1 step and its multi-GPU rehearsal (diagnostics)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11g; export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > gpurun_out/r11g/$tag.json 2> gpurun_out/r11g/$tag.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r11g/$tag.json')); g=d['diagnostics']; print('$tag', d['ms_per_step'], g.get('rehearsal_ms'), g.get('rehearsal_schedule_ms'), g.get('rehearsal_over_dp1'), g.get('rehearsal_schedule_over_dp1'))"; }
run base HIP_DUMMY=0 && run q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && run nopc DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run base2 HIP_DUMMY=0 && echo done
