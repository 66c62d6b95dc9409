#!/bin/bash
# HIP graph queue count 2 vs the runtime default: dp1 + rehearsal interleaved x3 on one box, then
# the captured peer-vehicle (real RCCL, W ranks on one GPU) tests under the 2-queue setting
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11i; export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > gpurun_out/r11i/$tag.json 2> gpurun_out/r11i/$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r11i/$tag.json')); g=d['diagnostics']; print('$tag', d['ms_per_step'], g.get('rehearsal_ms'), g.get('rehearsal_schedule_ms'), g.get('rehearsal_over_dp1'), g.get('rehearsal_schedule_over_dp1'))"; }
run d1 HIP_DUMMY=0 && run q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run d2 HIP_DUMMY=0 && run q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run d3 HIP_DUMMY=0 && run q3 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 600 python -u -m pytest tests/test_peer_gpu.py -x -v --timeout 200 --timeout-method thread -k "captured" > gpurun_out/r11i/peer_q2.log 2>&1; rc=$?; tail -3 gpurun_out/r11i/peer_q2.log; [ $rc -eq 0 ] && echo done
