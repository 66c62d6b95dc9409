#!/bin/bash
# rebuilt extension (after the write-through revert): smoke, driver-shaped bench, SyncBN config
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11j; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r11j/smoke.log 2>&1 || exit 1; tail -1 gpurun_out/r11j/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r11j/d1.json 2> gpurun_out/r11j/d1.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --syncbn > gpurun_out/r11j/syncbn.json 2> gpurun_out/r11j/syncbn.err || exit 1
for f in d1 syncbn; do python -c "import json; d=json.load(open('gpurun_out/r11j/$f.json')); print('$f', d['ms_per_step'], d['value'], d['diagnostics'].get('rehearsal_over_dp1'))"; done
timeout -k 10 600 python -u -m pytest tests/test_sync_gpu.py tests/test_bench_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r11j/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r11j/tests.log; [ $rc -eq 0 ] && echo done
