#!/bin/bash
# write-through (sc1) parameter stores in the wgrad + SGD epilogue (kOptWT, --sgd 152): numerics,
# then an interleaved A/B against the default (--sgd 24 = kOptLds | kOptNT) on one box
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11h; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py -x -q --timeout 120 --timeout-method thread -k "152 or sgd-24" > gpurun_out/r11h/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r11h/tests.log; [ $rc -eq 0 ] || exit 1
run() { tag=$1; shift; timeout -k 10 300 python -u scripts/run_with_variant.py "$@" -- bench.py --steps 200 --warmup 20 > gpurun_out/r11h/$tag.json 2> gpurun_out/r11h/$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r11h/$tag.json')); print('$tag', d['ms_per_step'])"; }
run nt1 --sgd 24 && run wt1 --sgd 152 && run nt2 --sgd 24 && run wt2 --sgd 152 && run nt3 --sgd 24 && run wt3 --sgd 152 && echo done
