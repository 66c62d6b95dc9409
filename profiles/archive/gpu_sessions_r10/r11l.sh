#!/bin/bash
# kOptWT (a workgroup's LAST tile of the persistent wgrad + SGD epilogue stores write-through,
# --sgd 152) vs the default (--sgd 24): numerics, interleaved A/B x3, dp1 kernel timelines of both
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11l; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py -x -q --timeout 120 --timeout-method thread -k "152 or sgd-24" > gpurun_out/r11l/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r11l/tests.log; [ $rc -eq 0 ] || exit 1
run() { tag=$1; shift; timeout -k 10 300 python -u scripts/run_with_variant.py "$@" -- bench.py --steps 200 --warmup 20 > gpurun_out/r11l/$tag.json 2> gpurun_out/r11l/$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r11l/$tag.json')); print('$tag', d['ms_per_step'])"; }
run nt1 --sgd 24 && run wt1 --sgd 152 && run nt2 --sgd 24 && run wt2 --sgd 152 && run nt3 --sgd 24 && run wt3 --sgd 152 || exit 1
for v in "nt:24" "wt:152"; do n=${v%%:*}; o=${v#*:}
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r11l/$n -o kt -- python3 scripts/rehearsal_probe.py --steps 100 --dp1 --opt-variant $o > gpurun_out/r11l/$n.log 2>&1 || exit 1
T=$(find gpurun_out/r11l/$n -name '*kernel_trace.csv' | head -1)
python3 scripts/step_timeline.py $T ce_fwd > gpurun_out/r11l/${n}_timeline.md 2>&1 || true
tail -14 gpurun_out/r11l/${n}_timeline.md
done
echo done
