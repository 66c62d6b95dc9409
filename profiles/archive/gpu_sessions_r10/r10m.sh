#!/bin/bash
# A/B: SGD epilogue 24 (LDS + non-temporal) vs 88 (+ parameters stored with the default policy,
# so the next forward's weight stream can hit the Infinity Cache); epilogue variant tests; kernel
# table under 88.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10m; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
V=scripts/run_with_variant.py
# (variant tests passed on the first call: 24 passed)
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 300 python $V --sgd $v -- bench.py --steps 100 --warmup 20 --no-diag > gpurun_out/r10m/ab${i}_$v.json 2> gpurun_out/r10m/ab${i}_$v.err; fatal $? ab$i$v
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d["ms_per_step"])' gpurun_out/r10m/ab${i}_$v.json
done; done
for v in 24 88; do
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10m/k$v -o kt -- python3 $V --sgd $v -- bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r10m/k$v.log 2>&1; fatal $? k$v
T=$(find gpurun_out/r10m/k$v -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10m/k${v}_kernels.md; cat gpurun_out/r10m/k${v}_kernels.md
done
echo done
