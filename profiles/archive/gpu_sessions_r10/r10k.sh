#!/bin/bash
# kOptPre A/B: the wgrad + SGD epilogue's first p / momentum batch touched into L2 under the K
# loop (opt variant 88) vs the default (24), dp1 captured step, interleaved; kernel traces of both.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10k; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2 3; do for v in 24 88; do
timeout -k 10 200 python scripts/rehearsal_probe.py --dp1 --steps 300 --opt-variant $v >> gpurun_out/r10k/ab.txt 2>> gpurun_out/r10k/ab.err; fatal $? ab$i$v
done; done
grep "ms/step" gpurun_out/r10k/ab.txt | cut -c1-60
for v in 24 88; do
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r10k/kt$v -o kt -- python3 scripts/rehearsal_probe.py --dp1 --steps 60 --opt-variant $v > gpurun_out/r10k/kt$v.log 2>&1; fatal $? kt$v
T=$(find gpurun_out/r10k/kt$v -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r10k/kernels_$v.md; head -5 gpurun_out/r10k/kernels_$v.md
done
timeout -k 10 300 python -u -m pytest tests/test_sync_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or epilogue or deterministic" > gpurun_out/r10k/tests.log 2>&1; tail -2 gpurun_out/r10k/tests.log
echo done
