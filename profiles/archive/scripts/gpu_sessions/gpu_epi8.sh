#!/bin/bash
# Optimizer-in-GEMM-epilogue (world size 1): GPU tests, bench default (fused auto = epilogue) vs
# the per-bucket / unfused paths, Adam, and a kernel-stats profile of the new default step.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/e8
export TMPDIR=/tmp
O=gpurun_out/e8
B="python bench.py --steps 200 --warmup 30"
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py tests/test_kernels_gpu.py tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 $B > $O/default.json 2> $O/default.err && \
TDP_OPT_EPILOGUE=0 timeout -k 10 120 $B > $O/bucket.json 2> $O/bucket.err && \
timeout -k 10 120 $B --fused-opt off > $O/unfused.json 2> $O/unfused.err && \
timeout -k 10 120 $B --optim adam > $O/adam.json 2> $O/adam.err && \
timeout -k 10 120 $B --optim adam > $O/adam2.json 2> $O/adam2.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 10 > $O/prof.log 2>&1
rc=$?
tail -3 $O/pytest.log
for f in $O/*.json; do echo "$f: $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["final_loss"])' 2>/dev/null)"; done
exit $rc
