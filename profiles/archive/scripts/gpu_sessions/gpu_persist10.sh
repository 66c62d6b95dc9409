#!/bin/bash
# Persistent optimizer-epilogue wgrad kernel (TDP_OPT_PERSIST) vs one-tile-per-workgroup launch.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/p10; mkdir -p $O; export TMPDIR=/tmp
B="python bench.py --steps 300 --warmup 30"
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 $B > $O/persist.json 2> $O/persist.err && \
TDP_OPT_PERSIST=0 timeout -k 10 120 $B > $O/flat.json 2> $O/flat.err && \
timeout -k 10 120 $B --optim adam > $O/persist_adam.json 2> $O/persist_adam.err && \
TDP_OPT_PERSIST=0 timeout -k 10 120 $B --optim adam > $O/flat_adam.json 2> $O/flat_adam.err && \
timeout -k 10 120 $B > $O/persist2.json 2> $O/persist2.err && \
TDP_OPT_PERSIST=0 timeout -k 10 120 $B > $O/flat2.json 2> $O/flat2.err
rc=$?
tail -3 $O/pytest.log
for f in $O/*.json; do echo "$f: $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["final_loss"])' 2>/dev/null)"; done
exit $rc
