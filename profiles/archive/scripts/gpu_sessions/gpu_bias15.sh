#!/bin/bash
# relu/bias-grad kernel rework: kernel tests, AlexNet / MLP benches, AlexNet kernel stats.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/b15; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_cnn_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/mlp.json 2> $O/mlp.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 > $O/alex.json 2> $O/alex.err && \
timeout -k 10 200 python bench.py --model alexnet --steps 50 --warmup 10 --impl torch > $O/alex_torch.json 2> $O/alex_torch.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_alex -o run -- python3 bench.py --model alexnet --steps 20 --warmup 5 > $O/prof_alex.log 2>&1
rc=$?
tail -3 $O/pytest.log
for f in $O/*.json; do echo "$f: $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["final_loss"])' 2>/dev/null)"; done
exit $rc
