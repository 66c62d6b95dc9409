#!/bin/bash
# Same-box CNN ratio vs stock torch DDP + torch.optim (ResNet-50, AlexNet; batch 128, fp32).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7g; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' $1; }
for m in resnet50 alexnet; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --no-diag > gpurun_out/r7g/t_$m.json 2>/dev/null; fatal $? t_$m; echo "tdp $m $(ms gpurun_out/r7g/t_$m.json)"
timeout -k 10 300 python bench.py --model $m --impl torch --steps 20 --warmup 5 --no-diag > gpurun_out/r7g/s_$m.json 2>/dev/null; fatal $? s_$m; echo "torch $m $(ms gpurun_out/r7g/s_$m.json)"
done
echo done
