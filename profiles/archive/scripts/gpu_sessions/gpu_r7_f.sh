#!/bin/bash
# Same-box ratio vs stock torch DDP + torch.optim (toy MLP SGD and Adam), interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7f; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["value"])' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7f/t.json 2>/dev/null; fatal $? t; echo "tdp sgd r$r $(ms gpurun_out/r7f/t.json)"
timeout -k 10 300 python bench.py --impl torch --no-diag > gpurun_out/r7f/s.json 2>/dev/null; fatal $? s; echo "torch sgd r$r $(ms gpurun_out/r7f/s.json)"
done
timeout -k 10 300 python bench.py --optim adam --no-diag > gpurun_out/r7f/ta.json 2>/dev/null; fatal $? ta; echo "tdp adam $(ms gpurun_out/r7f/ta.json)"
timeout -k 10 300 python bench.py --impl torch --optim adam --no-diag > gpurun_out/r7f/sa.json 2>/dev/null; fatal $? sa; echo "torch adam $(ms gpurun_out/r7f/sa.json)"
echo done
