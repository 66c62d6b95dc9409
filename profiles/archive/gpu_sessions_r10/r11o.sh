#!/bin/bash
# final-tree kernel tables: every BASELINE config at dp1 (bench.py --no-diag, so the trace's last
# steps are timed steps), summarised per training step (marker: the cross-entropy forward)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r11o; export TMPDIR=/tmp
for v in "mlp:--steps 100 --warmup 10" "adam:--steps 100 --warmup 10 --optim adam" "syncbn:--steps 100 --warmup 10 --syncbn" "resnet50:--steps 12 --warmup 3 --model resnet50" "alexnet:--steps 30 --warmup 5 --model alexnet"; do
n=${v%%:*}; f=${v#*:}
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r11o/$n -o kt -- python3 bench.py --no-diag $f > gpurun_out/r11o/$n.json 2> gpurun_out/r11o/$n.err || { echo "$n failed"; exit 1; }
T=$(find gpurun_out/r11o/$n -name '*kernel_trace.csv' | head -1)
last=40; case $n in resnet50) last=8;; alexnet) last=20;; esac
python3 scripts/step_kernels.py $T ce_fwd $last > gpurun_out/r11o/${n}_kernels.md && head -1 gpurun_out/r11o/${n}_kernels.md | cut -c1-250
rm -f $T
done
echo done
