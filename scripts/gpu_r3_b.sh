#!/bin/bash
# hipGraph replay: which hardware queue runs which node. The ResNet-50 rehearsal trace showed a
# bucket collective and the next backward GEMM serialised on one queue; compare runtime knobs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
R="$GRAFT_REPO_ROOT"
run() {  # name, env assignments...
  name=$1; shift
  (cd /tmp && env "$@" TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r3b_$name" -o t -- python3 "$R/bench.py" --model resnet50 --graph --steps 4 --warmup 3 --no-diag > "$R/gpurun_out/r3b_$name.log" 2>&1)
  fatal $? $name
  python3 scripts/overlap_report.py gpurun_out/r3b_$name/t_kernel_trace.csv --step-marker gather_batch --last-steps 3 --title $name | sed -n 3,6p
}
run base X=1
run hwq8 GPU_MAX_HW_QUEUES=8
run gq2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
run gq8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8
for e in X=1 GPU_MAX_HW_QUEUES=8 DEBUG_HIP_FORCE_GRAPH_QUEUES=2; do
  env $e timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/r3b_bench_$e.json 2>/dev/null; fatal $? bench_$e
  echo "$e $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["diagnostics"])' gpurun_out/r3b_bench_$e.json)"
done
