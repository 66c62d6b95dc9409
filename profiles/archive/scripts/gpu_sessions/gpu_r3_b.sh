#!/bin/bash
# hipGraph replay: which hardware queue runs which node. The ResNet-50 rehearsal trace showed a
# bucket collective and the next backward GEMM serialised on one queue. Fork probe under runtime
# knobs, then the rehearsal with and without the reducer's fork marker.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
R="$GRAFT_REPO_ROOT"
for e in X=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=8 GPU_MAX_HW_QUEUES=8; do
  echo "== $e"; env $e timeout -k 10 120 python scripts/graph_fork_probe.py 8; fatal $? probe
done
run() {  # name, env assignments...
  name=$1; shift
  (cd /tmp && env "$@" TDP_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r3b_$name" -o t -- python3 "$R/bench.py" --model resnet50 --graph --steps 4 --warmup 3 --no-diag > "$R/gpurun_out/r3b_$name.log" 2>&1)
  fatal $? $name
  python3 scripts/overlap_report.py gpurun_out/r3b_$name/t_kernel_trace.csv --step-marker gather_batch --last-steps 3 --title $name | sed -n 3,6p
}
run marker X=1
run nomarker TDP_GRAPH_FORK_MARKER=0
for m in toy_mlp resnet50; do for e in TDP_GRAPH_FORK_MARKER=1 TDP_GRAPH_FORK_MARKER=0; do
  env $e timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r3b_bench_${m}_$e.json 2>/dev/null; fatal $? bench_$e
  echo "$m $e $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["diagnostics"])' gpurun_out/r3b_bench_${m}_$e.json)"
done; done
