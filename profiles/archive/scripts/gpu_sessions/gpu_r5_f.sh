#!/bin/bash
# Timing-only bound: the whole toy-MLP step with the GEMM operand split removed (numerically
# wrong by design, TDP_GEMM_EXP): 0 = production, 1 = A pre-split, 2 = B, 3 = both.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do for e in 0 1 2 3; do
  TDP_GEMM_EXP=$e timeout -k 10 200 python bench.py --no-diag > gpurun_out/r5f_exp$e.json 2>/dev/null || exit $?
  echo "round $r exp $e $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' gpurun_out/r5f_exp$e.json)"
done; done
TDP_GEMM_EXP=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r5f_prof3" -o mlp -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --no-diag > gpurun_out/r5f_prof3.log 2>&1 || exit $?
echo done
