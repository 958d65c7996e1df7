#!/bin/bash
# Split reduces of the main stream's weight gradients before the join of the branch streams (1)
# vs all after it (0): parity (models, graphed step, DP), bench A/B (seg, DA).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_dp_gpu.py > gpurun_out/r5au_pytest.log 2>&1 || { tail -30 gpurun_out/r5au_pytest.log; exit 1; }
tail -1 gpurun_out/r5au_pytest.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python3 tools/diag/reduce_order_bench.py $v --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5au_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('seg own_first', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5au_bench.json $v | tee -a gpurun_out/r5au_ab.txt
  done
done
for v in 0 1; do
  timeout -k 10 300 python3 tools/diag/reduce_order_bench.py $v --workload bisenet-da --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5au_bench.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('da own_first', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5au_bench.json $v | tee -a gpurun_out/r5au_ab.txt
done
