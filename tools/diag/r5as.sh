#!/bin/bash
# Weight-gradient split reduces started early (batches of REDUCE_EARLY on a reduce stream beside
# the backward) vs all at the end: parity (models, graphed step, DP, configs), bench A/B.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_dp_gpu.py tests/test_configs_gpu.py > gpurun_out/r5as_pytest.log 2>&1 || { tail -30 gpurun_out/r5as_pytest.log; exit 1; }
tail -1 gpurun_out/r5as_pytest.log
for r in 1 2 3; do
  for v in 0 4 8; do
    timeout -k 10 300 python3 tools/diag/reduce_early_bench.py $v --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5as_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('seg early', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5as_bench.json $v | tee -a gpurun_out/r5as_ab.txt
  done
done
for v in 0 4; do
  for w in bisenet-da deeplab-seg; do
    timeout -k 10 300 python3 tools/diag/reduce_early_bench.py $v --workload $w --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5as_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[3], 'early', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5as_bench.json $v $w | tee -a gpurun_out/r5as_ab.txt
  done
done
