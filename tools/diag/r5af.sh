#!/bin/bash
# BiSeNet branch-stream role swap A/B: context path on the branch stream (1) vs the spatial path (0)
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_models_gpu.py -k "branch or graphed" > gpurun_out/r5af_pytest.log 2>&1 || { tail -20 gpurun_out/r5af_pytest.log; exit 1; }
tail -1 gpurun_out/r5af_pytest.log
for r in 1 2; do
  for f in 0 1; do
    timeout -k 10 300 python3 tools/diag/swap_bench.py $f  # (removed after the A/B) --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5af_bench.json 2>gpurun_out/r5af_bench.err || { tail -5 gpurun_out/r5af_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('swap', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'], d['final_loss'])" gpurun_out/r5af_bench.json $f | tee -a gpurun_out/r5af_ab.txt
  done
done
