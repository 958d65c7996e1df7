#!/bin/bash
# BiSeNet spatial path enqueued after the context path (its backward then runs beside layer4..2's)
# vs enqueued at the fork point: models / graphed-step parity, bench A/B (seg + DA), step timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_models_gpu.py > gpurun_out/r5ar_pytest.log 2>&1 || { tail -30 gpurun_out/r5ar_pytest.log; exit 1; }
tail -1 gpurun_out/r5ar_pytest.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python3 tools/diag/spatial_order_bench.py $v --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ar_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('seg last', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5ar_bench.json $v | tee -a gpurun_out/r5ar_ab.txt
  done
done
for v in 0 1; do
  timeout -k 10 300 python3 tools/diag/spatial_order_bench.py $v --workload bisenet-da --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ar_bench.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('da last', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5ar_bench.json $v | tee -a gpurun_out/r5ar_ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5ar -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches > gpurun_out/r5ar.log 2>&1 || exit 1
cp /tmp/r5ar/run_kernel_trace.csv gpurun_out/r5ar_kernel_trace.csv
python3 tools/diag/step_timeline.py gpurun_out/r5ar_kernel_trace.csv 25 > gpurun_out/r5ar_timeline.txt
head -8 gpurun_out/r5ar_timeline.txt
