#!/bin/bash
# BiSeNet spatial-path fork point A/B (train step, branch graph): -1 / 0 / 1 / 2 (current)
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for f in 2 -1 0 1; do
    timeout -k 10 300 python3 tools/diag/fork_bench.py $f --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ae_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('fork_after', sys.argv[2], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5ae_bench.json $f | tee -a gpurun_out/r5ae_ab.txt
  done
done
