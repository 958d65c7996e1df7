#!/bin/bash
# side-stream weight gradients (RTSDS_OVERLAP=1; excludes the branch streams) vs the branch streams
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in "0 0" "1 0" "1 16384"; do
    set -- $v
    RTSDS_OVERLAP=$1 RTSDS_OVERLAP_MAXROWS=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ag_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('overlap', sys.argv[2], 'maxrows', sys.argv[3], d['value'], d['ms_per_step'], d['graph_submit'])" gpurun_out/r5ag_bench.json $1 $2 | tee -a gpurun_out/r5ag_ab.txt
  done
done
