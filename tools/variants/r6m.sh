#!/bin/bash
# tree vs previous-revision Python (same library): kernel traces, then 5 more alternating bench rounds
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in tree old; do
  d=.; [ "$v" = old ] && d=_abtree
  (cd $d && RTSDS_LIB=$GRAFT_REPO_ROOT/rtsds_amd/librtsds_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6m_prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r6m_bench_$v.json 2>/dev/null) || exit 1
done
timeout -k 10 1200 bash tools/ab_tree.sh 5 > gpurun_out/r6m_step.txt 2>&1; cat gpurun_out/r6m_step.txt
