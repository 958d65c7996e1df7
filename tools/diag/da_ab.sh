set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python3 -u bench.py --workload bisenet-da --no-cpu-baseline --no-conv-profile"
$B --steps 10 > gpurun_out/ab_f10.json 2>/dev/null
$B --steps 160 > gpurun_out/ab_f160.json 2>/dev/null
$B --steps 10 --da-unfused > gpurun_out/ab_u10.json 2>/dev/null
$B --steps 160 --da-unfused > gpurun_out/ab_u160.json 2>/dev/null
$B --steps 40 --graph off > gpurun_out/ab_fe40.json 2>/dev/null
echo ok
