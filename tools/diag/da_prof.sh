set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="bench.py --workload bisenet-da --no-cpu-baseline --no-conv-profile --steps 5 --warmup 1 --graph off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dap/f -o run -- python3 $A > gpurun_out/dap_f.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dap/u -o run -- python3 $A --da-unfused > gpurun_out/dap_u.log 2>&1
echo ok
