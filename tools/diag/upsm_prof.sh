set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/upsm/kt -o run -- python3 tools/diag/upsm_bench.py 10 > gpurun_out/upsm.log 2>&1
python3 tools/kstats.py /tmp/upsm/kt/run_kernel_stats.csv 10 >> gpurun_out/upsm.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d /tmp/upsm/pmc -o run -- python3 tools/diag/upsm_bench.py 3 >> gpurun_out/upsm.log 2>&1
python3 - >> gpurun_out/upsm.log <<'PY'
import csv, glob, collections
p = glob.glob('/tmp/upsm/pmc/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.Counter())
for r in csv.DictReader(open(p)):
    if 'upsoftmax' in r['Kernel_Name']:
        agg[r['Kernel_Name'][:40]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    print(k, dict(v))
PY
echo done
