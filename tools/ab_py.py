"""Run bench.py with class / module attributes overridden (Python-level A/B on one box):
    python3 tools/ab_py.py 'rtsds_amd.models.bisenet.build_bisenet.BiSeNet.eval_branch_batch=0' -- [bench args]"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
i = sys.argv.index("--")
for spec in sys.argv[1:i]:
    target, value = spec.split("=", 1)
    parts = target.split(".")
    for k in range(len(parts) - 1, 0, -1):
        try:
            obj = importlib.import_module(".".join(parts[:k]))
        except ImportError:
            continue
        for a in parts[k:-1]:
            obj = getattr(obj, a)
        setattr(obj, parts[-1], eval(value))
        break
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
