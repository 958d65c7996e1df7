"""bench.py with functional.REDUCE_OWN_FIRST set: reduce_order_bench.py 0|1 [bench args]."""
import sys
sys.path.insert(0, ".")
import rtsds_amd.functional as F  # noqa: E402
F.REDUCE_OWN_FIRST = bool(int(sys.argv[1]))
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402
bench.main()
