"""bench.py with functional.REDUCE_EARLY set: reduce_early_bench.py N [bench args] (0: every
weight-gradient split reduce at the end of the backward)."""
import sys
sys.path.insert(0, ".")
import rtsds_amd.functional as F  # noqa: E402
F.REDUCE_EARLY = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402
bench.main()
