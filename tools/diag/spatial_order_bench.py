"""bench.py with BiSeNet.spatial_enqueued_last set: spatial_order_bench.py 0|1 [bench args]."""
import sys
sys.path.insert(0, ".")
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet  # noqa: E402
BiSeNet.spatial_enqueued_last = bool(int(sys.argv[1]))
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402
bench.main()
