"""bench.py with the BiSeNet spatial-path fork point set: fork_bench.py FORK_AFTER [bench args]
(-1 before the stem, 0 after the stem, 1 after layer1, 2 after layer2)."""
import sys
sys.path.insert(0, ".")
from rtsds_amd.models.bisenet.build_contextpath import _ContextPath  # noqa: E402
_ContextPath.fork_after = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402
bench.main()
