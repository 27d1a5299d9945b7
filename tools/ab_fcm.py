"""A/B of the FCM MFMA accumulate pass: ``python tools/ab_fcm.py {one,x3} <bench.py args>``.

``one``: one-product distances with the stats pass's two-nearest fix-up (the default);
``x3``: bf16x3 distances in the accumulate pass (HipMfmaFCM.one_product = False).  The
stagger of the accumulate kernel is switched by TDC_FCM_NOSTAG=1 in the environment."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_clustering_amd import ops  # noqa: E402

mode = sys.argv[1]
assert mode in ("one", "x3"), mode
ops.HipMfmaFCM.one_product = mode == "one"
import bench  # noqa: E402

sys.exit(bench.main(sys.argv[2:]))
