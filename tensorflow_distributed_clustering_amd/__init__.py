"""MI355X-native distributed clustering (K-Means, Fuzzy C-Means, mini-batch K-Means).

Same capabilities as ``Jhonsonzhangxing/tensorflow-distributed-clustering`` re-designed
for AMD Instinct MI355X: one process per GPU over RCCL/xGMI, hand-written CDNA4 HIP
kernels (MFMA distance + fused argmin, LDS-privatised centroid update, fused FCM) and
PyTorch-ROCm for memory/streams.  See SURVEY.md for the reference map.
"""
from .config import ClusterConfig
from .models.kmeans import KMeans, ClusterResult
from .models.fcm import FuzzyCMeans
from .models.minibatch import MiniBatchKMeans
from .parallel.dist import Comm, init_comm, local_comm, shard_bounds
from .serving import ClusterPredictor

__version__ = "0.1.0"

__all__ = ["ClusterConfig", "KMeans", "FuzzyCMeans", "MiniBatchKMeans", "ClusterResult",
           "ClusterPredictor", "Comm", "init_comm", "local_comm", "shard_bounds", "__version__"]
