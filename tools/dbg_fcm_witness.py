# Debug helper (GPU): one MFMA FCM step vs the fp64 oracle on a small sample; prints the
# per-cluster weight sums side by side (bench.py fcm_witness reported 0.0 weight-sum error).
import torch
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import make_fcm_ops
from tensorflow_distributed_clustering_amd.ops import reference as ref
dev = torch.device("cuda", 0)
n, d, k = 65536, 128, 1024
x = gaussian_blobs(n, d, k, seed=0, dtype=torch.float32, device=dev)
C = x[torch.randperm(n, device=dev)[:k]].double()
for dt in ("bf16", "fp32"):
    ops = make_fcm_ops(x, k, dt, 2.0, True)
    wx = torch.zeros(k, d, dtype=torch.float64, device=dev)
    ws = torch.zeros(k, dtype=torch.float64, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    ops.step(C.to(ops.c_dtype).contiguous(), lab, wx, ws)
    wr, wsr, _ = ref.fcm_partial(x.double(), C, 2.0, True, acc_dtype=torch.float64)
    print(dt, ops.name, "ws[:4]", ws[:4].tolist(), "wsr[:4]", wsr[:4].tolist())
    print(dt, "max rel ws err", float(((ws - wsr).abs() / wsr).max()),
          "centroid err", float(((wx / ws[:, None]) - (wr / wsr[:, None])).abs().max() / (wr / wsr[:, None]).abs().max()))
