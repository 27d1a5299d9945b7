# Debug helper (GPU): where the bf16 MFMA FCM's per-cluster weight sums part from the fp64
# oracle on the fcm10m preset's clustered data (cluster_std 0.25): worst clusters, their
# oracle weight, how many sample rows have them nearest / second nearest, and the same
# numbers for the 'one' and 'x3' forms, at the random-row init.
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs  # noqa: E402
from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM, HipTowerFCM  # noqa: E402
from tensorflow_distributed_clustering_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda", 0)
n, d, k, m = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 128, 1024, 2.0
std = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
x = gaussian_blobs(n, d, k, seed=0, cluster_std=std, dtype=torch.bfloat16, device=dev)
g = torch.Generator().manual_seed(1)
C = x[torch.randperm(n, generator=g)[:k].to(dev)].double()
C = C + 0.01 * torch.randn(C.shape, generator=g, dtype=torch.float64).to(dev)  # off the rows
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if iters:  # exact fp32 tower iterations from C: a realistic late-iteration centroid set
    tw = HipTowerFCM(x.float(), k, "fp32", m, True)
    for _ in range(iters):
        wx = torch.zeros(k, d, dtype=torch.float64, device=dev)
        ws = torch.zeros(k, dtype=torch.float64, device=dev)
        lab = torch.empty(n, dtype=torch.int32, device=dev)
        tw.step(C.float().contiguous(), lab, wx, ws)
        keep = ws > 0
        C[keep] = wx[keep] / ws[keep, None]
    print(f"after {iters} exact iterations")
wr, wsr, labr = ref.fcm_partial(x.double(), C, m, True, acc_dtype=torch.float64, exact=True)
tops, colmin = [], torch.full((k,), float("inf"), dtype=torch.float64, device=dev)
for r0 in range(0, n, 8192):  # chunked: the [n, K, D] difference block would not fit
    dd = ref.pairwise_sqdist(x[r0:r0 + 8192].double(), C, exact=True)
    tops.append(dd.topk(3, dim=1, largest=False))
    colmin = torch.minimum(colmin, dd.min(0).values)
from types import SimpleNamespace
top3 = SimpleNamespace(values=torch.cat([t.values for t in tops]),
                       indices=torch.cat([t.indices for t in tops]))
near1 = torch.bincount(top3.indices[:, 0], minlength=k)
near2 = torch.bincount(top3.indices[:, 1], minlength=k)
near3 = torch.bincount(top3.indices[:, 2], minlength=k)
print(f"n={n} std={std} d2 nearest median {float(top3.values[:, 0].median()):.3f} "
      f"2nd {float(top3.values[:, 1].median()):.3f} 3rd {float(top3.values[:, 2].median()):.3f}")
ok = wsr > 1e-6 * float(wsr.sum())
print("clusters ok", int(ok.sum()), "wsr min/median/max", float(wsr[ok].min()),
      float(wsr[ok].median()), float(wsr.max()))
for name, mk in (("tower fp32", lambda: HipTowerFCM(x.float(), k, "fp32", m, True)),
                 ("mfma x3", lambda: HipMfmaFCM(x, k, m, True)),
                 ("mfma one", lambda: HipMfmaFCM(x, k, m, True))):
    ops = mk()
    if name == "mfma one":
        ops.one_product = True
    wx = torch.zeros(k, d, dtype=torch.float64, device=dev)
    ws = torch.zeros(k, dtype=torch.float64, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    ops.step(C.to(ops.c_dtype).contiguous(), lab, wx, ws)
    torch.cuda.synchronize()
    rel = (ws - wsr).abs() / wsr.clamp_min(1e-300)
    rel[~ok] = 0
    worst = rel.topk(5).indices
    cr = wx / ws.clamp_min(1e-300)[:, None]
    cref = wr / wsr.clamp_min(1e-300)[:, None]
    cerr = float((cr - cref)[ok].abs().max()) / float(cref[ok].abs().max())
    xx = ((x.double() - C.mean(0)) ** 2).sum(1)
    if name == "mfma x3":
        print(f"   rows with nearest d2 <= 2^-16 ||x - mu||^2 (zero floor): "
              f"{int((top3.values[:, 0] <= xx * 2 ** -16).sum())}")
    print(f"{name}: max rel ws {float(rel.max()):.3e}  median {float(rel[ok].median()):.3e}  "
          f"centroid err {cerr:.3e}  label agree {float((lab == labr).double().mean()):.5f}")
    for j in worst.tolist():
        print(f"   k={j} wsr {float(wsr[j]):.4e} ws {float(ws[j]):.4e} near1 {int(near1[j])} "
              f"near2 {int(near2[j])} near3 {int(near3[j])} min d2 {float(colmin[j]):.3f}")
