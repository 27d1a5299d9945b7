import torch, numpy as np, sys
sys.path.insert(0, ".")
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs, blob_centers
from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM, HipTowerFCM, reference as ref
gpu = torch.device("cuda", 0)
d, k, n = 128, 256, 30000
x = gaussian_blobs(n, d, k, seed=2, dtype=torch.float64, device=gpu)
c0 = torch.as_tensor(blob_centers(k, d, 2) + 0.3, device=gpu)
xf = x.float()
mf = HipMfmaFCM(xf, k, 2.0, True)
tw = HipTowerFCM(xf, k, "fp32", 2.0, True)
cm, ct, cr = c0.float().clone(), c0.float().clone(), c0.clone()
for it in range(4):
    out = []
    for ops, c in ((mf, cm), (tw, ct)):
        lab = torch.empty(n, dtype=torch.int32, device=gpu)
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu); ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.step(c, lab, wx, ws)
        c.copy_((wx / ws[:, None]).float())
        out.append((ws, lab))
    a, b, lr = ref.fcm_partial(x, cr, 2.0, True)
    cr = a / b[:, None]
    dm = (cm.double() - cr).abs().max(1).values; dt = (ct.double() - cr).abs().max(1).values
    j = int(dm.argmax())
    print(it, "mfma max", dm.max().item(), "at", j, "tower max", dt.max().item(), "ws m/t/r", out[0][0][j].item(), out[1][0][j].item(), b[j].item(),
          "minws", b.min().item())
d2 = ((x[:, None, :] - cr[None, j, :]) ** 2).sum(-1) if False else None
