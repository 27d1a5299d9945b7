"""CPU model of the bf16 FCM distance forms against the fp64 oracle (no GPU).

Rows: the fcm10m data (gaussian_blobs N=10M D=128 K=1024, bf16), a sample of 8192 evenly
spaced rows; centroids: 1024 random rows (the bench's random-row init); m = 2.  Each form
computes d2 = ||x - mu||^2 + ||c - mu||^2 + (x - mu).(-2 (c - mu)) from bf16 hi/lo splits of
the shifted operands (mu = mean of the centroids, as the native split), memberships in
fp64, weights rounded to bf16, and reports the centroid error max|c - c_ref| / max|c_ref| and
the worst relative error of sum_i w_ik, as bench.py's FCM witness does:

    exact+bf16w   exact distances, bf16 weights (the floor any bf16-weight form has)
    x3            bf16x3: xh.ch + xh.cl + xl.ch
    one           xh.ch only
    one+topR      one product, the R nearest (by the one-product d2) corrected to bf16x3
    one+f8x       xh.ch + an fp8 e4m3 cross term (xl 2^8 . ch + xh . cl 2^8) / 2^8
    f8x+topR      the fp8 cross term and the R nearest corrected

    PYTHONPATH=. python tools/fcm_precision_model.py   (~2 minutes, ~6 GB of RAM)
"""
import torch

from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs


def main():
    N, D, K = 10_000_000, 128, 1024
    n = 8192
    idx = (torch.arange(n, dtype=torch.float64) * (N / n)).floor().long()
    X = gaussian_blobs(N, D, K, seed=0, dtype=torch.bfloat16, device="cpu")
    xs = X[idx].double()
    g = torch.Generator().manual_seed(1)
    C = X[torch.randperm(N, generator=g)[:K]].double()
    del X
    mu = C.mean(0)

    def bf(t):
        return t.float().to(torch.bfloat16).double()

    def f8(t):
        return t.float().to(torch.float8_e4m3fn).double()

    xsh, csh = xs - mu, C - mu
    xh, ch = bf(xsh), bf(-2 * csh)
    xl, cl = bf(xsh - xh), bf(-2 * csh - ch)
    xx = (xsh ** 2).sum(1, keepdim=True)
    cc = (csh ** 2).sum(1)
    d_ex = ((xs[:, None, :] - C[None]) ** 2).sum(-1)
    d_one = xx + cc + xh @ ch.T
    d_x3 = d_one + xh @ cl.T + xl @ ch.T
    d_f8 = d_one + (f8(xl * 256) @ f8(ch).T + f8(xh) @ f8(cl * 256).T) / 256

    def memb(d2):
        t = 1 / d2.clamp_min(1e-30)
        return t / t.sum(1, keepdim=True)

    w_ex = memb(d_ex) ** 2
    ws_r = w_ex.sum(0)
    c_r = (w_ex.T @ xs) / ws_r[:, None]
    ok = ws_r > 1e-6 * ws_r.sum()

    def report(name, d2):
        w = bf(memb(d2) ** 2)
        ws = w.sum(0)
        c = (w.T @ xs) / ws[:, None]
        cerr = float((c - c_r)[ok].abs().max() / c_r[ok].abs().max())
        werr = float(((ws - ws_r).abs() / ws_r)[ok].max())
        print(f"{name:14s} centroid err {cerr:.2e}   sum-w err {werr:.2e}")

    def fixed(base, R):
        d = base.clone()
        sel = base.argsort(1)[:, :R]
        d.scatter_(1, sel, d_x3.gather(1, sel))
        return d

    report("exact+bf16w", d_ex)
    report("x3", d_x3)
    report("one", d_one)
    for R in (2, 3, 4, 6, 8):
        report(f"one+top{R}", fixed(d_one, R))
    report("one+f8x", d_f8)
    for R in (1, 2):
        report(f"f8x+top{R}", fixed(d_f8, R))
    r = (xx.sqrt() * cc.sqrt()[None] / d_ex).gather(1, d_ex.argsort(1)[:, :1])
    print(f"median |x||c| / d2 of the nearest centroid: {float(r.median()):.1f}")


if __name__ == "__main__":
    main()
