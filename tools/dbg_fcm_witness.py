# Debug helper (GPU): re-runs bench.py's FCM witness on a small FCM bench config and prints
# its intermediates (bench.py reported fcm_weight_sum_rel_err == 0.0 exactly on the GPU).
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

orig = bench.fcm_witness


def traced(eng, x, n_global, s, e, comm, torch, a):
    from tensorflow_distributed_clustering_amd.ops import make_fcm_ops
    from tensorflow_distributed_clustering_amd.ops import reference as ref
    dev = comm.device
    C = eng.centers().double()
    k, d = C.shape
    g = torch.arange(bench.WITNESS_ROWS, dtype=torch.float64) * (n_global / bench.WITNESS_ROWS)
    g = torch.unique(g.floor().long())
    loc = (g[(g >= s) & (g < e)] - s).to(dev)
    xs = x.index_select(0, loc)[:, :d]
    print("x", tuple(x.shape), x.dtype, "xs", tuple(xs.shape), "C", tuple(C.shape),
          "dtype_name", eng.dtype_name)
    ops = make_fcm_ops(xs.float(), k, eng.dtype_name, eng.m, eng.cfg.fcm_nan_to_zero,
                       eng.cfg.backend)
    wx = torch.zeros(k, d, dtype=torch.float64, device=dev)
    ws = torch.zeros(k, dtype=torch.float64, device=dev)
    lab = torch.empty(xs.shape[0], dtype=torch.int32, device=dev)
    ops.step(C.to(ops.c_dtype).contiguous(), lab, wx, ws)
    wr, wsr, _ = ref.fcm_partial(xs.double(), C, eng.m, eng.cfg.fcm_nan_to_zero,
                                 acc_dtype=torch.float64)
    wre, wsre, _ = ref.fcm_partial(xs.double(), C, eng.m, eng.cfg.fcm_nan_to_zero,
                                   acc_dtype=torch.float64, exact=True)
    print("ops", ops.name, "ws[:6]", ws[:6].tolist())
    print("wsr[:6]", wsr[:6].tolist())
    print("wsr exact[:6]", wsre[:6].tolist())
    ok = wsr > 1e-6 * float(wsr.sum())
    print("ok", int(ok.sum()), "ws sum", float(ws.sum()), "wsr sum", float(wsr.sum()),
          "max rel", float(((ws - wsr).abs() / wsr.clamp_min(1e-300))[ok].max()),
          "max rel vs exact", float(((ws - wsre).abs() / wsre.clamp_min(1e-300))[ok].max()),
          "nan ws", int(torch.isnan(ws).sum()), "nan wsr", int(torch.isnan(wsr).sum()))
    return orig(eng, x, n_global, s, e, comm, torch, a)


bench.fcm_witness = traced
bench.main(["--method", "fcm", "--dtype", "bf16", "--dim", "128", "--k", "1024",
            "--n-per-gpu", "500000", "--fuzzifier", "2", "--steps", "3", "--warmup", "1",
            "--no-steady"])
