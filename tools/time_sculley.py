"""Time the Sculley mini-batch finalize (N3 variant) in isolation on the GPU:
python tools/time_sculley.py  -> us per call for K=4096 D=64 (minibatch1b shape)."""
import sys
import torch
sys.path.insert(0, ".")
from tensorflow_distributed_clustering_amd import _native

ops = _native.require()
dev = torch.device("cuda", 0)
K, D, DP = 4096, 64, 64
sums = torch.rand(K, D, device=dev) * 100
counts = torch.randint(0, 300, (K,), device=dev).float()
C = torch.randn(K, D, device=dev)
v = torch.rand(K, dtype=torch.float64, device=dev) * 1000
shift = torch.zeros(1, device=dev)
cm2 = torch.zeros(K, DP, dtype=torch.bfloat16, device=dev)
cn = torch.zeros(K, device=dev)
for name, args in (("full", (shift, cm2, cn)), ("no-prep", (shift, None, None)),
                   ("no-shift", (None, cm2, cn))):
    for _ in range(5):
        ops.sculley_update(sums, counts, C, v, *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        ops.sculley_update(sums, counts, C, v, *args)
    e1.record()
    torch.cuda.synchronize()
    print(f"sculley {name}: {e0.elapsed_time(e1) * 10:.1f} us/call")
