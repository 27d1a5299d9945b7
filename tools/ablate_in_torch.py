"""Run tools/ablate_assign.hip (built as build/libablate.so with -DABLATE_NO_MAIN) inside a
PyTorch process, i.e. on torch's bundled HIP runtime, and on torch-allocated tensors.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DABLATE_NO_MAIN -I csrc \
        tools/ablate_assign.hip -o build/libablate.so
    python tools/ablate_in_torch.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "build", "libablate.so"))
lib.ablate_main.argtypes = [ctypes.c_longlong, ctypes.c_int]
lib.ablate_ring_on.restype = ctypes.c_float
lib.ablate_ring_on.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
torch.cuda.init()
lib.ablate_main(0, 0)
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs  # noqa: E402
from tensorflow_distributed_clustering_amd.ops import HipBf16Lloyd  # noqa: E402
n, k = 10_000_000, 1024
dev = torch.device("cuda", 0)
x = gaussian_blobs(n, 128, k, seed=0, dtype=torch.bfloat16, device=dev)
loc = HipBf16Lloyd(x, k)
loc.prepare(x[torch.randperm(n, device=dev)[:k]].float())
lab = torch.zeros(n, dtype=torch.int32, device=dev)
md = torch.zeros(n, dtype=torch.float32, device=dev)
torch.cuda.synchronize()
print("torch tensors: ring %.3f ms" % lib.ablate_ring_on(x.data_ptr(), n, loc.cm2.data_ptr(),
                                                        loc.cnorm.data_ptr(), k, lab.data_ptr(),
                                                        md.data_ptr()))
