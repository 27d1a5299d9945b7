"""NPZ input (the reference CLI's data format: keys ``X`` [N, D] float64, ``Y``).

``np.savez`` writes an uncompressed (ZIP_STORED) archive, so each member's ``.npy``
payload is a contiguous byte range of the file.  :func:`open_npz_member` memory-maps it
directly: rank r touches only the pages of its own row shard instead of every rank
loading the whole dataset as the reference did (`scripts/distribuitedClustering.py:322-324`).
Compressed archives fall back to ``np.load`` (never with ``allow_pickle``).
"""
from __future__ import annotations

import ast
import struct
import zipfile
from typing import Tuple

import numpy as np


def _npy_header(buf: bytes) -> Tuple[dict, int]:
    if buf[:6] != b"\x93NUMPY":
        raise ValueError("not a .npy payload")
    major = buf[6]
    if major == 1:
        hlen = struct.unpack("<H", buf[8:10])[0]
        start = 10
    else:
        hlen = struct.unpack("<I", buf[8:12])[0]
        start = 12
    header = ast.literal_eval(buf[start:start + hlen].decode("latin1"))
    return header, start + hlen


def open_npz_member(path: str, key: str = "X") -> np.ndarray:
    """Read-only array view of ``key`` (memory-mapped when the member is stored)."""
    name = key + ".npy"
    with zipfile.ZipFile(path) as zf:
        info = zf.getinfo(name)
        if info.compress_type != zipfile.ZIP_STORED:
            with np.load(path, allow_pickle=False) as z:
                return z[key]
        with open(path, "rb") as f:
            f.seek(info.header_offset)
            local = f.read(30)
            if local[:4] != b"PK\x03\x04":
                raise ValueError("corrupt zip local header")
            n_name, n_extra = struct.unpack("<HH", local[26:30])
            data_off = info.header_offset + 30 + n_name + n_extra
            f.seek(data_off)
            head = f.read(4096)
    header, hlen = _npy_header(head)
    if header.get("fortran_order", False):
        with np.load(path, allow_pickle=False) as z:
            return z[key]
    dtype = np.dtype(header["descr"])
    if dtype.hasobject:
        raise ValueError("object arrays are not supported (no pickle loading)")
    return np.memmap(path, dtype=dtype, mode="r", offset=data_off + hlen, shape=tuple(header["shape"]))


def load_shard(path: str, rank: int, world: int, key: str = "X") -> Tuple[np.ndarray, int, int]:
    """This rank's contiguous ``array_split`` shard of ``key`` -> (rows, n_global, row_offset)."""
    from ..parallel.dist import shard_bounds
    arr = open_npz_member(path, key)
    n = arr.shape[0]
    s, e = shard_bounds(n, world, rank)
    return np.array(arr[s:e], copy=True), n, s
