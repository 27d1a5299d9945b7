"""Property-based checks (hypothesis) of the invariants the distributed engine relies on."""
import numpy as np
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from tensorflow_distributed_clustering_amd.data.synth import gaussian_blob_rows, gaussian_blobs
from tensorflow_distributed_clustering_amd.models.init import _hash_uniform, floyd_sample
from tensorflow_distributed_clustering_amd.parallel.dist import shard_bounds, shard_sizes


@given(st.integers(0, 10_000), st.integers(1, 64))
def test_shard_bounds_is_array_split(n, world):
    parts = np.array_split(np.arange(n), world)
    for r in range(world):
        s, e = shard_bounds(n, world, r)
        assert (s, e) == ((int(parts[r][0]), int(parts[r][-1]) + 1) if len(parts[r]) else (s, s))
    assert sum(shard_sizes(n, world)) == n


@given(st.integers(1, 5000), st.integers(0, 2**31 - 1), st.data())
def test_floyd_sample_distinct_in_range(n, seed, data):
    k = data.draw(st.integers(1, min(n, 300)))
    s = floyd_sample(n, k, seed)
    assert len(s) == k == len(set(s)) and all(0 <= v < n for v in s)
    assert s == floyd_sample(n, k, seed)  # deterministic


@settings(max_examples=25, deadline=None)
@given(st.integers(1, 2000), st.integers(1, 7), st.integers(1, 6), st.integers(0, 10**6),
       st.integers(0, 5000))
def test_blob_generator_is_shard_invariant(n, d, k, seed, off):
    full = gaussian_blobs(n + off, d, k, seed=seed, dtype=torch.float64)
    part = gaussian_blobs(n, d, k, seed=seed, row_offset=off, dtype=torch.float64)
    assert torch.equal(full[off:], part)
    idx = [off, off + n - 1]
    assert torch.equal(gaussian_blob_rows(idx, d, k, seed=seed), full[idx].double())


@given(st.integers(0, 10**9), st.integers(0, 10))
def test_hash_uniform_range_and_determinism(seed, rnd):
    rows = torch.arange(0, 5000, dtype=torch.int64)
    u = _hash_uniform(rows, seed, rnd)
    assert bool(((u >= 0) & (u < 1)).all())
    assert torch.equal(u, _hash_uniform(rows, seed, rnd))
    assert torch.equal(u[100:200], _hash_uniform(rows[100:200], seed, rnd))
