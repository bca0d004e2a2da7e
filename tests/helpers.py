"""Shared test helpers: problem builders (numpy RNG, independent of the product generator) and
conversions between torch tensors and the oracle's numpy representation."""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle

DTYPES = {"f32": torch.float32, "f64": torch.float64, "bf16": torch.bfloat16, "f16": torch.float16}


def to_oracle(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def from_f32(x: np.ndarray, dtype: torch.dtype) -> torch.Tensor:
    """f32 numpy -> torch dtype with RNE rounding (bf16 via the oracle's bit routine)."""
    if dtype == torch.bfloat16:
        return torch.from_numpy(oracle.f32_to_bf16_bits(x).view(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(np.ascontiguousarray(x)).to(dtype)


def random_csr(m, k, degrees, rng, idx_dtype=torch.int32, val_dtype=torch.float32, exact=False,
               hub_rows=None):
    """CSR with the given per-row degree list (sorted unique columns)."""
    degrees = np.asarray(degrees, dtype=np.int64)
    rp = np.zeros(m + 1, dtype=np.int64)
    rp[1:] = np.cumsum(degrees)
    cols = np.empty(rp[-1], dtype=np.int64)
    for r in range(m):
        d = degrees[r]
        if d:
            cols[rp[r]:rp[r + 1]] = np.sort(rng.choice(k, size=d, replace=False))
    nnz = int(rp[-1])
    if exact:
        vals = rng.choice(np.array([-2.0, -1.0, 1.0, 2.0], dtype=np.float32), size=nnz)
    else:
        vals = rng.uniform(-1, 1, size=nnz).astype(np.float32)
    np_idx = np.int32 if idx_dtype == torch.int32 else np.int64
    return (torch.from_numpy(rp.astype(np_idx)), torch.from_numpy(cols.astype(np_idx)),
            from_f32(vals, val_dtype))


def random_dense(k, n, rng, dtype=torch.float32, exact=False):
    if exact:
        x = rng.integers(-8, 9, size=(k, n)).astype(np.float32)
    else:
        x = rng.uniform(-1, 1, size=(k, n)).astype(np.float32)
    return from_f32(x, dtype)


def dtype_name(dt: torch.dtype) -> str:
    return {v: k for k, v in DTYPES.items()}[dt]


def oracle_spmm(rp, ci, vals, b, **kw):
    return oracle.spmm(to_oracle(rp), to_oracle(ci), to_oracle(vals), to_oracle(b),
                       dtype=dtype_name(b.dtype), **kw)


def assert_bitwise(out: torch.Tensor, ref: np.ndarray, what=""):
    got = to_oracle(out)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    g = np.ascontiguousarray(got).view(np.uint8)
    r = np.ascontiguousarray(ref).view(np.uint8)
    if not np.array_equal(g, r):
        gf, rf = got.astype(np.float64) if got.dtype != np.uint16 else oracle.bf16_bits_to_f32(got), \
            ref.astype(np.float64) if ref.dtype != np.uint16 else oracle.bf16_bits_to_f32(ref)
        diff = np.abs(np.asarray(gf, dtype=np.float64) - np.asarray(rf, dtype=np.float64))
        idx = np.unravel_index(np.argmax(diff), diff.shape)
        raise AssertionError(f"{what}: not bit-exact; {int((g != r).sum())} bytes differ, "
                             f"max |diff| {diff.max():.3e} at {idx}")


def power_law_degrees(m, nnz, k, rng, gamma=2.5):
    if nnz > m * k:
        raise ValueError(f"power_law_degrees: {nnz} nonzeros do not fit {m} x {k}")
    w = (np.arange(1, m + 1, dtype=np.float64)) ** (-1.0 / (gamma - 1.0))
    d = np.floor(nnz * w / w.sum()).astype(np.int64)
    d = np.minimum(d, k)
    rem = nnz - d.sum()
    i = 0
    while rem > 0:
        if d[i % m] < k:
            d[i % m] += 1
            rem -= 1
        i += 1
    rng.shuffle(d)
    return d
