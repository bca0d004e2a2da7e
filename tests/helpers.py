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


def sub_problem(rp: np.ndarray, cols: np.ndarray, vals: np.ndarray, rows):
    """The rows `rows` of a CSR as a standalone problem over only the B rows they reference:
    (sub_row_ptr, sub_cols into `uniq`, sub_vals, uniq).  Row lengths are unchanged, so the
    operator's hub schedule (a function of the row length and N) is the same as in the full
    problem, and the oracle on the sub-problem gives those rows' bits."""
    rows = np.asarray(rows, dtype=np.int64)
    deg = rp[rows + 1] - rp[rows]
    sub_rp = np.zeros(len(rows) + 1, dtype=np.int64)
    sub_rp[1:] = np.cumsum(deg)
    idx = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows]) if len(rows) else \
        np.zeros(0, dtype=np.int64)
    uniq, inv = np.unique(cols[idx], return_inverse=True)
    return sub_rp, inv.astype(np.int64), vals[idx], uniq


def check_sampled_rows(rp, cols, vals_t, d_b, out, rows, rtol, what, nthreads=16):
    """Rows `rows` of a device result `out` (= A @ d_b) against the oracle: bit-exact with the
    operator's schedule, and both the result and the pure reference order (ascending j, no
    split) within rtol * |.|-sum of the fp64 product C64.  Only the B rows the
    sample references leave the device."""
    dev = d_b.device
    vals_np = to_oracle(vals_t)
    sub_rp, sub_c, sub_v, uniq = sub_problem(rp, cols, vals_np, rows)
    b_sub = to_oracle(d_b.index_select(0, torch.from_numpy(uniq).to(dev)))
    got = out.index_select(0, torch.from_numpy(np.asarray(rows, dtype=np.int64)).to(dev))
    dname = dtype_name(d_b.dtype)
    ref = oracle.spmm(sub_rp, sub_c, sub_v, b_sub, dtype=dname, nthreads=nthreads)
    assert_bitwise(got, ref, f"{what}: sampled rows vs the oracle's schedule")
    f32 = (lambda x: oracle.bf16_bits_to_f32(x)) if dname == "bf16" else \
        (lambda x: np.asarray(x, dtype=np.float32))
    c64, absum = oracle.ref64(sub_rp, sub_c, f32(sub_v), f32(b_sub), nthreads=nthreads)
    ok, worst = oracle.within_tolerance(f32(to_oracle(got)), c64, absum, rtol)
    assert ok, f"{what}: device result vs C64, worst {worst:.3e} > {rtol:.3e}"
    ordered = oracle.spmm(sub_rp, sub_c, sub_v, b_sub, dtype=dname, ordered=True, nthreads=nthreads)
    ok, worst = oracle.within_tolerance(f32(ordered), c64, absum, rtol)
    assert ok, f"{what}: reference order vs C64, worst {worst:.3e} > {rtol:.3e}"
    return len(uniq)
