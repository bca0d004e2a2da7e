"""Randomised properties (hypothesis on CPU, a seeded sweep on the GPU): for arbitrary small
shapes, degrees (empty rows, hub rows past the split), widths, index/value dtypes, split/chunk
schedules and row ranges, the operator's kernels equal the oracle bit for bit, and the row-range
form equals the corresponding slice of the full product."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oneflow_spmm import ops

from helpers import DTYPES, assert_bitwise, oracle_spmm, random_csr, random_dense


def _case(seed, m, k, n, dtype, idx, hub, split):
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, min(k, 12) + 1, size=m)
    if hub and m:
        deg[rng.integers(0, m)] = k  # a full row: longer than the split below when k > split
    rp, ci, v = random_csr(m, k, deg, rng, idx_dtype=idx, val_dtype=DTYPES[dtype])
    b = random_dense(k, n, rng, dtype=DTYPES[dtype])
    opts = ops.make_options(split=split, chunk=max(1, split // 2)) if split else None
    return rp, ci, v, b, opts


problem = st.tuples(
    st.integers(0, 2**31 - 1),                 # seed
    st.integers(0, 60),                        # m
    st.integers(1, 90),                        # k
    st.integers(1, 40),                        # n
    st.sampled_from(["f32", "f64", "bf16", "f16"]),
    st.sampled_from([torch.int32, torch.int64]),
    st.booleans(),                             # a hub row
    st.sampled_from([0, 4, 16]),               # split threshold (0 = default)
)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(problem, st.data())
def test_cpu_kernel_equals_oracle(p, data):
    seed, m, k, n, dtype, idx, hub, split = p
    rp, ci, v, b, opts = _case(seed, m, k, n, dtype, idx, hub, split)
    lo = data.draw(st.integers(0, m))
    hi = data.draw(st.integers(lo, m))
    kw = {}
    if split:
        kw = dict(split=split, chunk=max(1, split // 2))
    got = ops.spmm_csr_cpu(rp, ci, v, b, m, k, row_begin=lo, row_end=hi, options=opts)
    assert_bitwise(got, oracle_spmm(rp, ci, v, b, row_begin=lo, row_end=hi, **kw),
                   f"cpu m={m} k={k} n={n} {dtype} rows [{lo},{hi})")


@pytest.mark.gpu
def test_gpu_kernel_equals_oracle_random_sweep(device):
    rng = np.random.default_rng(2024)
    for it in range(80):
        m, k, n = int(rng.integers(0, 300)), int(rng.integers(1, 400)), int(rng.integers(1, 300))
        dtype = ["f32", "f64", "bf16", "f16"][it % 4]
        idx = (torch.int32, torch.int64)[(it // 4) % 2]
        split = [0, 4, 16, 64][(it // 8) % 4]
        rp, ci, v, b, opts = _case(int(rng.integers(0, 2**31)), m, k, n, dtype, idx,
                                   bool(it % 3 == 0), split)
        lo = int(rng.integers(0, m + 1))
        hi = int(rng.integers(lo, m + 1))
        kw = dict(split=split, chunk=max(1, split // 2)) if split else {}
        out = torch.full((hi - lo, n), float("nan"), dtype=DTYPES[dtype], device=device)
        ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                            out=out, row_begin=lo, row_end=hi, options=opts)
        torch.cuda.synchronize()
        assert_bitwise(out, oracle_spmm(rp, ci, v, b, row_begin=lo, row_end=hi, **kw),
                       f"gpu it={it} m={m} k={k} n={n} {dtype} split={split} rows [{lo},{hi})")
