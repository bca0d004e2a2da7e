"""Column indices outside [0, K): the reference gather's semantics.

OneFlow's CPU gather zero-fills the gathered row of an index >= the table size and CHECK-fails on
a negative one (oneflow/user/kernels/gather_kernel_util.cpp:80-89); its CUDA gather zero-fills
any index outside [0, size) (gather_kernel_util.cu:36).  Composed into the SpMM, such a nonzero
adds val * 0 (+-0, or NaN for a non-finite value) in its place of the accumulation order.  So:

  col >= K   zero row in the HIP kernel (every form), the kCPU kernel and the oracle, bit-exact;
  col < 0    the kCPU kernel and the oracle raise (CHECK_GE); the HIP kernel zero-fills, the
             CUDA gather's semantics (oracle negative="zero").

An independent restatement: appending a zero row K to B and pointing every out-of-range column
at it must give the same bits.  The gradient ops follow: the SDDMM reads the same zero row, and
the transpose leaves the out-of-range entries out of every row of A^T (sorted past row_ptr_T[K]).
"""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import ops
from oracle import oracle
from tests.helpers import DTYPES, assert_bitwise, oracle_spmm, random_csr, random_dense


def _problem(rng, m=300, k=2000, n=16, idx=torch.int32, dtype=torch.float32, hub=1500):
    deg = rng.integers(0, 40, size=m)
    deg[5] = hub  # a hub row: split at every width (chunks <= 512)
    deg[9] = 200
    rp, ci, v = random_csr(m, k, deg, rng, idx, dtype)
    # out-of-range columns: = K, far past K, in the hub row (in several chunks) and in short rows
    bad = rng.choice(ci.numel(), size=40, replace=False)
    ci = ci.clone()
    ci[bad[:20]] = k
    ci[bad[20:30]] = k + 12345
    ci[int(rp[5]) + np.array([0, 1, 511, 512, 1000, 1499])] = k
    b = random_dense(k, n, rng, dtype)
    return m, k, n, rp, ci, v, b


def _appended(ci, b, k, negative_too=False):
    """The same problem with B given a zero row K and every out-of-range column pointed at it."""
    c = ci.clone().long()
    bad = (c >= k) | (c < 0) if negative_too else (c >= k)
    c[bad] = k
    zero = torch.zeros((1, b.shape[1]), dtype=b.dtype, device=b.device)
    return c.to(ci.dtype), torch.cat([b, zero], 0)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64", "f16"])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_oracle_and_cpu_kernel_zero_fill_col_ge_k(dtype, idx):
    rng = np.random.default_rng(7)
    m, k, n, rp, ci, v, b = _problem(rng, idx=idx, dtype=DTYPES[dtype])
    ci2, b2 = _appended(ci, b, k)
    ref = oracle_spmm(rp, ci2, v, b2)  # independent: a real zero row
    assert_bitwise(torch.from_numpy(np.ascontiguousarray(ref)) if dtype != "bf16" else
                   torch.from_numpy(ref.view(np.int16)).view(torch.bfloat16),
                   oracle_spmm(rp, ci, v, b), "oracle zero fill vs appended zero row")
    out = fs.spmm(rp, ci, v, m, k, b)  # the kCPU kernel through the op layer
    assert_bitwise(out, ref, f"kCPU {dtype}")
    for split, chunk in [(100, 100), (300, 77)]:
        o = ops.spmm_csr_cpu(rp, ci, v, b, m, k, options=ops.make_options(split=split, chunk=chunk))
        assert_bitwise(o, oracle_spmm(rp, ci2, v, b2, split=split, chunk=chunk), f"{split}/{chunk}")


def test_nonfinite_value_on_a_zero_row_gives_nan():
    """val * 0 is NaN for val = inf / NaN: the zero-filled row does not drop the nonzero."""
    rp = torch.tensor([0, 2, 3], dtype=torch.int32)
    ci = torch.tensor([0, 5, 5], dtype=torch.int32)  # K = 4: columns 5 are out of range
    v = torch.tensor([1.0, float("inf"), -2.0])
    b = torch.ones((4, 3))
    out = fs.spmm(rp, ci, v, 2, 4, b)
    assert torch.isnan(out[0]).all()
    assert torch.equal(out[1], torch.zeros(3))  # -2 * 0 = -0, and +0 + -0 = +0
    assert not torch.signbit(out[1]).any()
    ref = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy(), k=4)
    assert np.isnan(ref[0]).all() and (ref[1] == 0).all()


def test_negative_column_raises_on_cpu():
    rng = np.random.default_rng(3)
    m, k, n, rp, ci, v, b = _problem(rng)
    ci[17] = -1
    with pytest.raises(fs.OfxError, match="negative column"):
        fs.spmm(rp, ci, v, m, k, b)
    with pytest.raises(ValueError, match="negative column"):
        oracle_spmm(rp, ci, v, b)
    # the CUDA gather's semantics (the device kernel's): a zero row, like col >= K
    ci2, b2 = _appended(ci, b, k, negative_too=True)
    np.testing.assert_array_equal(oracle_spmm(rp, ci, v, b, negative="zero").view(np.uint32),
                                  oracle_spmm(rp, ci2, v, b2).view(np.uint32))


def test_cpu_gradient_ops_raise_on_a_negative_column():
    """The kCPU transpose and SDDMM report a negative column as the kCPU forward does (the CPU
    gather's CHECK_GE, gather_kernel_util.cpp:80), instead of zero-filling it."""
    rng = np.random.default_rng(17)
    m, k, n, rp, ci, v, b = _problem(rng, n=8)
    ci[33] = -2
    with pytest.raises(fs.OfxError, match="negative column"):
        fs.csr_transpose(rp, ci, k)
    with pytest.raises(fs.OfxError, match="negative column"):
        fs.sddmm(rp, ci, random_dense(m, n, rng), b)


def test_cpu_transpose_and_sddmm_with_out_of_range_columns():
    rng = np.random.default_rng(11)
    m, k, n, rp, ci, v, b = _problem(rng, n=24)
    inr = (ci.long() >= 0) & (ci.long() < k)
    rp_t, ci_t, perm = fs.csr_transpose(rp, ci, k)
    o_rp, o_ci, o_perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    np.testing.assert_array_equal(rp_t.numpy(), o_rp)
    np.testing.assert_array_equal(ci_t.numpy(), o_ci)
    np.testing.assert_array_equal(perm.numpy(), o_perm)
    assert int(rp_t[-1]) == int(inr.sum())  # A^T's rows hold exactly the in-range entries
    # the out-of-range entries sit past row_ptr_T[K], in ascending nonzero order
    tail = perm[int(rp_t[-1]):].long()
    assert torch.equal(tail, torch.nonzero(~inr).flatten())
    a = random_dense(m, n, rng)
    got = fs.sddmm(rp, ci, a, b)
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), a.numpy(), b.numpy())
    np.testing.assert_array_equal(got.numpy().view(np.uint32), ref.view(np.uint32))
    ci2, b2 = _appended(ci, b, k)
    ref2 = oracle.sddmm(rp.numpy(), ci2.numpy(), a.numpy(), b2.numpy())
    np.testing.assert_array_equal(ref.view(np.uint32), ref2.view(np.uint32))


# ---- HIP ----------------------------------------------------------------------------------------
# auto, small, mid (two), bandwidth, prefetching with / without wave items, global B loads
FORMS = [0, 30000, 30001, 30002, 30003, 30004, 30005, 30006]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64"])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("n", [1, 16, 64, 128])
def test_gpu_zero_fill_every_form(device, dtype, idx, n):
    rng = np.random.default_rng(n)
    m, k, n, rp, ci, v, b = _problem(rng, n=n, idx=idx, dtype=DTYPES[dtype])
    ci[3] = -1  # device: a zero row (the CUDA gather's semantics)
    ci[4] = torch.iinfo(idx).max
    ci2, b2 = _appended(ci, b, k, negative_too=True)
    ref = oracle_spmm(rp, ci2, v, b2)
    np.testing.assert_array_equal(
        np.ascontiguousarray(oracle_spmm(rp, ci, v, b, negative="zero")).view(np.uint8),
        np.ascontiguousarray(ref).view(np.uint8))
    d = [t.to(device) for t in (rp, ci, v, b)]
    for form in FORMS:
        out = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=form))
        assert_bitwise(out, ref, f"form {form} {dtype} n={n}")
    out = fs.spmm(*d[:3], m, k, d[3])  # the op layer
    assert_bitwise(out, ref, "op layer")


@pytest.mark.gpu
def test_gpu_zero_fill_row_split_and_wave_items(device):
    """A launch over a row range (S(0) slice) and the small-launch wave items."""
    rng = np.random.default_rng(5)
    m, k, n, rp, ci, v, b = _problem(rng, m=3000, k=5000, n=32, hub=4000)
    ci2, b2 = _appended(ci, b, k)
    d = [t.to(device) for t in (rp, ci, v, b)]
    full = oracle_spmm(rp, ci2, v, b2)
    for form in FORMS:
        sub = ops.spmm_csr_device(*d, m, k, row_begin=1, row_end=2900,
                                  options=ops.make_options(variant=form))
        assert_bitwise(sub, full[1:2900], f"row range, form {form}")


@pytest.mark.gpu
def test_gpu_transpose_and_sddmm_with_out_of_range_columns(device):
    rng = np.random.default_rng(13)
    m, k, n, rp, ci, v, b = _problem(rng, n=40)
    ci[2] = -7
    rp_t, ci_t, perm = fs.csr_transpose(rp.to(device), ci.to(device), k)
    o_rp, o_ci, o_perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    np.testing.assert_array_equal(rp_t.cpu().numpy(), o_rp)
    np.testing.assert_array_equal(ci_t.cpu().numpy(), o_ci)
    np.testing.assert_array_equal(perm.cpu().numpy(), o_perm)
    for nn in (40, 3000):  # narrow and wide SDDMM kernels
        aa = random_dense(m, nn, rng)
        bb = random_dense(k, nn, rng)
        got = fs.sddmm(rp.to(device), ci.to(device), aa.to(device), bb.to(device))
        ref = oracle.sddmm(rp.numpy(), ci.numpy(), aa.numpy(), bb.numpy())
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,n", [("f32", 16), ("f32", 99), ("bf16", 32)])
def test_gpu_zero_fill_mid_size_automatic_forms(device, dtype, n):
    """out-of-range columns in launches of more than 32,768 rows and more than 3M
    nonzeros, where only the automatic choice reaches the N = 16 narrow form (16-lane wave items),
    the shifted window (odd widths), the 16-bit lane layouts and the by-index light rows; and the
    same graph below 3M nonzeros (the prefetching form, its in-kernel hub reduce)."""
    dt = DTYPES[dtype]
    for nnz in (3_300_000, 2_900_000):
        m = k = 100_000
        rp, ci, v = fs.synth.csr(m, k, nnz, val_dtype=dt)
        rng = np.random.default_rng(nnz + n)
        ci = ci.clone()
        bad = rng.choice(ci.numel(), size=2000, replace=False)
        ci[bad[:1000]] = k
        ci[bad[1000:]] = k + 777
        hub = int(torch.argmax(rp[1:] - rp[:-1]))  # the longest row: a split hub
        ci[int(rp[hub]) + np.arange(0, 2048, 97)] = k
        b = random_dense(k, n, rng, dt)
        ci2, b2 = _appended(ci, b, k)
        ref = oracle_spmm(rp, ci2, v, b2)
        d = [t.to(device) for t in (rp, ci, v, b)]
        out = fs.spmm(*d[:3], m, k, d[3])
        torch.cuda.synchronize()
        assert_bitwise(out, ref, f"{dtype} n={n} nnz={nnz} auto "
                                 f"({ops.describe(m, k, n, nnz, dt)['form']})")
