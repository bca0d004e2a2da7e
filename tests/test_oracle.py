"""CPU: pin the oracle against the golden fixtures (scipy f64 / torch.sparse f32 / exact cases /
integer partition vectors).  Parity with the reference itself is unpinned (no SpMM there)."""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# ref_*.npz hold the reference's own vectors, checked by test_reference_fixtures.py
CASES = sorted(p for p in glob.glob(os.path.join(GOLD, "*.npz"))
               if not os.path.basename(p).startswith(("fused_", "ref_")))
FUSED = sorted(glob.glob(os.path.join(GOLD, "fused_*.npz")))


def test_manifest_hashes():
    man = json.load(open(os.path.join(GOLD, "MANIFEST.json")))
    for name, digest in man["files"].items():
        assert hashlib.sha256(open(os.path.join(GOLD, name), "rb").read()).hexdigest() == digest, name


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p) for p in CASES])
def test_oracle_matches_fixture(path):
    z = np.load(path)  # allow_pickle=False (default)
    rp, c, v, b = z["row_ptr"], z["col_idx"], z["values"], z["b"]
    e64, absum, e32 = z["expected_f64"], z["absum"], z["expected_t32"]
    for ordered in (True, False):
        got = oracle.spmm(rp, c, v, b, ordered=ordered, nthreads=4)
        ok, worst = oracle.within_tolerance(got, e64, absum, 1e-5)
        assert ok, f"{path} ordered={ordered}: worst rel {worst}"
        ok, worst = oracle.within_tolerance(got, e32.astype(np.float64), absum, 2e-6 * 8)
        assert ok, f"{path} vs torch.sparse: worst rel {worst}"
        if "exact" in path:
            np.testing.assert_array_equal(got, e64.astype(np.float32))
            np.testing.assert_array_equal(got, e32)
    c64, ab = oracle.ref64(rp, c, v, b)
    np.testing.assert_allclose(c64, e64, rtol=0, atol=1e-12)
    np.testing.assert_allclose(ab, absum, rtol=1e-12, atol=1e-12)


def test_oracle_reference_order_is_sequential():
    """The ordered oracle is literally ((0 + p0) + p1) + ... with p = fl(val*b): check one row by hand."""
    z = np.load(os.path.join(GOLD, "n3_f32.npz"))
    rp, c, v, b = z["row_ptr"], z["col_idx"], z["values"], z["b"]
    got = oracle.spmm(rp, c, v, b, ordered=True, nthreads=1)
    for r in (1, 50):
        acc = np.zeros(3, dtype=np.float32)
        for j in range(rp[r], rp[r + 1]):
            acc = (acc + (np.float32(v[j]) * b[c[j]]).astype(np.float32)).astype(np.float32)
        np.testing.assert_array_equal(got[r], acc)


def test_oracle_chunked_schedule_by_hand():
    z = np.load(os.path.join(GOLD, "hub_n128_f32.npz"))
    rp, c, v, b = z["row_ptr"], z["col_idx"], z["values"], z["b"]
    split, chunk = 512, 512
    got = oracle.spmm(rp, c, v, b, split=split, chunk=chunk, nthreads=2)
    r = 3  # 2900 nonzeros -> 5 chunks, the last one 852 long
    j0, j1 = rp[r], rp[r + 1]
    nc = (j1 - j0) // chunk
    acc = np.zeros(128, dtype=np.float32)
    for q in range(nc):
        a = j0 + q * chunk
        e = j1 if q == nc - 1 else a + chunk
        part = np.zeros(128, dtype=np.float32)
        for j in range(a, e):
            part = (part + (v[j] * b[c[j]]).astype(np.float32)).astype(np.float32)
        acc = (acc + part).astype(np.float32)
    np.testing.assert_array_equal(got[r], acc)


def test_oracle_default_schedule_at_n256_by_hand():
    """N = 256: the default split is 256 nonzeros; the 900-nonzero row is 3 chunks (256, 256, 388),
    the 257-nonzero row 1 chunk (floor(257 / 256) chunks, the last taking the remainder: the
    whole row from +0), the 600-nonzero row 2 chunks (256, 344)."""
    z = np.load(os.path.join(GOLD, "n256_f32.npz"))
    rp, c, v, b = z["row_ptr"], z["col_idx"], z["values"], z["b"]
    got = oracle.spmm(rp, c, v, b, nthreads=2)
    for r, want_chunks in ((5, 3), (61, 1), (119, 2), (60, 1)):
        j0, j1 = int(rp[r]), int(rp[r + 1])
        nc = max(1, (j1 - j0) // 256) if j1 - j0 > 256 else 1
        assert nc == want_chunks
        acc = np.zeros(256, dtype=np.float32)
        for q in range(nc):
            a = j0 + q * 256
            e = j1 if q == nc - 1 else a + 256
            part = np.zeros(256, dtype=np.float32)
            for j in range(a, e):
                part = (part + (v[j] * b[c[j]]).astype(np.float32)).astype(np.float32)
            acc = (acc + part).astype(np.float32) if nc > 1 else part
        np.testing.assert_array_equal(got[r], acc)


def test_balanced_range_fixture():
    part = json.load(open(os.path.join(GOLD, "partition.json")))
    for key, ranges in part["balanced"].items():
        total, g = map(int, key.split("/"))
        for r, (lo, hi) in enumerate(ranges):
            assert oracle.balanced_range(total, g, r) == (lo, hi)


def test_bf16_rounding_helpers():
    x = np.array([1.0, 1.00390625, 1.005859375, -3.3, 0.0, -0.0, np.inf, np.nan], dtype=np.float32)
    bits = oracle.f32_to_bf16_bits(x)
    back = oracle.bf16_bits_to_f32(bits)
    assert back[0] == 1.0 and back[1] == 1.0  # tie to even
    assert back[2] == np.float32(1.0078125)
    assert np.isnan(back[-1]) and np.isinf(back[-2])
    assert oracle.default_split(128) == 512 and oracle.default_split(1) == 512
    assert oracle.default_split(16) == 512 and oracle.default_split(64) == 512
    assert oracle.default_split(256) == 256 and oracle.default_split(1024) == 128


@pytest.mark.parametrize("path", FUSED, ids=[os.path.basename(p) for p in FUSED])
def test_oracle_bias_act_matches_fused_fixture(path):
    """oracle.bias_act(oracle.spmm(.)) against scipy's fp64 product + bias, relu; exact mode
    bit for bit, fp32 within 1e-5 of the |.|-sum (bias add and relu are 1-Lipschitz, one more
    rounding); and the operator's CPU op path equals the oracle composition bit for bit."""
    import torch

    from oneflow_spmm import _C
    z = np.load(path)
    rp, c, v, b, bias = z["row_ptr"], z["col_idx"], z["values"], z["b"], z["bias"]
    want, absum = z["expected_relu_f64"], z["absum"]
    got = oracle.bias_act(oracle.spmm(rp, c, v, b, nthreads=4), bias, "relu")
    if "exact" in path:
        np.testing.assert_array_equal(got, want.astype(np.float32))
    else:
        bound = 1e-5 * (absum + np.abs(bias.astype(np.float64))[None, :]) + 1e-30
        assert (np.abs(got.astype(np.float64) - want) <= bound).all()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    op = _C.fused_spmm_csr(t(rp), t(c), t(v), int(z["m"]), int(z["k"]), t(b), t(bias), relu=True)
    np.testing.assert_array_equal(op.numpy().view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_oracle_16bit_products_rounded_like_torch_mul(dtype):
    """16-bit dtypes: each product is the tensor-dtype multiply (BinaryFunctor<kMul>,
    oneflow/core/ep/common/primitive/binary_functor.h:46-51: static_cast<Dst>(src0 * src1)),
    summed in fp32 in ascending j and rounded once (unsorted_segment_sum_kernel.cpp:146-205).
    Restated independently with torch's own CPU 16-bit multiply; the unrounded-product variant
    must differ somewhere, so the test sees the rounding."""
    import torch

    from tests.helpers import DTYPES, random_csr, random_dense, to_oracle
    tdt = DTYPES[dtype]
    rng = np.random.default_rng(5)
    m, k, n = 40, 30, 9
    rp, ci, v, b = *random_csr(m, k, rng.integers(0, 25, size=m), rng, val_dtype=tdt), None
    b = random_dense(k, n, rng, tdt)
    got = oracle.spmm(to_oracle(rp), to_oracle(ci), to_oracle(v), to_oracle(b), dtype=dtype,
                      ordered=True, nthreads=1)
    want = torch.zeros((m, n), dtype=torch.float32)
    plain = torch.zeros((m, n), dtype=torch.float32)
    for r in range(m):
        for j in range(int(rp[r]), int(rp[r + 1])):
            want[r] = want[r] + (v[j] * b[ci[j]]).float()  # 16-bit multiply, fp32 add
            plain[r] = plain[r] + v[j].float() * b[ci[j]].float()
    np.testing.assert_array_equal(got, to_oracle(want.to(tdt)))
    assert not np.array_equal(got, to_oracle(plain.to(tdt)))
    x = rng.standard_normal(10000).astype(np.float32) * 3
    ref = to_oracle(torch.from_numpy(x).to(tdt).float())
    np.testing.assert_array_equal(oracle.round16(x, dtype).view(np.uint32), ref.view(np.uint32))
