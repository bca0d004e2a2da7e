"""CPU: the product's DeviceType::kCPU kernel and host utilities against the oracle, bit for bit."""
import json
import os

import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import ops, synth
from oracle import oracle
from tests.helpers import (DTYPES, assert_bitwise, oracle_spmm, power_law_degrees, random_csr,
                           random_dense, to_oracle)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("n", [1, 5, 16, 128])
def test_cpu_kernel_bitexact(dtype, n):
    rng = np.random.default_rng(n)
    m, k = 200, 300
    deg = rng.integers(0, 30, size=m)
    deg[3] = 290
    rp, ci, v = random_csr(m, k, deg, rng, torch.int64 if n == 5 else torch.int32, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    out = fs.spmm(rp, ci, v, m, k, b)
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"cpu {dtype} n={n}")


def test_cpu_kernel_schedules():
    rng = np.random.default_rng(2)
    m, k, n = 64, 4000, 32
    deg = rng.integers(0, 100, size=m)
    deg[7] = 3900
    rp, ci, v = random_csr(m, k, deg, rng)
    b = random_dense(k, n, rng)
    for split, chunk in [(0, 0), (100, 100), (300, 77), (10**9, 0)]:
        out = ops.spmm_csr_cpu(rp, ci, v, b, m, k, options=ops.make_options(split=split, chunk=chunk))
        assert_bitwise(out, oracle_spmm(rp, ci, v, b, split=split, chunk=chunk), f"{split}/{chunk}")
    out = ops.spmm_csr_cpu(rp, ci, v, b, m, k, options=ops.make_options(ordered=True))
    assert_bitwise(out, oracle_spmm(rp, ci, v, b, ordered=True), "ordered")
    # row sub-range + thread-count independence
    out1 = ops.spmm_csr_cpu(rp, ci, v, b, m, k, row_begin=5, row_end=40, num_threads=1)
    out8 = ops.spmm_csr_cpu(rp, ci, v, b, m, k, row_begin=5, row_end=40, num_threads=8)
    assert torch.equal(out1, out8)
    assert_bitwise(out1, oracle_spmm(rp, ci, v, b)[5:40], "row range")


@pytest.mark.parametrize("name", ["cora_f32", "cora_exact", "hub_n128_f32", "hub_n128_exact",
                                  "n1_f32", "n3_f32", "n17_f32", "empty_f32"])
def test_cpu_kernel_on_golden(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    rp = torch.from_numpy(z["row_ptr"])
    ci = torch.from_numpy(z["col_idx"])
    v = torch.from_numpy(z["values"])
    b = torch.from_numpy(z["b"])
    out = fs.spmm(rp, ci, v, int(z["m"]), int(z["k"]), b)
    ok, worst = oracle.within_tolerance(out.numpy(), z["expected_f64"], z["absum"], 1e-5)
    assert ok, worst
    if "exact" in name:
        np.testing.assert_array_equal(out.numpy(), z["expected_f64"].astype(np.float32))


def test_partition_fixture_host_utils():
    part = json.load(open(os.path.join(GOLD, "partition.json")))
    for key, ranges in part["balanced"].items():
        total, g = map(int, key.split("/"))
        for r, (lo, hi) in enumerate(ranges):
            assert fs._C.balanced_range(total, g, r) == (lo, hi)
    rp = torch.tensor(part["row_ptr"], dtype=torch.int64)
    for key, sl in part["slices"].items():
        lo, hi = sl["rows"]
        out, n0, n1 = ops.csr_row_slice(rp, lo, hi)
        assert out.tolist() == sl["row_ptr"] and [n0, n1] == sl["nnz"]
    from oneflow_spmm.distributed import padded_owner_remap
    k = part["k"]
    for g, expect in part["padded_remap"].items():
        got = padded_owner_remap(torch.arange(k, dtype=torch.int32), k, int(g))
        assert got.tolist() == expect


def test_synth_generator_properties():
    m, k, nnz = 5000, 4000, 60000
    rp = synth.row_ptr(m, k, nnz)
    assert rp[0] == 0 and rp[-1] == nnz and np.all(np.diff(rp) >= 0)
    c1 = synth.columns(m, k, rp, threads=1)
    c8 = synth.columns(m, k, rp, threads=8)
    np.testing.assert_array_equal(c1, c8)
    for r in range(0, m, 97):
        row = c1[rp[r]:rp[r + 1]]
        assert np.all(np.diff(row) > 0) and (row.size == 0 or (row[0] >= 0 and row[-1] < k))
    # partial generation equals the slice of the full one
    part = synth.columns(m, k, rp, 1000, 2000)
    np.testing.assert_array_equal(part, c1[rp[1000]:rp[2000]])
    deg = np.diff(rp)
    assert deg.max() > 20 * deg.mean()  # power law: hubs exist
    v1 = synth.values(10, 5000)
    v2 = synth.values(0, 6000)[10:5000]
    assert torch.equal(v1, v2) and float(v1.abs().max()) <= 1.0
    ex = synth.values(0, 1000, exact=True)
    assert set(ex.unique().tolist()) <= {-2.0, -1.0, 1.0, 2.0}
    d = synth.dense(3, 9, 7)
    d2 = synth.dense(0, 12, 7)[3:9]
    assert torch.equal(d, d2)


def test_synth_baseline_shapes_small():
    cfg = synth.CONFIGS["cora"]
    rp, ci, v = synth.csr(cfg["m"], cfg["k"], cfg["nnz"])
    assert rp.shape == (2709,) and ci.shape == (10556,) and v.shape == (10556,)
    b = synth.dense(0, cfg["k"], cfg["n"])
    out = fs.spmm(rp, ci, v, cfg["m"], cfg["k"], b)
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), "cora synth")


def test_power_law_helper_sums():
    rng = np.random.default_rng(0)
    d = power_law_degrees(1000, 20000, 500, rng)
    assert d.sum() == 20000 and d.max() <= 500


@pytest.mark.parametrize("dtype,rtol", [("f32", 1e-5), ("bf16", 2.0 ** -8)])
def test_sampled_rows_check_on_cpu(dtype, rtol):
    """The sampled-row checker the full-size GPU tests use (tests/helpers.check_sampled_rows):
    a sub-problem of the sampled rows over only the B rows they reference gives those rows'
    bits, with hub rows that split."""
    from tests.helpers import check_sampled_rows, sub_problem
    rng = np.random.default_rng(8)
    m, k, n = 300, 5000, 64
    deg = rng.integers(0, 40, size=m)
    deg[[4, 77]] = [4500, ops.default_split(n) + 3]
    rp, ci, v = random_csr(m, k, deg, rng, torch.int32, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    out = fs.spmm(rp, ci, v, m, k, b)
    rows = np.array([0, 4, 5, 77, 299])
    sub_rp, sub_c, _, uniq = sub_problem(rp.numpy().astype(np.int64), ci.numpy(), to_oracle(v), rows)
    assert sub_rp[-1] == sum(deg[r] for r in rows) and np.all(uniq[sub_c] >= 0)
    check_sampled_rows(rp.numpy().astype(np.int64), ci.numpy(), v, b, out, rows, rtol, dtype, 4)
    bad = out.clone()
    bad[77, 3] += 1
    with pytest.raises(AssertionError):
        check_sampled_rows(rp.numpy().astype(np.int64), ci.numpy(), v, b, bad, rows, rtol, dtype, 4)
