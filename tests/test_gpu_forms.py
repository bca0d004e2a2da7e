"""GPU: the automatic prefetching form on both sides of kPrefetchNnz (ADVICE r3
medium).  Launches of more than 32,768 rows with nonzeros just below and just above 3 * 2^20 take
the prefetching form (U = 32 / 16 loads in flight, the next (col, val) batch prefetched, wave items
at 16 < N <= 64) and the bandwidth form (U = 8) respectively (tests/test_form_rules.py asserts the
rule itself on the CPU).  Each launch is bit-exact against the oracle and against the automatic
pick: fp32 N = 1 / 8 / 25 / 64 / 128, bf16 and f16 N = 8 / 16 / 64, bf16 N = 32, f16 N = 24,
bf16 N = 41, f16 N = 63 (odd
widths: one-element lanes in 16 / 32-lane groups), int32 and int64; a row range, a
plan built once, the fused epilogue, and variants 30004 / 30005 (the prefetching form with and
without wave items) forced."""
import functools

import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import ops
from oracle import oracle
from helpers import DTYPES, assert_bitwise, oracle_spmm, random_csr, random_dense, to_oracle

pytestmark = pytest.mark.gpu

K_PREFETCH_NNZ = 3 << 20
M = 100_000
SIDES = {"below": K_PREFETCH_NNZ - 5_000, "above": K_PREFETCH_NNZ + 5_000}
CASES = [("f32", 1), ("f32", 8), ("f32", 25), ("f32", 64), ("f32", 128), ("bf16", 8),
         ("bf16", 16), ("bf16", 32), ("bf16", 41), ("bf16", 64), ("f16", 8), ("f16", 16),
         ("f16", 24), ("f16", 63), ("f16", 64)]


@functools.lru_cache(maxsize=4)
def _graph(side: str, idx: torch.dtype):
    """A power-law CSR of M rows with the side's nonzeros (hubs included: split rows)."""
    return fs.synth.csr(M, M, SIDES[side], idx_dtype=idx, val_dtype=torch.float32)


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("dtype,n", CASES)
@pytest.mark.parametrize("side", ["below", "above"])
def test_prefetch_form_threshold(device, side, dtype, n, idx):
    dt = DTYPES[dtype]
    rp, ci, v32 = _graph(side, idx)
    v = v32.to(dt)
    nnz = ci.numel()
    d_form = ops.describe(M, M, n, nnz, dt, idx)
    # below kPrefetchNnz: the narrow shapes for 8 / 16 columns and, round 5, launch_mid_width_pf
    # for every other width up to 128 (fp32) / 256 (16-bit) columns
    narrow_below = n <= (128 if dtype == "f32" else 256)
    assert d_form["form"] == (("narrow" if narrow_below else "prefetch") if side == "below" else
                              ("narrow" if (dtype, n) == ("f32", 16) else "bandwidth")), d_form
    rng = np.random.default_rng(7000 + n)
    b = random_dense(M, n, rng, dt)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], M, M, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{side} {dtype} n={n} auto ({d_form['form']})")
    kern = ops.SpmmCsrKernel(M, M, n, nnz, idx, dt, device)
    sub = torch.full((60_000, n), float("nan"), dtype=dt, device=device)
    kern(*d, sub, row_begin=20_000, row_end=80_000)
    torch.cuda.synchronize()
    assert_bitwise(sub, ref[20_000:80_000], "row range")
    kern.plan(d[0], 0, M)
    o2 = torch.full((M, n), float("nan"), dtype=dt, device=device)
    kern(*d, o2, 0, M, planned=True)
    torch.cuda.synchronize()
    assert_bitwise(o2, ref, "planned")
    bias = random_dense(1, n, rng, dt)[0]
    o3 = torch.full((M, n), float("nan"), dtype=dt, device=device)
    kern(*d, o3, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(o3, oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype), "epilogue")
    for variant in (30004, 30005):
        o = ops.spmm_csr_device(*d, M, M, options=ops.make_options(variant=variant))
        torch.cuda.synchronize()
        assert torch.equal(o.view(torch.uint8), out.view(torch.uint8)), f"variant {variant}"


@pytest.mark.parametrize("dtype,n", [("f32", 16), ("f32", 64), ("bf16", 16), ("bf16", 41)])
def test_plan_reused_workspace(device, dtype, n):
    """The one-launch planner (round 4) writes its look-back status words (epoch-tagged), the work
    list and the in-kernel hub reduce's arrival counters into a workspace that is never zeroed.
    One workspace serves three different graphs of the same shape in turn, then the first again:
    every output bit-exact against the oracle, so no launch reads another launch's status words,
    counters or list.  Graph 2 has no row above the heavy threshold and no hub (wave items with
    nothing to do), graph 3 many hubs (their arrival counters reset by the last chunk)."""
    dt = DTYPES[dtype]
    m = k = 60_000
    rng = np.random.default_rng(4400 + n)
    graphs = []
    for kind in ("power", "flat", "hubs"):
        if kind == "power":
            rp, ci, v = fs.synth.csr(m, k, 1_200_000, val_dtype=torch.float32)
        else:
            deg = np.full(m, 8) if kind == "flat" else rng.integers(0, 12, size=m)
            if kind == "hubs":
                deg[rng.choice(m, size=300, replace=False)] = 2_000
            rp, ci, v = random_csr(m, k, deg, rng, torch.int32, torch.float32)
        graphs.append((rp, ci, v.to(dt)))
    b = random_dense(k, n, rng, dt)
    d_b = b.to(device)
    kerns = [ops.SpmmCsrKernel(m, k, n, g[1].numel(), torch.int32, dt, device) for g in graphs]
    shared = torch.empty(max(kk.ws_bytes for kk in kerns), dtype=torch.uint8, device=device)
    for kk in kerns:  # one workspace for every launch
        kk.workspace = shared
    for gi in (0, 1, 2, 0):
        rp, ci, v = graphs[gi]
        assert ops.describe(m, k, n, ci.numel(), dt)["LR"] == 1
        out = torch.full((m, n), float("nan"), dtype=dt, device=device)
        kerns[gi](rp.to(device), ci.to(device), v.to(device), d_b, out)
        torch.cuda.synchronize()
        assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"graph {gi} {dtype} n={n}")
