"""GPU parity on the committed golden fixtures and on the BASELINE.json configurations at full size.

- every tests/golden/*.npz through the HIP path (op layer -> C-ABI -> kernels): exact-mode cases
  equal the fixture's fp64 product bit for bit, fp32 cases lie within 1e-5 of it relative to the
  |.|-sum, and all of them equal the oracle's schedule bit for bit;
- the partition fixture (BalancedSplitter ranges, rebased row slices, padded remaps) through
  the device kernels;
- Reddit-shaped (232,965^2, 114.6M nnz, N=256 bf16): the whole output against the oracle, bit
  for bit, and sampled rows within 2^-8 |.|-sum of C64 (SURVEY.md §8c bf16 rule) for the result
  and for the reference order; then the 4-rank row split (all ranks on this GPU, gloo carrying
  the exchanged bytes) with every rank's rows compared;
- papers100M-scale (111M rows, 1.6B nnz, N=128 fp32) on one GPU: sampled rows including the
  maximum-degree row, bit-exact and within 1e-5 of C64.

Reference anchors: the semantics restate gather_kernel_util.cpp:72-92 and
unsorted_segment_sum_kernel_util.cpp:29-45; 16-bit accumulation in fp32 as
unsorted_segment_sum_kernel.cpp:146-205.
"""
import glob
import json
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oneflow_spmm as fs
from oneflow_spmm import ops, synth
from oracle import oracle
from tests.helpers import assert_bitwise, check_sampled_rows, oracle_spmm, to_oracle

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# ref_*.npz hold the reference's own vectors, checked by test_reference_fixtures.py
SPMM_FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz"))
                       if not os.path.basename(p).startswith(("fused", "ref_")))
FUSED_FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "fused*.npz")))
BF16_RTOL = 2.0 ** -8


def _log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("name", SPMM_FIXTURES)
def test_golden_fixture_on_gpu(device, name, idx):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    m, k = int(z["m"]), int(z["k"])
    rp = torch.from_numpy(z["row_ptr"]).to(idx)
    ci = torch.from_numpy(z["col_idx"]).to(idx)
    v, b = torch.from_numpy(z["values"]), torch.from_numpy(z["b"])
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ok, worst = oracle.within_tolerance(got, z["expected_f64"], z["absum"], 1e-5)
    assert ok, f"{name}: worst {worst:.3e} relative to the |.|-sum"
    if "exact" in name:  # every summation order gives the same bits
        np.testing.assert_array_equal(got, z["expected_f64"].astype(np.float32))
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"{name} vs the oracle's schedule")
    # the pure reference order through the `ordered` option, bit for bit
    out_o = ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                                options=ops.make_options(ordered=True))
    torch.cuda.synchronize()
    assert_bitwise(out_o, oracle_spmm(rp, ci, v, b, ordered=True), f"{name} ordered")


@pytest.mark.parametrize("name", FUSED_FIXTURES)
def test_golden_fused_fixture_on_gpu(device, name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    m, k = int(z["m"]), int(z["k"])
    rp, ci = torch.from_numpy(z["row_ptr"]), torch.from_numpy(z["col_idx"])
    v, b, bias = (torch.from_numpy(z[x]) for x in ("values", "b", "bias"))
    out = fs._C.fused_spmm_csr(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device),
                               bias.to(device), relu=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    # relu is 1-Lipschitz and the bias add rounds once: the spmm tolerance plus one rounding
    bound_abs = z["absum"] + np.abs(z["bias"].astype(np.float64))[None, :]
    ok, worst = oracle.within_tolerance(got, z["expected_relu_f64"], bound_abs, 1e-5)
    assert ok, f"{name}: worst {worst:.3e}"
    if "exact" in name:
        np.testing.assert_array_equal(got, z["expected_relu_f64"].astype(np.float32))
    ref = oracle.bias_act(oracle_spmm(rp, ci, v, b), z["bias"], "relu")
    assert_bitwise(out, ref, f"{name} vs the oracle's composition")


def test_partition_fixture_on_gpu(device):
    part = json.load(open(os.path.join(GOLD, "partition.json")))
    for idx in (torch.int32, torch.int64):
        rp = torch.tensor(part["row_ptr"], dtype=idx, device=device)
        for key, sl in part["slices"].items():
            lo, hi = sl["rows"]
            out, _, _ = ops.csr_row_slice(rp, lo, hi)
            torch.cuda.synchronize()
            assert out.cpu().tolist() == sl["row_ptr"], key
    from oneflow_spmm.distributed import RowSplitSpmm
    k = part["k"]
    for g, expect in part["padded_remap"].items():
        for idx in (torch.int32, torch.int64):
            col = torch.arange(k, dtype=idx, device=device)
            got = torch.empty_like(col)
            fs._lib.check(fs._lib.LIB.ofx_padded_owner_remap(
                fs._C.current_stream_handle(col), fs._C.dtype_code(idx), k, k, int(g),
                col.data_ptr(), got.data_ptr()), "remap")
            torch.cuda.synchronize()
            assert got.cpu().tolist() == expect, (g, idx)
    del RowSplitSpmm


# ---- Reddit-shaped, N=256 bf16 --------------------------------------------------------------

def _reddit_host():
    cfg = synth.CONFIGS["reddit"]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    rp = synth.row_ptr(m, k, nnz)
    cols = synth.columns(m, k, rp, threads=16)
    vals = synth.values(0, nnz, dt)
    return cfg, rp, cols, vals


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_reddit_full_size_bf16(device):
    cfg, rp, cols, vals = _reddit_host()
    m, k, n, dt = cfg["m"], cfg["k"], cfg["n"], cfg["dtype"]
    _log("reddit: inputs generated")
    d_b = synth.dense(0, k, n, dt, device=device)
    out = fs.spmm(torch.from_numpy(rp.astype(np.int32)).to(device), torch.from_numpy(cols).to(device),
                  vals.to(device), m, k, d_b)
    torch.cuda.synchronize()
    _log("reddit: GPU done; full oracle")
    deg = np.diff(rp)
    split = ops.default_split(n)
    hubs = np.nonzero(deg > split)[0]
    assert len(hubs) > 100_000 and deg.max() == k  # hub rows dominate; one row is dense
    # every row, bit for bit, against the oracle's schedule (full B on the host: 119 MB)
    ref = oracle.spmm(rp, cols, to_oracle(vals), to_oracle(d_b), dtype="bf16", nthreads=16)
    assert_bitwise(out, ref, "reddit: all rows")
    del ref
    _log("reddit: all rows bit-exact; C64 tolerance on sampled rows")
    heavy = np.argsort(deg)[-500:]
    rows = np.unique(np.concatenate([heavy, hubs[::200], np.arange(100_000, 102_000)]))
    check_sampled_rows(rp, cols, vals, d_b, out, rows, BF16_RTOL, "reddit")


def _reddit_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "of-spmm_amd")):
        sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import synth as sy
        from oneflow_spmm.distributed import RowSplitSpmm
        from oracle import oracle as orc
        from tests.helpers import to_oracle as to_o

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        cfg = sy.CONFIGS["reddit"]
        m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
        lo, hi = orc.balanced_range(m, world, rank)
        lrp, lci, lv = sy.csr(m, k, nnz, val_dtype=dt, row_begin=lo, row_end=hi, rebase=True,
                              threads=4)
        rs = RowSplitSpmm(m, k, n, lci.numel(), dt, torch.int32, dev, comm="torch")
        assert rs.row_range == (lo, hi)
        klo, khi = rs.k_range
        rs.load_shard(sy.dense(klo, khi, n, dt, device=dev))
        d_rp, d_ci, d_v = lrp.to(dev), lci.to(dev), lv.to(dev)
        ref = orc.spmm(lrp.numpy(), lci.numpy(), to_o(lv), to_o(sy.dense(0, k, n, dt)),
                       dtype="bf16", nthreads=4)
        same = lambda o: np.array_equal(to_o(o).view(np.uint8), ref.view(np.uint8))  # noqa: E731
        res = {}
        out = rs(d_rp, rs.remap_columns(d_ci), d_v)  # padded in-place all-gather + local SpMM
        torch.cuda.synchronize()
        res["allgather"] = same(out)
        rs.set_pipeline(2)  # two column blocks, gathered on the side stream
        out.fill_(float("nan"))
        rs(d_rp, rs.remap_columns(d_ci), d_v, out=out)
        torch.cuda.synchronize()
        res["allgather/p2"] = same(out)
        rs.set_pipeline(1)
        rs.bind(d_rp, d_ci, d_v, halo=True)
        rs.exchange = "halo"
        out.fill_(float("nan"))
        rs.step(out)
        torch.cuda.synchronize()
        res["halo"] = same(out)
        q.put((rank, res, (lo, hi), lci.numel()))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_reddit_four_rank_row_split_device_path(device):
    """BASELINE configs[3]'s layout: 4 ranks, each with its BalancedSplitter rows of the Reddit
    CSR and its B shard; the padded all-gather (one and two column blocks) and the halo exchange
    run their device kernels on this GPU with gloo moving the bytes (RCCL refuses two ranks on one
    GPU); every rank's rows equal the oracle's bit for bit."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_reddit_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=540) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1]["error"] for r in res if "error" in r[1]]
    assert not errs, errs[0]
    cfg = synth.CONFIGS["reddit"]
    assert sorted(r[2] for r in res) == [oracle.balanced_range(cfg["m"], world, i) for i in range(world)]
    assert sum(r[3] for r in res) == cfg["nnz"]
    for rank, ok, _, _ in res:
        assert all(ok.values()), (rank, ok)


# ---- papers100M-scale, N=128 fp32, one GPU ---------------------------------------------------

@pytest.mark.slow
@pytest.mark.timeout(900)
def test_papers_scale_sampled_rows(device):
    cfg = synth.CONFIGS["papers"]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    free, _ = torch.cuda.mem_get_info(device)
    need = 4 * (m + 1) + 8 * nnz + 2 * 4 * m * n
    if free < need * 1.05:
        pytest.skip(f"needs {need / 2**30:.0f} GiB of device memory, {free / 2**30:.0f} free")
    t0 = time.time()
    rp = synth.row_ptr(m, k, nnz)
    cols = synth.columns(m, k, rp, threads=16)
    vals = synth.values(0, nnz, dt)
    _log(f"papers: host inputs in {time.time() - t0:.0f} s")
    d_rp = torch.from_numpy(rp.astype(np.int32)).to(device)
    d_ci = torch.from_numpy(cols).to(device)
    d_v = vals.to(device)
    d_b = synth.dense(0, k, n, dt, device=device)
    out = torch.empty((m, n), dtype=dt, device=device)
    fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out)
    torch.cuda.synchronize()
    _log(f"papers: GPU done at {time.time() - t0:.0f} s; sampled rows")
    del d_rp, d_ci, d_v
    deg = np.diff(rp)
    split = ops.default_split(n)
    heavy = np.argsort(deg)[-20:]
    assert deg[heavy[-1]] == deg.max() and deg.max() > 1_000_000
    hubs = np.nonzero(deg > split)[0]
    rows = np.unique(np.concatenate([
        np.arange(0, 2000), np.arange(m // 2, m // 2 + 2000), np.arange(m - 2000, m), heavy,
        hubs[:: max(len(hubs) // 200, 1)]]))
    check_sampled_rows(rp, cols, vals, d_b, out, rows, 1e-5, "papers")
    # size-independent property over every row: no NaN/Inf, rows with no nonzeros are +0
    empty = torch.from_numpy(np.nonzero(deg == 0)[0][:100_000]).to(device)
    assert torch.isfinite(out).all()
    if empty.numel():
        assert not out.index_select(0, empty).abs().sum().item()
    _log(f"papers: done at {time.time() - t0:.0f} s")
