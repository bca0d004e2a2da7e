"""GPU parity: the HIP kernel (through the C-ABI and through the op layer) against the oracle.

Bar: bit-exact against the oracle run with the operator's schedule for every
dtype; bit-exact against the pure reference order (gather -> multiply -> segment_sum) whenever
no row is split or with `ordered`; within 1e-5 of the fp64 product relative to the |.|-sum for
fp32 with hub rows split (BASELINE.json: "within 1e-5 rel on fp32 values").
"""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import ops
from oracle import oracle
from tests.helpers import (DTYPES, assert_bitwise, check_sampled_rows, oracle_spmm,
                           power_law_degrees, random_csr, random_dense, to_oracle)

pytestmark = pytest.mark.gpu


def _dev(t, device):
    return t.to(device)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("n", [1, 3, 16, 17, 64, 128, 256])
def test_dtype_width_sweep(device, dtype, idx, n):
    rng = np.random.default_rng(1000 + n)
    m, k = 300, 257
    deg = rng.integers(0, 40, size=m)
    deg[5] = 0
    deg[7] = 250  # long row
    rp, ci, v = random_csr(m, k, deg, rng, idx, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device))
    torch.cuda.synchronize()
    assert out.dtype == DTYPES[dtype] and out.shape == (m, n)
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"{dtype}/{idx}/n={n}")


@pytest.mark.parametrize("variant", [104, 108, 116, 132, 164, 204, 232, 264, 404, 432, 464])
def test_forced_variants_bitexact(device, variant):
    rng = np.random.default_rng(variant)
    m, k, n = 500, 400, 128
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 12000, k, rng), rng)
    b = random_dense(k, n, rng)
    opts = ops.make_options(variant=variant)
    out = ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                              options=opts)
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"variant {variant}")


# The tuning table is an A/B build's (make -C of-spmm_amd tuning): its tests
# run when OFX_SPMM_LIB selects that library and skip on the release one.
needs_tuning_table = pytest.mark.skipif(not fs.__version__.endswith("+tuning"),
                                        reason="release library: no tuning table (make tuning)")


@needs_tuning_table
@pytest.mark.parametrize("n", [16, 128])
@pytest.mark.parametrize("tuned", list(range(1, 18)) + list(range(21, 45)))
def test_tuning_table_bitexact(device, tuned, n):
    """Every entry of the tuning table (variant 10000 + id, spmm_csr.hip launch_tuned) computes
    the contract's bits: only the launch shape and loads in flight differ."""
    rng = np.random.default_rng(1000 + tuned)
    m, k = 700, 600
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 20000, k, rng), rng)
    b = random_dense(k, n, rng)
    out = ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                              options=ops.make_options(variant=10000 + tuned))
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"tuning variant {tuned} n={n}")


@pytest.mark.parametrize("n", [16, 64, 128, 256])
def test_hub_rows_split_bitexact_and_tolerance(device, n):
    rng = np.random.default_rng(7 + n)
    m, k = 64, 60000
    deg = rng.integers(1, 100, size=m)
    deg[3] = 50000  # hub row, far above the split threshold
    deg[40] = ops.default_split(n) + 1  # just above
    deg[41] = ops.default_split(n)  # just at (not split)
    deg[42] = 2 * ops.default_split(n) + 7
    rp, ci, v = random_csr(m, k, deg, rng)
    b = random_dense(k, n, rng)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device))
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), "split schedule")
    c64, absum = oracle.ref64(to_oracle(rp), to_oracle(ci), to_oracle(v), to_oracle(b))
    ok, worst = oracle.within_tolerance(to_oracle(out), c64, absum, 1e-5)
    assert ok, worst
    ref_order = oracle_spmm(rp, ci, v, b, ordered=True)
    ok, worst = oracle.within_tolerance(ref_order, c64, absum, 1e-5)
    assert ok, worst
    # ordered option: the pure reference order, bit for bit
    out2 = ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                               options=ops.make_options(ordered=True))
    torch.cuda.synchronize()
    assert_bitwise(out2, ref_order, "ordered")


def test_custom_split_and_chunk(device):
    rng = np.random.default_rng(3)
    m, k, n = 40, 5000, 64
    deg = rng.integers(0, 300, size=m)
    deg[0] = 4000
    rp, ci, v = random_csr(m, k, deg, rng)
    b = random_dense(k, n, rng)
    for split, chunk in [(128, 128), (256, 100), (1000, 333), (64, 1)]:
        opts = ops.make_options(split=split, chunk=chunk)
        out = ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                                  options=opts)
        torch.cuda.synchronize()
        assert_bitwise(out, oracle_spmm(rp, ci, v, b, split=split, chunk=chunk), f"{split}/{chunk}")


def test_exact_mode_matches_any_order(device):
    rng = np.random.default_rng(11)
    m, k, n = 200, 3000, 128
    deg = rng.integers(0, 60, size=m)
    deg[9] = 2900
    rp, ci, v = random_csr(m, k, deg, rng, exact=True)
    b = random_dense(k, n, rng, exact=True)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device))
    torch.cuda.synchronize()
    ref = oracle_spmm(rp, ci, v, b, ordered=True)
    assert_bitwise(out, ref, "exact mode")
    import scipy.sparse as sp
    a = sp.csr_matrix((to_oracle(v).astype(np.float64), to_oracle(ci), to_oracle(rp)), shape=(m, k))
    np.testing.assert_array_equal(a @ to_oracle(b).astype(np.float64), to_oracle(out))


def test_edge_cases(device):
    rng = np.random.default_rng(5)
    # M == 0
    rp = torch.zeros(1, dtype=torch.int32)
    out = fs.spmm(rp.to(device), torch.zeros(0, dtype=torch.int32, device=device),
                  torch.zeros(0, device=device), 0, 10, torch.ones(10, 8, device=device))
    assert out.shape == (0, 8)
    # nnz == 0: zeros
    rp = torch.zeros(6, dtype=torch.int32)
    out = fs.spmm(rp.to(device), torch.zeros(0, dtype=torch.int32, device=device),
                  torch.zeros(0, device=device), 5, 10, torch.ones(10, 8, device=device))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), torch.zeros(5, 8))
    # N == 0
    rp, ci, v = random_csr(7, 9, rng.integers(0, 5, size=7), rng)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), 7, 9, torch.ones(9, 0, device=device))
    assert out.shape == (7, 0)
    # K != M, every row empty but one
    deg = np.zeros(50, dtype=np.int64)
    deg[49] = 33
    rp, ci, v = random_csr(50, 1000, deg, rng)
    b = random_dense(1000, 64, rng)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), 50, 1000, b.to(device))
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), "one nonempty row")


def test_unaligned_and_strided_views(device):
    rng = np.random.default_rng(9)
    m, k, n = 120, 200, 64
    rp, ci, v = random_csr(m, k, rng.integers(0, 30, size=m), rng)
    b = random_dense(k, n, rng)
    big = torch.zeros(k * n + 1, dtype=torch.float32)
    big[1:] = b.reshape(-1)
    b_unaligned = big.to(device)[1:].view(k, n)  # 4-B aligned only -> VEC=1 path
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b_unaligned)
    torch.cuda.synchronize()
    ref = oracle_spmm(rp, ci, v, b)
    assert_bitwise(out, ref, "unaligned b")
    wide = torch.zeros(k, n + 36, dtype=torch.float32)
    wide[:, 4:4 + n] = b
    b_strided = wide.to(device)[:, 4:4 + n]  # ldb = n + 36, 16-B aligned
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b_strided)
    torch.cuda.synchronize()
    assert_bitwise(out, ref, "strided b")
    # output with ldc > n through the C-ABI
    c_wide = torch.full((m, n + 12), 7.0, device=device)
    ops.spmm_csr_device(rp.to(device), ci.to(device), v.to(device), b.to(device), m, k,
                        out=c_wide[:, :n])
    torch.cuda.synchronize()
    assert_bitwise(c_wide[:, :n], ref, "strided c")
    assert torch.all(c_wide[:, n:] == 7.0)


def test_row_range_and_global_form(device):
    rng = np.random.default_rng(21)
    m, k, n = 1001, 700, 32
    rp, ci, v = random_csr(m, k, rng.integers(0, 50, size=m), rng)
    b = random_dense(k, n, rng)
    full = oracle_spmm(rp, ci, v, b)
    for parts in (2, 3, 8):
        for pid in range(parts):
            lo, hi = oracle.balanced_range(m, parts, pid)
            out = fs._C.spmm_csr(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device),
                                 _parallel=(pid, parts, 0))
            torch.cuda.synchronize()
            assert out.shape == (hi - lo, n)
            assert_bitwise(out, full[lo:hi], f"rank {pid}/{parts}")


def test_determinism_and_validate(device):
    rng = np.random.default_rng(4)
    m, k, n = 3000, 3000, 128
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 90000, k, rng), rng)
    b = random_dense(k, n, rng).to(device)
    rp, ci, v = rp.to(device), ci.to(device), v.to(device)
    o1 = fs.spmm(rp, ci, v, m, k, b)
    o2 = fs.spmm(rp, ci, v, m, k, b)
    torch.cuda.synchronize()
    assert torch.equal(o1.view(torch.int32), o2.view(torch.int32))
    assert ops.validate_csr(rp, ci, m, k) == 0
    bad = ci.clone()
    bad[10] = k
    assert ops.validate_csr(rp, bad, m, k) == 2
    badrp = rp.clone()
    badrp[5] = badrp[6] + 1
    assert ops.validate_csr(badrp, ci, m, k) == 1


def test_op_errors_on_device(device):
    rp = torch.zeros(6, dtype=torch.int32, device=device)
    ci = torch.zeros(0, dtype=torch.int32, device=device)
    with pytest.raises(RuntimeError, match="a_num_rows"):
        fs.spmm(rp, ci, torch.zeros(0, device=device), 4, 10, torch.ones(10, 8, device=device))
    with pytest.raises(TypeError):
        fs.spmm(rp, ci, torch.zeros(0, device=device, dtype=torch.float64), 5, 10,
                torch.ones(10, 8, device=device))
    with pytest.raises(RuntimeError, match="same device"):
        fs.spmm(rp, ci, torch.zeros(0, device=device), 5, 10, torch.ones(10, 8))


def test_synth_dense_device_matches_host(device):
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
        h = fs.synth.dense(100, 250, 40, dt)
        d = fs.synth.dense(100, 250, 40, dt, device=device)
        torch.cuda.synchronize()
        assert torch.equal(h.view(-1).view(torch.uint8), d.cpu().view(-1).view(torch.uint8))


@pytest.mark.parametrize("name", ["cora", "plaw1m"])
def test_baseline_configs_bitexact(device, name):
    cfg = fs.synth.CONFIGS[name]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    rp, ci, v = fs.synth.csr(m, k, nnz, val_dtype=dt)
    b = fs.synth.dense(0, k, n, dt)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b.to(device))
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), name)
    c64, absum = oracle.ref64(to_oracle(rp), to_oracle(ci), to_oracle(v), to_oracle(b))
    ok, worst = oracle.within_tolerance(to_oracle(out), c64, absum, 1e-5)
    assert ok, worst


@pytest.mark.parametrize("n,alt_variant", [(16, 116), (32, 408)])
def test_plaw1m_narrow_widths_bitexact(device, n, alt_variant):
    """1M power-law (20M nonzeros) at N=16 / 32, the whole output bit for bit against the oracle
    and against a second configuration of the same width.  The automatic picks: at N=16 the narrow
    form past kPrefetchNnz (2-lane float2 light rows, 16-lane wave items for the hub chunks and
    heavy rows), against VEC 1 / LPR 16 forced (variant 116: one element per lane over 16
    lanes); at N=32 the bandwidth configuration, against VEC 4 / LPR 8 forced (variant 408)."""
    cfg = fs.synth.CONFIGS["plaw1m"]
    m, k, nnz = cfg["m"], cfg["k"], cfg["nnz"]
    rp, ci, v = fs.synth.csr(m, k, nnz)
    b = fs.synth.dense(0, k, n)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    out = fs.spmm(*d[:3], m, k, d[3])
    alt = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=alt_variant))
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), alt.view(torch.int32))
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), f"plaw1m n={n}")


def test_mid_size_n16_narrow_form_bitexact(device):
    """A 15M-nonzero power-law graph (750k rows) at N=16: the narrow form past kPrefetchNnz
    (2-lane float2 light rows, hub chunks and heavy rows as 16-lane wave items); the output bit for
    bit against the oracle, the one-element bandwidth configuration (VEC 1 / LPR 16 forced,
    variant 116) and the mid form forced (variant 30002, block items)."""
    m = k = 750_000
    nnz, n = 15_000_000, 16
    rp, ci, v = fs.synth.csr(m, k, nnz)
    b = fs.synth.dense(0, k, n)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    out = fs.spmm(*d[:3], m, k, d[3])
    for variant in (116, 30002):
        alt = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=variant))
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), alt.view(torch.int32)), variant
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), "15M n=16")


@pytest.mark.slow
def test_products_scale_sampled_rows(device):
    """ogbn-products-shaped (2.45M rows, 123.7M nnz, N=128): every hub row and a contiguous
    block of ordinary rows against the oracle, bit for bit."""
    cfg = fs.synth.CONFIGS["products"]
    m, k, nnz, n = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"]
    rp, ci, v = fs.synth.csr(m, k, nnz)
    b = fs.synth.dense(0, k, n, device=device)
    out = fs.spmm(rp.to(device), ci.to(device), v.to(device), m, k, b)
    torch.cuda.synchronize()
    b_h = b.cpu()
    rp_n, ci_n, v_n, b_n = to_oracle(rp), to_oracle(ci), to_oracle(v), to_oracle(b_h)
    # the oracle takes int64 indices: convert once, not per call
    rp_n, ci_n = rp_n.astype(np.int64), ci_n.astype(np.int64)
    deg = np.diff(rp_n)
    hubs = np.nonzero(deg > ops.default_split(n))[0]
    assert len(hubs) > 100
    out_h = out.cpu()
    for r in list(hubs[:200]) + [hubs[-1]]:
        ref = oracle.spmm(rp_n, ci_n, v_n, b_n, row_begin=int(r), row_end=int(r) + 1)
        assert_bitwise(out_h[r:r + 1], ref, f"hub row {r}")
    ref = oracle.spmm(rp_n, ci_n, v_n, b_n, row_begin=1_000_000, row_end=1_100_000)
    assert_bitwise(out_h[1_000_000:1_100_000], ref, "row block")
    # BASELINE's "within 1e-5 rel" on the split hub rows (and the reference order on the same
    # rows), relative to the |.|-sum: the 200 first hubs, the 20 heaviest (max degree 306k), the last
    heavy = np.argsort(deg)[-20:]
    rows = np.unique(np.concatenate([hubs[:200], heavy, hubs[-1:]]))
    check_sampled_rows(rp_n, ci_n, v, b, out, rows, 1e-5, "products hubs")
    # every row, through linearity (size-independent): the row checksums C.1 against A.(B.1) taken
    # in float64 on the host (scipy), each within 1e-5 of its row's |A|.(|B|.1); then the checksum
    # of those checksums, 1'.C.1 against 1'.A.(B.1), within 1e-5 of 1'.|A|.(|B|.1)
    import scipy.sparse as sp
    assert torch.isfinite(out_h).all()
    a64 = sp.csr_matrix((v_n.astype(np.float64), ci_n, rp_n), shape=(m, k))
    b64 = b_n.astype(np.float64)
    want = a64 @ b64.sum(axis=1)
    scale = abs(a64) @ np.abs(b64).sum(axis=1)
    got = out.double().sum(dim=1).cpu().numpy()
    err = np.abs(got - want)
    bad = np.nonzero(err > 1e-5 * np.maximum(scale, 1e-30))[0]
    assert len(bad) == 0, f"{len(bad)} rows off, first {bad[:5]}, worst {float(np.max(err / np.maximum(scale, 1e-30)))}"
    assert abs(got.sum() - want.sum()) <= 1e-5 * scale.sum()


def test_row_split_rccl_single_rank(device):
    """The RCCL C-ABI path (unique id -> comm init -> in-place ncclAllGather -> local SpMM) with one
    rank; multi-rank semantics are covered by tests/test_distributed_gloo.py."""
    import socket

    import torch.distributed as dist
    from oneflow_spmm.distributed import RowSplitSpmm

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=device)
    try:
        rng = np.random.default_rng(17)
        m, k, n = 777, 3555, 128
        rp, ci, v = random_csr(m, k, power_law_degrees(m, 60000, k, rng), rng)
        b = random_dense(k, n, rng)
        rs = RowSplitSpmm(m, k, n, ci.numel(), torch.float32, torch.int32, device)
        assert rs.comm_kind == "rccl"
        rs.shard_view().copy_(b.to(device))
        out = rs(rp.to(device), rs.remap_columns(ci.to(device)), v.to(device))
        torch.cuda.synchronize()
        assert_bitwise(out, oracle_spmm(rp, ci, v, b), "rccl row split")
        # column-block pipeline on the side stream (ring, point-to-point and pull schedules; one
        # rank's pull has no peer to read, its barriers and buffer mapping still run)
        for kind, chunks in (("rccl", 4), ("rccl-p2p", 2), ("rccl-pull", 2)):
            rs.comm_kind = kind
            rs.set_pipeline(chunks)
            out2 = torch.full_like(out, float("nan"))
            for _ in range(3):  # back-to-back steps: stream ordering between them
                rs(rp.to(device), rs.remap_columns(ci.to(device)), v.to(device), out=out2)
            torch.cuda.synchronize()
            assert_bitwise(out2, oracle_spmm(rp, ci, v, b), f"{kind} pipeline {chunks}")
            # load_shard into the column-block layout (one copy_blocks launch) from a strided shard
            b_new = random_dense(k, n + 3, rng)
            rs.load_shard(b_new.to(device)[:, :n])
            rs(rp.to(device), rs.remap_columns(ci.to(device)), v.to(device), out=out2)
            torch.cuda.synchronize()
            assert_bitwise(out2, oracle_spmm(rp, ci, v, b_new[:, :n].contiguous()), f"{kind} load_shard")
            rs.load_shard(b.to(device))
        # the setup-time choice runs every candidate step and keeps one; output stays exact
        d = (rp.to(device), ci.to(device), v.to(device))
        rs.bind(*d, halo=True, full_csr=d, grid_subs=(1, 4))
        assert rs.halo.halo_rows == 0 and rs.halo.k_compact == k  # one rank owns every row
        # the IPC pull is opt-in: absent from the default kinds, measured when named
        times = rs.tune(out2, reps=1, force=True)
        assert len(times) == 11 and not any(t.startswith("rccl-pull") for t in times)
        times = rs.tune(out2, reps=1, force=True, kinds=("rccl", "rccl-p2p", "rccl-pull"))
        assert len(times) == 14 and "rccl-pull/p4" in times and "halo" in times and "nsplit" in times and "nsplit/s4" in times
        assert "halo/p2" in times and "halo/p4" in times
        for exchange in ("allgather", "halo", "halo/p4", "nsplit", "nsplit/s4"):
            rs.exchange = exchange.split("/p")[0]
            if rs.exchange == "halo":  # column blocks of the halo exchange on the side stream
                rs.set_halo_pipeline(int(exchange.split("/p")[1]) if "/p" in exchange else 1)
            out2.fill_(float("nan"))
            for _ in range(2):
                rs.step(out2)
            torch.cuda.synchronize()
            assert_bitwise(out2, oracle_spmm(rp, ci, v, b), f"after tune, {exchange}")
        rs.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16"])
@pytest.mark.parametrize("n", [3, 64, 256])
@pytest.mark.parametrize("epi", [False, True])
def test_deep_and_shallow_hub_reduce(device, dtype, n, epi):
    """Both hub-reduce kernels: shallow hubs (<= 64 chunks: 16-B vectors, many hubs per wave)
    and deep hubs (> 64 chunks: one lane per column, 64 partials in flight, LDS-compacted hub
    list), with the fused bias + relu epilogue, 16-B and scalar partial rows (n = 3)."""
    rng = np.random.default_rng(70 + n)
    split = ops.default_split(n)
    m, k = 700, max(4096, 160 * split)
    deg = rng.integers(0, 20, size=m)
    deg[[3, 100, 650]] = [150 * split + 7, 65 * split, 64 * split + split - 1]  # deep x2, shallow
    deg[200:260] = rng.integers(split + 1, 5 * split, size=60)  # many shallow hubs
    deg = np.minimum(deg, k)
    rp, ci, v = random_csr(m, k, deg, rng, torch.int32, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    bias = random_dense(1, n, rng, DTYPES[dtype])[0] if epi else None
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), torch.int32, DTYPES[dtype], device)
    out = torch.full((m, n), float("nan"), dtype=DTYPES[dtype], device=device)
    kern(rp.to(device), ci.to(device), v.to(device), b.to(device), out,
         bias=bias.to(device) if epi else None, relu=epi)
    torch.cuda.synchronize()
    ref = oracle_spmm(rp, ci, v, b)
    if epi:
        ref = oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype)
    assert_bitwise(out, ref, f"{dtype} n={n} epilogue={epi}")


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_plan_once_compute_many(device, idx):
    """ofx_spmm_csr_plan builds the work list once; planned launches (hub chunks, degree bins,
    a row range of the full CSR) give the same bits as self-planning ones for new B each time."""
    rng = np.random.default_rng(51)
    m, k, n = 40000, 30000, 64
    deg = power_law_degrees(m, 900000, k, rng)
    rp, ci, v = random_csr(m, k, deg, rng, idx)
    assert int(np.diff(rp.numpy()).max()) > ops.default_split(n)  # hub rows are split
    d_rp, d_ci, d_v = rp.to(device), ci.to(device), v.to(device)
    for rb, re in ((0, m), (1234, 38000)):
        kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), idx, torch.float32, device).plan(d_rp, rb, re)
        for it in range(3):
            b = random_dense(k, n, np.random.default_rng(60 + it))
            out = torch.full((re - rb, n), float("nan"), device=device)
            kern(d_rp, d_ci, d_v, b.to(device), out, rb, re, planned=True)
            torch.cuda.synchronize()
            ref = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy(), row_begin=rb, row_end=re)
            assert_bitwise(out, ref, f"planned launch {it} rows [{rb},{re})")
        with pytest.raises(RuntimeError):  # a planned launch needs a plan of this range
            kern(d_rp, d_ci, d_v, b.to(device), out[:10], 0, 10, planned=True)


@pytest.mark.graph_capture
def test_hipgraph_capture_replay(device):
    """The op launches are capture-safe (no allocation / sync inside): capture into a graph,
    replay on new data, same bits as eager."""
    rng = np.random.default_rng(33)
    m, k, n = 20000, 20000, 128
    deg = power_law_degrees(m, 400000, k, rng)
    rp, ci, v = random_csr(m, k, deg, rng)
    b = random_dense(k, n, rng).to(device)
    rp, ci, v = rp.to(device), ci.to(device), v.to(device)
    out = torch.empty((m, n), device=device)
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), torch.int32, torch.float32, device)
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        kern(rp, ci, v, b, out)  # warm (outside capture)
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        kern(rp, ci, v, b, out)
    b.copy_(random_dense(k, n, np.random.default_rng(34)).to(device))
    g.replay()
    torch.cuda.synchronize()
    ref = oracle_spmm(rp.cpu(), ci.cpu(), v.cpu(), b.cpu())
    assert_bitwise(out, ref, "graph replay")


@pytest.mark.graph_capture
def test_row_split_step_hipgraph_capture(device):
    """The whole row-split step (RCCL exchange + local SpMM; the pipelined form on two streams;
    the halo form) is capture-safe: capture once, load a new B shard, replay, same bits."""
    import socket

    import torch.distributed as dist
    from oneflow_spmm.distributed import RowSplitSpmm

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=device)
    try:
        rng = np.random.default_rng(41)
        m, k, n = 3000, 2500, 128
        rp, ci, v = random_csr(m, k, power_law_degrees(m, 90000, k, rng), rng)
        b1, b2 = random_dense(k, n, rng), random_dense(k, n, rng)
        rs = RowSplitSpmm(m, k, n, ci.numel(), torch.float32, torch.int32, device)
        rs.load_shard(b1.to(device))
        d = (rp.to(device), ci.to(device), v.to(device))
        rs.bind(*d, halo=True, full_csr=d, grid_subs=(1, 2))
        out = torch.empty((m, n), device=device)
        for exchange, chunks in (("allgather", 1), ("allgather", 2), ("halo", 1), ("nsplit", 1),
                                 ("nsplit/s2", 1)):
            rs.exchange = exchange
            rs.set_pipeline(chunks)
            rs.load_shard(b1.to(device))
            side = torch.cuda.Stream(device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                rs.step(out)  # warm, outside the capture
            torch.cuda.current_stream(device).wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                rs.step(out)
            rs.load_shard(b2.to(device))
            out.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize()
            assert_bitwise(out, oracle_spmm(rp, ci, v, b2), f"graph replay {exchange}/p{chunks}")
            del g
        rs.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype,idx", [("f32", torch.int32), ("bf16", torch.int64),
                                       ("f64", torch.int32), ("f16", torch.int32)])
@pytest.mark.parametrize("n", [1, 4, 16, 17, 64, 128])
def test_small_launch_wave_items(device, dtype, idx, n):
    """Small launches (<= 32768 rows): hub chunks and heavy rows (> 5x the mean degree) are taken
    by a whole wave whose groups interleave the nonzeros and add the products in nonzero order
    through cross-lane moves; light rows by one group.  Same bits as the oracle, with and without
    the fused epilogue, and through the gathered-values form."""
    rng = np.random.default_rng(500 + n)
    m, k = 3000, 12000
    deg = rng.integers(0, 12, size=m)
    deg[[7, 70, 700, 2999]] = [300, 2500, 9000, 65]   # heavy rows, a hub at every n here
    deg[100:110] = rng.integers(100, 600, size=10)
    rp, ci, v = random_csr(m, k, deg, rng, idx, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    ref = oracle_spmm(rp, ci, v, b)
    assert_bitwise(out, ref, f"{dtype} n={n}")
    bias = random_dense(1, n, rng, DTYPES[dtype])[0]
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), idx, DTYPES[dtype], device)
    out2 = torch.full((m, n), float("nan"), dtype=DTYPES[dtype], device=device)
    kern(*d, out2, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(out2, oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype), "epilogue")
    perm = torch.from_numpy(rng.permutation(ci.numel()).astype(np.int64)).to(idx)
    vals_src = torch.empty_like(v)
    vals_src[perm.long()] = v  # values[perm[j]] == v[j]
    out3 = ops.spmm_csr_gathered(d[0], d[1], vals_src.to(device), perm.to(device), d[3], m, k)
    torch.cuda.synchronize()
    assert_bitwise(out3, ref, "gathered values")


@pytest.mark.parametrize("dtype,idx", [("f32", torch.int32), ("f32", torch.int64), ("bf16", torch.int32),
                                       ("f16", torch.int64), ("f64", torch.int32)])
@pytest.mark.parametrize("n", [1, 4, 16, 17, 33, 64, 300])
def test_small_form_single_launch(device, dtype, idx, n):
    """Launches of <= 32768 rows and <= 2^20 products (nnz * n) run as one kernel with no plan and
    no workspace: light rows by one lane-group, rows above the light cut by the whole block (LDS
    products added in nonzero order), split rows chunk by chunk with the chunk sums added in chunk
    order.  Same bits as the oracle for every row class, the light-cut boundary, several column
    passes (n = 300), the ordered option, row ranges, the epilogue and gathered values."""
    rng = np.random.default_rng(900 + n)
    budget = (1 << 20) // n
    split = ops.default_split(n)
    m, k = 1500, 9000
    deg = rng.integers(0, 5, size=m)
    light = 32  # the default cut is 2 x the group's loads in flight: 32 or 64 here
    special = [31, 32, 33, 63, 64, 65, 128, 300, split, split + 1, 2 * split + 7, 3 * split]
    for i, d in enumerate(special):
        deg[17 + 97 * i] = min(d, k)
    while deg.sum() > budget:  # keep the launch inside the small form
        big = int(np.argmax(deg))
        deg[big] = max(deg[big] // 2, light + 1)
        if deg.sum() > budget:
            deg[deg < light] = deg[deg < light] // 2
    rp, ci, v = random_csr(m, k, deg, rng, idx, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    nnz = ci.numel()
    assert nnz * n <= (1 << 20)
    assert ops.workspace_size(idx, DTYPES[dtype], m, k, n, nnz) == 0  # the small form
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    ref = oracle_spmm(rp, ci, v, b)
    assert_bitwise(out, ref, f"{dtype} n={n}")
    kern = ops.SpmmCsrKernel(m, k, n, nnz, idx, DTYPES[dtype], device)
    sub = torch.full((700, n), float("nan"), dtype=DTYPES[dtype], device=device)
    kern(*d, sub, row_begin=400, row_end=1100)
    torch.cuda.synchronize()
    assert_bitwise(sub, ref[400:1100], "row range")
    bias = random_dense(1, n, rng, DTYPES[dtype])[0]
    out2 = torch.full((m, n), float("nan"), dtype=DTYPES[dtype], device=device)
    kern(*d, out2, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(out2, oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype), "epilogue")
    opts = ops.make_options(ordered=True)
    out3 = ops.spmm_csr_device(*d, m, k, options=opts)
    torch.cuda.synchronize()
    assert_bitwise(out3, oracle_spmm(rp, ci, v, b, ordered=True), "ordered")
    perm = torch.from_numpy(rng.permutation(nnz).astype(np.int64)).to(idx)
    vals_src = torch.empty_like(v)
    vals_src[perm.long()] = v
    out4 = ops.spmm_csr_gathered(d[0], d[1], vals_src.to(device), perm.to(device), d[3], m, k)
    torch.cuda.synchronize()
    assert_bitwise(out4, ref, "gathered values")
    for cut in (1, 7, 1000):  # the light/whole-block cut moves work, never bits
        out5 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(heavy=cut))
        torch.cuda.synchronize()
        assert_bitwise(out5, ref, f"light cut {cut}")


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("mean_deg", [25, 90])
def test_narrow_form_n16(device, idx, mean_deg):
    """fp32 N = 16 above the mid form (launch_narrow): 4-lane float4 light rows with 16-lane wave
    items up to kPrefetchNnz nonzeros (mean degree 25: 1M), 2-lane float2 ones past it (90: 3.6M).
    Same bits as the oracle for the whole matrix, a row range, a plan built once, heavy cuts, the
    epilogue and gathered values, and as the forced bandwidth configuration."""
    rng = np.random.default_rng(1700 + mean_deg)
    n, m, k = 16, 40_000, 40_000
    split = ops.default_split(n)
    deg = rng.integers(0, 2 * mean_deg, size=m)
    for i, d in enumerate([split, split + 1, 2 * split - 1, 2 * split, 5 * split + 3, 20_000]):
        deg[7 + 5003 * i] = d
    deg[30_000:30_300] = rng.integers(100, 500, size=300)
    rp, ci, v = random_csr(m, k, deg, rng, idx, torch.float32)
    b = random_dense(k, n, rng)
    nnz = ci.numel()
    assert (nnz > (3 << 20)) == (mean_deg == 90)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(*d[:3], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"narrow auto nnz={nnz}")
    kern = ops.SpmmCsrKernel(m, k, n, nnz, idx, torch.float32, device)
    sub = torch.full((20_000, n), float("nan"), device=device)
    kern(*d, sub, row_begin=10_000, row_end=30_000)
    kp = ops.SpmmCsrKernel(m, k, n, nnz, idx, torch.float32, device).plan(d[0], 0, m)
    o2 = torch.full((m, n), float("nan"), device=device)
    kp(*d, o2, 0, m, planned=True)
    torch.cuda.synchronize()
    assert_bitwise(sub, ref[10_000:30_000], "row range")
    assert_bitwise(o2, ref, "planned")
    for cut in (1, 129, 100_000):
        o3 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(heavy=cut))
        torch.cuda.synchronize()
        assert_bitwise(o3, ref, f"heavy cut {cut}")
    big = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=30003))
    torch.cuda.synchronize()
    assert torch.equal(big.view(torch.int32), out.view(torch.int32))
    bias = random_dense(1, n, rng)[0]
    o4 = torch.full((m, n), float("nan"), device=device)
    kern(*d, o4, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(o4, oracle.bias_act(ref, to_oracle(bias), "relu", dtype="f32"), "epilogue")
    perm = torch.from_numpy(rng.permutation(nnz).astype(np.int64)).to(idx)
    vals_src = torch.empty_like(v)
    vals_src[perm.long()] = v
    o5 = ops.spmm_csr_gathered(d[0], d[1], vals_src.to(device), perm.to(device), d[3], m, k)
    torch.cuda.synchronize()
    assert_bitwise(o5, ref, "gathered values")


@pytest.mark.parametrize("dtype,idx", [("f32", torch.int32), ("f32", torch.int64), ("bf16", torch.int32),
                                       ("f16", torch.int64), ("f64", torch.int32)])
@pytest.mark.parametrize("n", [1, 16, 17, 64, 128, 300])
def test_mid_form_block_items(device, dtype, idx, n):
    """Mid-size launches (above the small form, <= 2^28 products): every hub chunk and every row
    above the heavy threshold is taken by a whole block (block_accumulate), the other rows by one
    lane-group, after a plan.  Same bits as the oracle in the automatic choice and in each forced
    form (30000 small, 30001 mid, 30002 mid with prefetching light rows), for row ranges, a plan
    built once, the epilogue, gathered values, the ordered option and any heavy cut."""
    rng = np.random.default_rng(1300 + n)
    split = ops.default_split(n)
    m, k = 5000, 24000
    deg = rng.integers(0, 20, size=m)
    special = [127, 128, 129, 1000, split, split + 1, 2 * split - 1, 2 * split + 7, 3 * split + 5,
               min(9 * split, k)]
    for i, d in enumerate(special):
        deg[11 + 431 * i] = min(d, k)
    deg[4000:4040] = rng.integers(130, 700, size=40)
    rp, ci, v = random_csr(m, k, deg, rng, idx, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    nnz = ci.numel()
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{dtype} n={n} auto (products {nnz * n})")
    for variant in (30000, 30001, 30002):
        opts = ops.make_options(variant=variant)
        o = ops.spmm_csr_device(*d, m, k, options=opts)
        torch.cuda.synchronize()
        assert_bitwise(o, ref, f"form {variant}")
        kern = ops.SpmmCsrKernel(m, k, n, nnz, idx, DTYPES[dtype], device, opts)
        sub = torch.full((3100, n), float("nan"), dtype=DTYPES[dtype], device=device)
        kern(*d, sub, row_begin=900, row_end=4000)
        torch.cuda.synchronize()
        assert_bitwise(sub, ref[900:4000], f"form {variant} row range")
        if variant != 30000:  # a plan built once (the small form has none)
            kp = ops.SpmmCsrKernel(m, k, n, nnz, idx, DTYPES[dtype], device, opts).plan(d[0], 0, m)
            o2 = torch.full((m, n), float("nan"), dtype=DTYPES[dtype], device=device)
            kp(*d, o2, 0, m, planned=True)
            torch.cuda.synchronize()
            assert_bitwise(o2, ref, f"form {variant} planned")
        for cut in (1, 129, 100000):  # the block-item cut moves work, never bits
            o3 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=variant, heavy=cut))
            torch.cuda.synchronize()
            assert_bitwise(o3, ref, f"form {variant} heavy cut {cut}")
    opts = ops.make_options(variant=30001)
    kern = ops.SpmmCsrKernel(m, k, n, nnz, idx, DTYPES[dtype], device, opts)
    bias = random_dense(1, n, rng, DTYPES[dtype])[0]
    out2 = torch.full((m, n), float("nan"), dtype=DTYPES[dtype], device=device)
    kern(*d, out2, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(out2, oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype), "epilogue")
    out3 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=30001, ordered=True))
    torch.cuda.synchronize()
    assert_bitwise(out3, oracle_spmm(rp, ci, v, b, ordered=True), "ordered")
    perm = torch.from_numpy(rng.permutation(nnz).astype(np.int64)).to(idx)
    vals_src = torch.empty_like(v)
    vals_src[perm.long()] = v
    out4 = ops.spmm_csr_gathered(d[0], d[1], vals_src.to(device), perm.to(device), d[3], m, k,
                                 options=opts)
    torch.cuda.synchronize()
    assert_bitwise(out4, ref, "gathered values")


@pytest.mark.parametrize("dtype,idx", [("bf16", torch.int32), ("f16", torch.int64)])
@pytest.mark.parametrize("n", [8, 16, 24, 48, 64])
def test_narrow_16bit_bandwidth_layout(device, dtype, idx, n):
    """16-bit rows of <= 128 B in the bandwidth configuration (above kPrefetchNnz nonzeros) take
    N / 16 elements per lane over >= 16 lanes (launch_typed, narrow16) at 8 / 16 / 32 / 64
    columns, and (round 5) shifted 4 / 8-element windows at the other widths (24, 48) instead of
    the widest vector.  Lane layout only: the same bits as the oracle and as the widest-vector
    configuration forced."""
    rng = np.random.default_rng(4100 + n)
    m, k = 120_000, 90_000
    deg = rng.integers(0, 60, size=m)
    deg[17] = 3000  # a hub row (split)
    rp, ci, v = random_csr(m, k, deg, rng, idx, DTYPES[dtype])
    assert ci.numel() > (3 << 20)
    b = random_dense(k, n, rng, DTYPES[dtype])
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{dtype} n={n} auto")
    wide = 8 if n % 8 == 0 else (4 if n % 4 == 0 else 2)
    lpr = max(4, 1 << (n // wide - 1).bit_length())
    o2 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=wide * 100 + lpr))
    torch.cuda.synchronize()
    assert torch.equal(o2.view(torch.int16), out.view(torch.int16))


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("n", [1, 3, 5, 17, 18, 41, 47, 63, 99, 301])
def test_shifted_window_odd_widths(device, idx, n):
    """fp32 widths that are not a multiple of 4 above N = 64 in the bandwidth configuration (above
    kPrefetchNnz nonzeros) run 16-B lanes whose last window ends at column n - 1 (Cfg::SH; the
    shifted lane repeats its neighbour's first columns with the same bits).  Bit-exact against the
    oracle for contiguous B / C, strided views with a 4-B-offset base (ldb, ldc > n), the fused
    epilogue, hub rows, and against the one-element-per-lane configuration forced."""
    rng = np.random.default_rng(5100 + n)
    m, k = 120_000, 90_000
    deg = rng.integers(0, 60, size=m)
    deg[17] = 3000
    deg[9_999] = 700
    rp, ci, v = random_csr(m, k, deg, rng, idx, torch.float32)
    assert ci.numel() > (3 << 20)
    b = random_dense(k, n, rng)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"n={n} auto")
    lpr = min(64, max(4, 1 << (n - 1).bit_length()))
    o1 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=100 + lpr))
    torch.cuda.synchronize()
    assert torch.equal(o1.view(torch.int32), out.view(torch.int32))
    # strided views, base offset by one element (4 B): B[:, 1:n+1] of a (k, n+3) buffer
    bbig = torch.zeros((k, n + 3), dtype=torch.float32, device=device)
    bbig[:, 1:n + 1] = d[3]
    cbig = torch.full((m, n + 5), float("nan"), device=device)
    ops.spmm_csr_device(d[0], d[1], d[2], bbig[:, 1:n + 1], m, k, out=cbig[:, 3:n + 3])
    torch.cuda.synchronize()
    assert_bitwise(cbig[:, 3:n + 3], ref, f"n={n} strided, offset base")
    assert torch.isnan(cbig[:, :3]).all() and torch.isnan(cbig[:, n + 3:]).all()
    bias = random_dense(1, n, rng)[0]
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), idx, torch.float32, device)
    o3 = torch.full((m, n), float("nan"), device=device)
    kern(*d, o3, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(o3, oracle.bias_act(ref, to_oracle(bias), "relu", dtype="f32"), "epilogue")


@pytest.mark.parametrize("dtype,n", [("f32", 17), ("f32", 47), ("f32", 99), ("bf16", 16), ("bf16", 48),
                                     ("f16", 8)])
def test_prefetch_form_lane_layouts(device, dtype, n):
    """Mid-size launches (the prefetching form, <= kPrefetchNnz nonzeros): 16-bit rows of <= 128 B
    take N / 16 elements per lane, odd fp32 widths above 16 the shifted 16-B window (Cfg::SH with
    the prefetching configuration).  Bit-exact against the oracle, including hub rows, a row range
    and the one-element-per-lane bandwidth configuration forced."""
    rng = np.random.default_rng(6100 + n)
    m, k = 60_000, 60_000
    deg = rng.integers(0, 30, size=m)
    deg[11] = 4000
    deg[777] = 600
    dt = DTYPES[dtype]
    rp, ci, v = random_csr(m, k, deg, rng, torch.int32, dt)
    assert 32_768 < m and ci.numel() <= (3 << 20)
    b = random_dense(k, n, rng, dt)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{dtype} n={n} auto")
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), torch.int32, dt, device)
    sub = torch.full((30_000, n), float("nan"), dtype=dt, device=device)
    kern(*d, sub, row_begin=5_000, row_end=35_000)
    lpr = min(64, max(4, 1 << (n - 1).bit_length()))
    o1 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=100 + lpr))
    torch.cuda.synchronize()
    assert_bitwise(sub, ref[5_000:35_000], "row range")
    assert torch.equal(o1.view(torch.uint8), out.view(torch.uint8))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n", [1, 3, 4, 7, 12, 15, 16, 17, 24, 31, 32, 33, 41, 47, 48, 63, 64, 65,
                               99, 128, 129, 255])
def test_mid_width_rule_bitexact(device, dtype, n):
    """Round 5's rows of 17-128 columns of mid-size launches (launch_mid_width_pf: shifted windows,
    32-lane wave items of HV elements, hubs added in the kernel) and 16 columns (the narrow forms).  Bit-exact against the oracle for the automatic
    launch (hub rows and heavy rows included), element-offset strided views, a row range and the
    fused epilogue (the hub tail writes it)."""
    rng = np.random.default_rng(7300 + n)
    m, k = 60_000, 60_000
    deg = rng.integers(0, 30, size=m)
    deg[11], deg[777], deg[5] = 4000, 600, 1500
    dt = DTYPES[dtype]
    rp, ci, v = random_csr(m, k, deg, rng, torch.int32, dt)
    b = random_dense(k, n, rng, dt)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    desc = ops.describe(m, k, n, ci.numel(), dt, b_addr=d[3].data_ptr(), c_addr=256)
    top = 128 if dtype == "f32" else 256  # the rule's widths (fp32 above 128: the prefetch form)
    assert (desc["form"] == "narrow") == (n <= top), desc
    hl = 0 if n > top else 4 if n < 4 else 8 if n <= 32 else 16 if n <= 64 else 32
    xl = 1 if n <= 64 or (dtype == "f32" and n <= top) else 0
    assert desc["HL"] == hl and desc["XL"] == xl, desc
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{dtype} n={n} auto")
    # views one element off their allocation, ldb = n + 3, ldc = n + 2
    bbig = torch.zeros((k, n + 3), dtype=dt, device=device)
    bbig[:, 1:n + 1] = d[3]
    cbig = torch.full((m, n + 2), float("nan"), dtype=dt, device=device)
    ops.spmm_csr_device(d[0], d[1], d[2], bbig[:, 1:n + 1], m, k, out=cbig[:, 1:n + 1])
    torch.cuda.synchronize()
    assert_bitwise(cbig[:, 1:n + 1], ref, f"{dtype} n={n} offset views")
    assert torch.isnan(cbig[:, 0]).all() and torch.isnan(cbig[:, n + 1]).all()
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), torch.int32, dt, device)
    sub = torch.full((30_000, n), float("nan"), dtype=dt, device=device)
    kern(*d, sub, row_begin=5_000, row_end=35_000)
    torch.cuda.synchronize()
    assert_bitwise(sub, ref[5_000:35_000], f"{dtype} n={n} row range")
    bias = random_dense(1, n, rng, dt)[0]
    o3 = torch.full((m, n), float("nan"), dtype=dt, device=device)
    kern(*d, o3, bias=bias.to(device), relu=True)
    torch.cuda.synchronize()
    assert_bitwise(o3, oracle.bias_act(ref, to_oracle(bias), "relu", dtype=dtype), f"{dtype} n={n} epilogue")


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n", [16, 17, 24, 31, 32, 33, 47, 48, 63, 64, 65, 66, 99, 104, 127, 255])
def test_shifted_window_16bit_wide_rows(device, dtype, n):
    """Round 5: 16-bit widths above 64 that are not a multiple of 8, and 17-63 but 32, in the
    bandwidth configuration (above kPrefetchNnz) run 4 / 8-element windows at 2-B alignment, the
    last one shifted to end at column n - 1 (launch_shift).  Bit-exact against the oracle for contiguous
    operands, element-offset strided views and hub rows, and equal to the one-element-per-lane
    configuration forced; 64 and 104 columns (the widths either side) keep their layouts."""
    rng = np.random.default_rng(8100 + n)
    m, k = 120_000, 90_000
    deg = rng.integers(0, 60, size=m)
    deg[17], deg[9_999] = 3000, 700
    dt = DTYPES[dtype]
    rp, ci, v = random_csr(m, k, deg, rng, torch.int32, dt)
    assert ci.numel() > (3 << 20)
    b = random_dense(k, n, rng, dt)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    desc = ops.describe(m, k, n, ci.numel(), dt, b_addr=d[3].data_ptr(), c_addr=256)
    shifted = (n > 64 and n % 8 != 0) or (16 < n < 64 and n != 32)
    assert desc["form"] == "bandwidth" and desc["SH"] == (1 if shifted else 0), desc
    ref = oracle_spmm(rp, ci, v, b)
    out = fs.spmm(d[0], d[1], d[2], m, k, d[3])
    torch.cuda.synchronize()
    assert_bitwise(out, ref, f"{dtype} n={n} auto")
    o1 = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=164))
    torch.cuda.synchronize()
    assert torch.equal(o1.view(torch.int16), out.view(torch.int16))
    bbig = torch.zeros((k, n + 3), dtype=dt, device=device)
    bbig[:, 1:n + 1] = d[3]
    cbig = torch.full((m, n + 2), float("nan"), dtype=dt, device=device)
    ops.spmm_csr_device(d[0], d[1], d[2], bbig[:, 1:n + 1], m, k, out=cbig[:, 1:n + 1])
    torch.cuda.synchronize()
    assert_bitwise(cbig[:, 1:n + 1], ref, f"{dtype} n={n} offset views")
    assert torch.isnan(cbig[:, 0]).all() and torch.isnan(cbig[:, n + 1]).all()


ROUND5_ENTRIES = (list(range(90, 105)) + list(range(105, 158)) + list(range(170, 210)))


@pytest.fixture(scope="module")
def round5_graph():
    rng = np.random.default_rng(9100)
    m, k = 60_000, 60_000
    deg = rng.integers(0, 30, size=m)
    deg[11], deg[777], deg[5] = 4000, 600, 1500
    return m, k, deg, rng


@needs_tuning_table
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("n", [13, 47])
def test_tuning_table_round5_bitexact(device, round5_graph, dtype, n):
    """Every round-5 tuning entry (variant 10000 + id: the mid-size shapes, wave-item group
    shapes, LDS-exchanged wave items, the bandwidth form's in-between widths) that exists for the
    dtype computes the oracle's bits on a mid-size graph with hub rows, every row compared."""
    m, k, deg, rng = round5_graph
    dt = DTYPES[dtype]
    rp, ci, v = random_csr(m, k, deg, np.random.default_rng(9200 + n), torch.int32, dt)
    b = random_dense(k, n, np.random.default_rng(9300 + n), dt)
    d = (rp.to(device), ci.to(device), v.to(device), b.to(device))
    ref = oracle_spmm(rp, ci, v, b)
    ran = 0
    for tid in ROUND5_ENTRIES:
        try:
            out = ops.spmm_csr_device(*d, m, k, options=ops.make_options(variant=10000 + tid))
        except ops._lib.OfxError as e:  # not an entry of this dtype / width
            assert "tuning variant" in str(e) or "not applicable" in str(e), (tid, str(e))
            continue
        torch.cuda.synchronize()
        assert_bitwise(out, ref, f"{dtype} n={n} tuning entry {10000 + tid}")
        ran += 1
    assert ran >= 15, ran
