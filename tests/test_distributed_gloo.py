"""CPU multi-process (gloo) tests of the row-split wrapper: BalancedSplitter rows, padded in-place
all-gather of the Split(0) dense shards, column remap, local SpMM — bit-exact against the
oracle's full product; column-block pipelining; the halo-only exchange (bound form).  The same
code path runs RCCL on GPUs (comm="rccl")."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, m, k, n, local_csr, pipeline, density, q, device="cpu"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import sys
    for p in (root, os.path.join(root, "of-spmm_amd")):
        sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import ops
        from oneflow_spmm.distributed import RowSplitSpmm
        from oracle import oracle
        from tests.helpers import power_law_degrees, random_csr, random_dense

        dev = torch.device(device)
        if dev.type == "cuda":  # every rank on the one GPU; gloo moves the bytes (host-staged)
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
        D = lambda t: t.to(dev)  # noqa: E731
        same = lambda got, want: np.array_equal(got.cpu().numpy().view(np.uint32),  # noqa: E731
                                                want.view(np.uint32))
        rng = np.random.default_rng(1234)
        rp, ci, v = random_csr(m, k, power_law_degrees(m, min(density * m, m * k // 2), k, rng), rng)
        b = random_dense(k, n, rng)
        full = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy())
        lo, hi = oracle.balanced_range(m, world, rank)
        if local_csr:
            lrp, n0, n1 = ops.csr_row_slice(rp, lo, hi)
            lci, lv = ci[n0:n1], v[n0:n1]
        else:
            lrp, lci, lv = rp, ci, v
        rs = RowSplitSpmm(m, k, n, lci.numel(), torch.float32, torch.int32, dev,
                          comm="torch", local_csr=local_csr, pipeline=pipeline)
        assert rs.row_range == (lo, hi)
        klo, khi = rs.k_range
        assert (klo, khi) == oracle.balanced_range(k, world, rank)
        drp, dci, dv = D(lrp), D(lci), D(lv)
        rs.load_shard(D(b[klo:khi]))
        out = rs(drp, rs.remap_columns(dci), dv)
        ok = same(out, full[lo:hi])
        # the gathered buffer holds every shard at its padded slot, in every column block
        nc = n // pipeline
        for c in range(pipeline):
            g = rs.block(c).cpu().view(world, rs.pad, nc)
            for r in range(world):
                a, e = oracle.balanced_range(k, world, r)
                ok = ok and torch.equal(g[r, : e - a], b[a:e, c * nc:(c + 1) * nc])
        # a second step with a new dense operand passed as a separate shard tensor
        b2 = random_dense(k, n, np.random.default_rng(99))
        out2 = rs(drp, rs.remap_columns(dci), dv, b_shard=D(b2[klo:khi]))
        full2 = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b2.numpy())
        ok = ok and same(out2, full2[lo:hi])
        # the bound form with the halo-only exchange: same bytes
        rs.bind(drp, dci, dv, halo=True)
        h = rs.halo
        ok = ok and h.k_compact == (khi - klo) + h.halo_rows and h.halo_rows <= k - (khi - klo)
        rs.exchange = "halo"
        out3 = torch.full_like(out2, float("nan"))
        rs.step(out3, b_shard=D(b[klo:khi]))
        ok = ok and same(out3, full[lo:hi])
        # every halo row holds the B row it stands for
        uniq = torch.unique((lci if local_csr else lci[int(lrp[lo]):int(lrp[hi])]).long())
        ok = ok and torch.equal(rs.compact[0, : h.k_own].cpu(), b[klo:khi])
        remote = uniq[(uniq < klo) | (uniq >= khi)]
        ok = ok and torch.equal(rs.compact[0, h.k_own:].cpu(), b[remote])
        # the halo exchange in column blocks (block-major compact B): same bytes
        for hp in (2, 4):
            if n % hp == 0:
                rs.set_halo_pipeline(hp)
                out3.fill_(float("nan"))
                rs.step(out3, b_shard=D(b2[klo:khi]))
                ok = ok and same(out3, full2[lo:hi])
                nc = n // hp
                for c in range(hp):
                    ok = ok and torch.equal(rs.compact[c, h.k_own:].cpu(), b2[remote, c * nc:(c + 1) * nc])
        rs.set_halo_pipeline(1)
        # the grids (B to column blocks, SpMM of the row group's rows, C back inside the group;
        # the column split is the 1 x G grid): same bytes
        # (and S = 2 sub-blocks, the pipelined form's layout)
        rs.bind(drp, dci, dv, halo=False, full_csr=(D(rp), D(ci), D(v)), grid_subs=(1, 2))
        want = {("nsplit" if c == world else f"grid{world // c}x{c}") + ("" if s == 1 else f"/s{s}")
                for c in range(2, world + 1) for s in (1, 2) if world % c == 0 and n % (c * s) == 0}
        ok = ok and set(rs.grids) == want and (rs.ns is not None) == (n % world == 0)
        for name, gp in rs.grids.items():
            rs.exchange = name
            out4 = torch.full_like(out2, float("nan"))
            rs.step(out4, b_shard=D(b2[klo:khi]))
            ok = ok and same(out4, full2[lo:hi])
            nb = n // gp.cn
            for s in range(gp.sub):
                c0 = gp.c * nb + s * gp.w
                ok = ok and torch.equal(gp.b_cols[s].cpu(), b2[:, c0:c0 + gp.w])
            ok = ok and (gp.glo, gp.ghi) == (oracle.balanced_range(m, world, gp.g * gp.cn)[0],
                                             oracle.balanced_range(m, world, gp.g * gp.cn + gp.cn - 1)[1])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m,k,n,local_csr", [
    (2, 301, 257, 16, True),    # K % G != 0 -> padded shards + remap
    (2, 300, 256, 32, False),   # full CSR broadcast, kernel computes the row range
    (3, 500, 400, 8, True),
    (4, 603, 1001, 16, True),   # 4 ranks: K % 4 = 1, one long shard and three short ones
    (6, 700, 1003, 12, False),  # 6 ranks: grids 3x2, 2x3 and the 1x6 column split
    (8, 1201, 1205, 32, True),  # the 8-GPU node's shape: grids 4x2, 2x4, 1x8 (and /s2 each)
    (8, 5, 6, 8, False),        # fewer rows and B rows than ranks: empty shards, 1-wide blocks
])
def test_row_split_gloo(world, m, k, n, local_csr):
    _run(world, m, k, n, local_csr, 1, 30)


@pytest.mark.parametrize("world,m,k,n,local_csr,pipeline", [
    (2, 400, 3001, 128, True, 4),   # hub rows > 2 x default_split(128) = 1024: blocks keep it
    (3, 301, 2999, 128, False, 2),
])
def test_row_split_pipelined_gloo(world, m, k, n, local_csr, pipeline):
    """Column-block pipelining: same bytes as pipeline 1 / the oracle with the full-N schedule."""
    _run(world, m, k, n, local_csr, pipeline, 60)


def _run(world, m, k, n, local_csr, pipeline, density, device="cpu"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, m, k, n, local_csr, pipeline,
                                               density, q, device)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    results = dict(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert results == {r: True for r in range(world)}, results


def _banded_worker(rank, world, port, q):
    """A graph with locality (every row references columns within +-w of itself): the halo
    exchange moves only the band edges instead of the whole B."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import sys
    for p in (root, os.path.join(root, "of-spmm_amd")):
        sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import ops
        from oneflow_spmm.distributed import RowSplitSpmm
        from oracle import oracle
        m = k = 3000
        n, w = 32, 20
        rng = np.random.default_rng(77)
        rows = [np.unique(np.clip(r + rng.integers(-w, w + 1, size=8), 0, k - 1)) for r in range(m)]
        rp = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in rows])]), dtype=torch.int32)
        ci = torch.tensor(np.concatenate(rows), dtype=torch.int32)
        v = torch.from_numpy(rng.uniform(-1, 1, ci.numel()).astype(np.float32))
        b = torch.from_numpy(rng.uniform(-1, 1, (k, n)).astype(np.float32))
        full = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy())
        lo, hi = oracle.balanced_range(m, world, rank)
        lrp, n0, n1 = ops.csr_row_slice(rp, lo, hi)
        rs = RowSplitSpmm(m, k, n, n1 - n0, torch.float32, torch.int32, "cpu")
        klo, khi = rs.k_range
        rs.load_shard(b[klo:khi])
        rs.bind(lrp, ci[n0:n1], v[n0:n1], halo=True)
        rs.exchange = "halo"
        out = rs.step(torch.empty((hi - lo, n)))
        ok = np.array_equal(out.numpy().view(np.uint32), full[lo:hi].view(np.uint32))
        ok = ok and 0 < rs.halo.halo_rows <= 2 * w * (world - 1)
        q.put((rank, bool(ok), rs.halo.halo_rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_halo_exchange_moves_only_the_band_edges(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_banded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _ in res), res


def _tune_worker(rank, world, port, q, device="cpu"):
    """tune() over torch.distributed (gloo): every candidate (all-gather x pipeline depth, halo,
    every grid with and without sub-blocks) runs the real step, the max-reduced timings make every
    rank keep the same one, and the kept exchange still gives the oracle's bits."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import sys
    for p in (root, os.path.join(root, "of-spmm_amd")):
        sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import ops
        from oneflow_spmm.distributed import RowSplitSpmm
        from oracle import oracle
        from tests.helpers import power_law_degrees, random_csr, random_dense

        dev = torch.device(device)
        if dev.type == "cuda":
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
        rng = np.random.default_rng(55)
        m, k, n = 900, 850, 16
        rp, ci, v = random_csr(m, k, power_law_degrees(m, 20000, k, rng), rng)
        b = random_dense(k, n, rng)
        full = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy())
        lo, hi = oracle.balanced_range(m, world, rank)
        lrp, n0, n1 = ops.csr_row_slice(rp, lo, hi)
        rs = RowSplitSpmm(m, k, n, n1 - n0, torch.float32, torch.int32, dev, comm="torch")
        klo, khi = rs.k_range
        rs.load_shard(b[klo:khi].to(dev))
        rs.bind(lrp.to(dev), ci[n0:n1].to(dev), v[n0:n1].to(dev), halo=True,
                full_csr=(rp.to(dev), ci.to(dev), v.to(dev)), grid_subs=(1, 2))
        out = torch.empty((hi - lo, n), device=dev)
        # every exchange awaited under a deadline, as the bench's set-up runs them (round 5: gloo's
        # point-to-point works report completion only from wait(), which a poll never saw)
        rs.set_exchange_deadline(60.0)
        times = rs.tune(out, reps=1, prune=float("inf"))  # every candidate runs
        want = {"torch/p1", "torch/p2", "torch/p4", "halo", "halo/p2", "halo/p4", "grid2x2",
                "grid2x2/s2", "nsplit", "nsplit/s2"}
        ok = set(times) == want and all(np.isfinite(t) for t in times.values())
        out.fill_(float("nan"))
        rs.step(out)
        ok = ok and np.array_equal(out.cpu().numpy().view(np.uint32), full[lo:hi].view(np.uint32))
        q.put((rank, (bool(ok), rs.exchange, rs.comm_kind, rs.chunks, sorted(times))))
    finally:
        dist.destroy_process_group()


def _tune_run(device):
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_worker, args=(r, world, port, q, device))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(r[0] for r in res.values()), res
    assert len({r[1:4] for r in res.values()}) == 1, res  # the same exchange on every rank


def test_tune_over_gloo_keeps_one_choice_everywhere():
    _tune_run("cpu")


def _tune_corrupt_worker(rank, world, port, q):
    """tune() compares every candidate's output bits with the first candidate's (a sampled
    digest, max-reduced over ranks): a candidate made to write other bytes on ONE rank (the
    pipelined halo exchange, +1 on rank 1's first output row) is dropped on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import sys
    for p in (root, os.path.join(root, "of-spmm_amd")):
        sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import ops
        from oneflow_spmm.distributed import RowSplitSpmm
        from tests.helpers import power_law_degrees, random_csr, random_dense

        rng = np.random.default_rng(56)
        m, k, n = 600, 500, 8
        rp, ci, v = random_csr(m, k, power_law_degrees(m, 9000, k, rng), rng)
        b = random_dense(k, n, rng)
        from oracle import oracle
        lo, hi = oracle.balanced_range(m, world, rank)
        lrp, n0, n1 = ops.csr_row_slice(rp, lo, hi)
        rs = RowSplitSpmm(m, k, n, n1 - n0, torch.float32, torch.int32, torch.device("cpu"),
                          comm="torch")
        klo, khi = rs.k_range
        rs.load_shard(b[klo:khi])
        rs.bind(lrp, ci[n0:n1], v[n0:n1], halo=True)
        step = rs.step

        def corrupt_step(out, *a, **kw):
            r = step(out, *a, **kw)
            if rs.exchange == "halo" and rs.halo_chunks == 2 and rank == 1:
                out[0] += 1.0
            return r
        rs.step = corrupt_step
        out = torch.empty((hi - lo, n))
        times = rs.tune(out, reps=1, prune=float("inf"))
        q.put((rank, sorted(times), " ".join(rs.tune_errors.values())))
    finally:
        dist.destroy_process_group()


def test_tune_drops_a_candidate_whose_output_differs():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_corrupt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = dict((r[0], r[1:]) for r in (q.get(timeout=5) for _ in range(world)))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, (names, err) in res.items():
        assert "halo/p2" not in names and "halo" in names and "torch/p1" in names, (rank, names)
        assert "differs" in err, (rank, err)


# ---- the same ranks on the GPU --------------------------------------------------------------
# RCCL refuses two ranks on one GPU, so on a one-GPU box these tests put every rank on cuda:0 and
# let gloo carry the exchanged bytes (host-staged).  Everything else is the device path the
# RCCL runs take: the remap kernel, the halo row gather, the grid pack/unpack block copies
# (ofx_copy_blocks) with this rank's offsets, the planned row-range SpMM launches of every row
# group and column block — checked bit-exactly against the oracle at world sizes > 1.

def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.gpu
@pytest.mark.parametrize("world,m,k,n,local_csr,pipeline,density", [
    (2, 301, 257, 16, True, 1, 30),     # K % G != 0 -> padded shards + remap on the device
    (3, 500, 400, 8, False, 1, 30),     # full CSR, the kernel computes the row range
    (4, 400, 3001, 128, True, 4, 60),   # hub rows that split, four column blocks
    (8, 1201, 1205, 32, True, 2, 30),   # the 8-GPU node's grids 4x2, 2x4, 1x8 (and /s2 each)
    (8, 5, 6, 8, False, 1, 30),         # fewer rows and B rows than ranks
])
def test_row_split_device_path_multirank(world, m, k, n, local_csr, pipeline, density):
    _need_gpu()
    _run(world, m, k, n, local_csr, pipeline, density, device="cuda")


@pytest.mark.gpu
def test_tune_device_path_multirank():
    _need_gpu()
    _tune_run("cuda")
