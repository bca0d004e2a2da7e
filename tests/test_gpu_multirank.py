"""Multi-rank RCCL path on whatever GPUs the box has: 2 processes share the visible GPU(s)
(rank r on device r % ndev), torch.distributed/gloo is only the bootstrap store, the RCCL
communicator and both all-gather schedules (ring ncclAllGather, grouped send/recv) go through the
C-ABI.  Every rank's output rows are compared bit-exactly with the oracle in the parent.
RCCL may refuse two ranks on one device ("Duplicate GPU"): the test then skips, the 2-rank
semantics stay covered by tests/test_distributed_gloo.py."""
import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import assert_bitwise, oracle_spmm, power_law_degrees, random_csr, random_dense

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, kind, rp, ci, v, b, q):
    try:
        import torch.distributed as dist
        from oneflow_spmm.distributed import RowSplitSpmm

        ndev = torch.cuda.device_count()
        device = torch.device("cuda", rank % ndev)
        torch.cuda.set_device(device)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        m, k, n = rp.numel() - 1, b.shape[0], b.shape[1]
        try:
            rs = RowSplitSpmm(m, k, n, ci.numel(), torch.float32, torch.int32, device,
                              comm="rccl" if kind in ("tune", "halo", "halo/p2", "nsplit", "nsplit/s2") else kind,
                              local_csr=False)
        except Exception as e:  # OfxError(OFX_ECOMM) when RCCL rejects the layout
            q.put((rank, "skip", str(e)))
            dist.destroy_process_group()
            return
        lo, hi = rs.k_range
        rs.load_shard(b[lo:hi].to(device))
        out = torch.empty((rs.row_range[1] - rs.row_range[0], n), device=device)
        d = (rp.to(device), ci.to(device), v.to(device))
        rs.bind(*d, halo=kind in ("tune", "halo", "halo/p2"),
                full_csr=d if kind in ("tune", "nsplit", "nsplit/s2") else None, grid_subs=(1, 2))
        if kind == "halo/p2":
            rs.exchange = "halo"
            rs.set_halo_pipeline(2)
        elif kind in ("halo", "nsplit", "nsplit/s2"):
            rs.exchange = kind
        times = rs.tune(out, reps=2) if kind == "tune" else {}
        # clear everything received, so the checked step must exchange it again
        sh = rs.shard()
        rs.gathered.zero_()
        if rs.halo is not None:
            rs.compact.zero_()
        for gp in rs.grids.values():
            gp.b_cols.zero_()
        rs.load_shard(sh)
        out.zero_()
        rs.step(out)
        torch.cuda.synchronize()
        q.put((rank, "ok", (rs.row_range, out.cpu(), (rs.exchange, rs.comm_kind, rs.chunks), times)))
        rs.close()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.parametrize("kind", ["rccl", "rccl-p2p", "rccl-pull", "halo", "halo/p2", "nsplit", "nsplit/s2",
                                  "tune"])
def test_row_split_two_ranks(kind):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(29)
    m, k, n = 1001, 999, 64          # K % 2 != 0: exercises the padded slots
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 30000, k, rng), rng)
    b = random_dense(k, n, rng)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_old = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, rp, ci, v, b, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    if env_old is None:
        os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    errs = [r for r in res if r[1] == "err"]
    assert not errs, errs[0][2]
    skips = [r for r in res if r[1] == "skip"]
    if skips:
        pytest.skip(f"RCCL refused this rank layout: {skips[0][2][:200]}")
    ref = oracle_spmm(rp, ci, v, b)
    kinds = set()
    for _, _, ((lo, hi), out, ck, times) in res:
        assert_bitwise(out, ref[lo:hi], f"{kind} rows [{lo},{hi})")
        kinds.add(ck)
        if kind == "tune":
            # the IPC pull is opt-in: not a default tune kind
            assert {t.split("/")[0] for t in times} == {"rccl", "rccl-p2p", "halo", "nsplit"}
    assert len(kinds) == 1  # every rank made the same choice
