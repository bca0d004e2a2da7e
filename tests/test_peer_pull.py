"""The pull form of the row-split all-gather (include/ofx_spmm.h ofx_peer_*,
csrc/peer_pull.hip): every rank reads each peer's slot straight out of the peer's gathered buffer.

- CPU (gloo, 3 ranks): the tile plan the kernel runs (ofx_peer_pull_host, the same pull_tile()),
  over buffers that the ranks share through files in /dev/shm, against torch.distributed's
  all_gather of the same slots: slot sizes that take the 16-, 4- and 2-byte word paths, a slot of
  many tiles, and every rank position (the plan skips the caller's own slot).
- GPU (2 processes on the visible device, gloo as the bootstrap and the barrier): IPC handles
  exported / opened through the C-ABI (a buffer at an offset inside its allocation included),
  the publish + pull kernels, bit-exact against the slots each rank wrote; then every rank
  rewrites its slot and pulls again (nothing stale served from a cache).
The composed RCCL form (ofx_allgather_pull: barriers on the stream) is covered by
tests/test_gpu_multirank.py's "rccl-pull" (skipped where RCCL refuses two ranks on one device) and
by the single-rank row-split test."""
import ctypes
import os
import socket
import tempfile
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oneflow_spmm._lib import LIB, OFX_EINVAL, PEER_HANDLE_BYTES, check

# (rows per slot, columns, dtype): 16-B words, 4-B words, 2-B words, a slot of ~10 tiles
CASES = [(37, 64, torch.float32), (5, 3, torch.float32), (5, 7, torch.bfloat16),
         (300, 128, torch.float32)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slot(rank, rows, n, dt, round_=0):
    g = torch.Generator().manual_seed(1000 * round_ + 17 * rank + rows * 3 + n)
    return torch.randn(rows, n, generator=g).to(dt)


def _layout_worker(rank, world, port, shm_dir, q):
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        for ci, (rows, n, dt) in enumerate(CASES):
            own = _slot(rank, rows, n, dt)
            slot_bytes = own.numel() * own.element_size()
            path = os.path.join(shm_dir, f"case{ci}_rank{rank}")
            mine = np.memmap(path, dtype=np.uint8, mode="w+", shape=(world * slot_bytes,))
            mine[:] = 0xEE  # other slots: garbage until pulled
            mine[rank * slot_bytes:(rank + 1) * slot_bytes] = own.view(torch.uint8).reshape(-1).numpy()
            mine.flush()
            dist.barrier()  # every slot written
            maps = [mine if r == rank else
                    np.memmap(os.path.join(shm_dir, f"case{ci}_rank{r}"), dtype=np.uint8, mode="r",
                              shape=(world * slot_bytes,)) for r in range(world)]
            bufs = (ctypes.c_void_p * world)(*[m.ctypes.data for m in maps])
            check(LIB.ofx_peer_pull_host(world, rank, bufs, mine.ctypes.data, slot_bytes),
                  "peer_pull_host")
            parts = [torch.empty_like(own) for _ in range(world)]
            dist.all_gather(parts, own)
            want = torch.cat(parts).view(torch.uint8).reshape(-1).numpy()
            ok = bool(np.array_equal(np.asarray(mine), want))
            dist.barrier()  # every pull done before the files go
            del maps, mine
            q.put((rank, ci, "ok" if ok else "mismatch"))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, -1, traceback.format_exc()))


def test_pull_plan_matches_all_gather_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    with tempfile.TemporaryDirectory(dir=base, prefix="ofx_pull_") as d:
        procs = [ctx.Process(target=_layout_worker, args=(r, world, port, d, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=180) for _ in range(world * len(CASES))]
        for p in procs:
            p.join(timeout=60)
    errs = [r for r in res if r[2] != "ok"]
    assert not errs, errs[0]
    assert len(res) == world * len(CASES)


def test_pull_argument_errors():
    a = np.zeros(64, dtype=np.uint8)
    bufs = (ctypes.c_void_p * 2)(a.ctypes.data, a.ctypes.data)
    assert LIB.ofx_peer_pull_host(17, 0, bufs, a.ctypes.data, 16) == OFX_EINVAL  # > 16 ranks
    assert LIB.ofx_peer_pull_host(2, 2, bufs, a.ctypes.data, 16) == OFX_EINVAL   # rank >= ranks
    assert LIB.ofx_peer_pull_host(2, 0, bufs, a.ctypes.data, 7) == OFX_EINVAL    # odd slot
    nul = (ctypes.c_void_p * 2)(a.ctypes.data, None)
    assert LIB.ofx_peer_pull_host(2, 0, nul, a.ctypes.data, 16) == OFX_EINVAL    # peer 1 NULL
    assert LIB.ofx_peer_pull_host(1, 0, None, None, 16) == 0                     # nothing to pull
    assert LIB.ofx_peer_close(ctypes.c_void_p(a.ctypes.data)) == OFX_EINVAL      # never opened
    assert LIB.ofx_peer_close(None) == 0


def _gpu_worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        from oneflow_spmm._C import current_stream_handle
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        dev = torch.device("cuda", 0)
        results = []
        for ci, (rows, n, dt) in enumerate(CASES):
            # the buffer sits 3 rows into its allocation (the handle carries the offset)
            whole = torch.full((world * rows + 3, n), -7.0, dtype=dt, device=dev)
            buf = whole[3:]
            slot_bytes = rows * n * buf.element_size()
            h = ctypes.create_string_buffer(PEER_HANDLE_BYTES)
            check(LIB.ofx_peer_export(ctypes.c_void_p(buf.data_ptr()), h), "peer_export")
            hs = [None] * world
            dist.all_gather_object(hs, bytes(h.raw))
            ptrs = []
            for r in range(world):
                if r == rank:
                    ptrs.append(buf.data_ptr())
                    continue
                p = ctypes.c_void_p()
                check(LIB.ofx_peer_open(ctypes.create_string_buffer(hs[r], PEER_HANDLE_BYTES),
                                        ctypes.byref(p)), "peer_open")
                ptrs.append(p.value)
            arr = (ctypes.c_void_p * world)(*ptrs)
            s = current_stream_handle(buf)
            for rnd in range(2):  # the second round rewrites every slot and pulls again
                buf[rank * rows:(rank + 1) * rows].copy_(_slot(rank, rows, n, dt, rnd).to(dev))
                check(LIB.ofx_peer_publish(s), "peer_publish")
                torch.cuda.synchronize()
                dist.barrier()  # every slot written and published
                check(LIB.ofx_peer_pull(s, world, rank, arr, ctypes.c_void_p(buf.data_ptr()),
                                        slot_bytes), "peer_pull")
                torch.cuda.synchronize()
                dist.barrier()  # every pull done before the next round rewrites the slots
                want = torch.cat([_slot(r, rows, n, dt, rnd) for r in range(world)])
                got = buf.cpu()
                bits = {2: torch.int16, 4: torch.int32}[dt.itemsize]
                same = torch.equal(got.view(bits), want.view(bits))
                pad_ok = bool((whole[:3].cpu().float() == -7.0).all())
                results.append((ci, rnd, same, pad_ok))
            for r, p in enumerate(ptrs):
                if r != rank:
                    check(LIB.ofx_peer_close(ctypes.c_void_p(p)), "peer_close")
            dist.barrier()
        q.put((rank, "ok", results))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
def test_peer_pull_two_processes_bit_exact():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if r[1] == "err"]
    assert not errs, errs[0][2]
    for rank, _, results in res:
        assert len(results) == 2 * len(CASES)
        for ci, rnd, same, pad_ok in results:
            assert same, f"rank {rank} case {CASES[ci]} round {rnd}: pulled bytes differ"
            assert pad_ok, f"rank {rank} case {ci}: bytes before the buffer were written"
