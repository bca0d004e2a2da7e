"""The collective layer of the OneFlow mirror on the CPU (include/ofx_spmm.h, "collectives and
the lazy path"): the keyed ccl registry (REGISTER_COLLECTIVE_COMMUNICATION), the eager boxing
"ccl-s-to-b" check (oneflow/core/boxing/ccl_boxing_function.cpp:104-122) and run through op
eager_ccl_all_gather and its kCPU kernel (the ring of collective_communication/cpu/
cpu_all_gather.cpp:27-80) on 2-4 gloo ranks, InsertNcclLogicalOpPass's choices
(insert_nccl_logical_op_pass.cpp:150-240), EagerRcclCommMgr's key and rank, and the compiled
row-split job's plan.  The kHIP paths run in tests/test_ccl_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oneflow_spmm import OfxError, ccl
from oneflow_spmm.ccl import PlacementSpec


def test_registry_has_cpu_and_hip_collectives():
    assert ccl.ccl_registered("cpu") == (True, True)
    assert ccl.ccl_registered("hip") == (True, True)


def test_check_ccl_s2b_mirrors_the_reference_conditions():
    pl = PlacementSpec("cpu", 4, 1)
    ccl.check_ccl_s2b(pl, (8, 3))
    ccl.check_ccl_s2b(PlacementSpec("hip", 4, 0), (8, 3))
    with pytest.raises(OfxError, match="not divisible"):
        ccl.check_ccl_s2b(pl, (9, 3))  # K % G != 0: ccl_boxing_function.cpp:114
    with pytest.raises(OfxError):
        ccl.check_ccl_s2b(pl, (8, 3), in_sbp="S(1)")
    with pytest.raises(OfxError):
        ccl.check_ccl_s2b(pl, (8, 3), out_sbp="P")
    with pytest.raises(OfxError):
        ccl.check_ccl_s2b(pl, ())


@pytest.mark.parametrize("src,dst,shape,p,want", [
    ("S(0)", "B", (8, 4), 4, "_nccl_logical_all_gather"),
    ("S(0)", "B", (9, 4), 4, ""),  # K % P != 0: no logical collective
    ("S(1)", "B", (9, 4), 4, "_nccl_logical_all_gather_noncontinuous"),
    ("P", "B", (9, 4), 4, "_nccl_logical_all_reduce"),
    ("P", "S(0)", (8, 4), 4, "_nccl_logical_reduce_scatter"),
    ("P", "S(1)", (9, 4), 4, "_nccl_logical_reduce_scatter_noncontinuous"),
    ("S(0)", "S(1)", (8, 4), 4, "_nccl_logical_s2s"),
    ("B", "S(0)", (8, 4), 4, ""),
])
def test_insert_nccl_logical_op_pass(src, dst, shape, p, want):
    assert ccl.insert_nccl_logical_op(src, dst, shape, p) == want


def test_rccl_comm_key_and_rank():
    pl = PlacementSpec("hip", 4, 0, machine_ids=(3, 1, 2, 0), device_ids=(3, 1, 2, 0))
    key, rank = ccl.rccl_comm_key(pl, 2, 2)
    assert key == "eager_rccl_unique_id_rpc_key,0:0,1:1,2:2,3:3" and rank == 2
    assert ccl.rccl_comm_key(pl, 5, 0)[1] == -1
    key2, _ = ccl.rccl_comm_key(pl, 0, 0, stream_name="s1")
    assert key2.startswith("eager_rccl_unique_id_rpc_key/s1,") and key2 != key


def test_ccl_s2b_one_cpu_rank():
    ccl.install_control_plane()
    x = torch.arange(15, dtype=torch.float32).reshape(5, 3)
    out = ccl.ccl_s2b(x, PlacementSpec("cpu", 1, 0), 5)
    assert torch.equal(out, x)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _s2b_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oneflow_spmm import OfxError as Err
        from oneflow_spmm import ccl as c
        from oneflow_spmm.ccl import PlacementSpec as PS
        c.install_control_plane()
        pl = PS.of_process_group("cpu")
        ok = True
        for dt, k, n in ((torch.float32, 4 * world, 5), (torch.bfloat16, 2 * world, 33),
                         (torch.int64, 3 * world, 1), (torch.float32, 0, 7)):
            full = (torch.arange(k * n, dtype=torch.float64).reshape(k, n) * 1.25 - 7).to(dt)
            lo, hi = rank * (k // world), (rank + 1) * (k // world)
            out = c.ccl_s2b(full[lo:hi].clone(), pl, k)
            ok = ok and torch.equal(out.view(torch.uint8), full.view(torch.uint8))
        # in place: the rank's slot of `out` is the input
        k, n = 2 * world, 4
        full = torch.randn(k, n, generator=torch.Generator().manual_seed(3))
        out = torch.zeros(k, n)
        out[2 * rank:2 * rank + 2] = full[2 * rank:2 * rank + 2]
        c.ccl_s2b(out[2 * rank:2 * rank + 2], pl, k, out=out)
        ok = ok and torch.equal(out, full)
        # K % G != 0 is refused by the boxing's check on every rank (no rank enters the ring)
        try:
            c.ccl_s2b(torch.zeros(1, 3), pl, 2 * world + 1)
            ok = False
        except Err as e:
            ok = ok and "not divisible" in str(e)
        # the lazy job of a CPU placement keeps ordinary boxing: refused with the reason
        try:
            c.SpmmJob(pl, 10, 4 * world, 8, 20, torch.int32, torch.float32, "cpu")
            ok = False
        except Err as e:
            ok = ok and "device placements only" in str(e)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_ccl_s2b_ring_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_s2b_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert res == {r: True for r in range(world)}, res


def test_spmm_job_plan_and_one_device_cpu_run():
    from oracle import oracle
    from tests.helpers import power_law_degrees, random_csr, random_dense
    rng = np.random.default_rng(12)
    m, k, n = 300, 260, 16
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 6000, k, rng), rng)
    b = random_dense(k, n, rng)
    job = ccl.SpmmJob(PlacementSpec("cpu", 1, 0), m, k, n, ci.numel(), torch.int32,
                      torch.float32, "cpu")
    assert "no boxing" in job.plan and "spmm_csr" in job.plan
    out = job(rp, ci, v, b)
    ref = oracle.spmm(rp.numpy(), ci.numpy(), v.numpy(), b.numpy())
    assert np.array_equal(out.numpy().view(np.uint32), ref.view(np.uint32))
    with pytest.raises(ValueError, match="b_shard must be"):
        job(rp, ci, v, b[:-1])
    with pytest.raises(ValueError, match="col_idx must be"):
        job(rp, ci.long(), v, b)
    # graph mode is a device-stream feature: a host placement ignores it and runs eagerly
    job.set_graph(True)
    out2 = job(rp, ci, v, b)
    assert np.array_equal(out2.numpy().view(np.uint32), ref.view(np.uint32))
    assert job.graph_stats == {"captures": 0, "replays": 0, "updates": 0}
    # a HIP placement of 4 ranks compiles the logical collective into the plan (the RCCL
    # communicator is created on the first run, on the GPU)
    job4 = ccl.SpmmJob(PlacementSpec("hip", 4, 2), m, 4 * 65, n, ci.numel(), torch.int32,
                       torch.bfloat16, "cpu")
    assert "_nccl_logical_all_gather(src S(0), dst B" in job4.plan
    assert "(65,16) on this rank" in job4.plan and "rows [150,225)" in job4.plan
    assert job4.tmp_bytes >= 4 * 65 * n * 2
    # a multi-rank capture (ncclAllGather inside a hipGraph) is not validated on
    # hardware, so graph mode is refused at P > 1 (eager runs stay available)
    with pytest.raises(OfxError, match="graph mode with 4 ranks"):
        job4.set_graph(True)
    job4.set_graph(False)
    with pytest.raises(OfxError, match="K % P != 0"):
        ccl.SpmmJob(PlacementSpec("hip", 4, 0), m, 261, n, ci.numel(), torch.int32,
                    torch.float32, "cpu")
