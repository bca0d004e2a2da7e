"""GPU: attr static_csr keeps the work-list plan across calls.

The kernel state of `spmm_csr` (OpKernel::CreateOpKernelState, oneflow/core/framework/
op_kernel.h:292) plans a static CSR once and launches every later call with options.planned = 1
(no planner kernel).  Checked here, always against the oracle:
- eager op calls: one plan, then hits; the bits equal the unplanned call's;
- a call without the attribute still re-plans after row_ptr is rewritten in place, and a static
  call with a new static_csr value after the rewrite plans the new structure;
- a torch.cuda.graph capture of a static call (the plan built by an eager call before it) replays
  bit-exact with new b contents;
- the compiled job (SpmmJob) with static_csr, eager and in graph mode: one plan, exact replays;
- autograd's cached transpose: the d(b) SpMM of a constant-values graph reuses its plan.
"""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import _C, ccl
from tests.helpers import assert_bitwise, oracle_spmm, power_law_degrees, random_csr, random_dense

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fresh_plans():
    _C.static_plans(release=True)
    yield
    torch.cuda.synchronize()
    _C.static_plans(release=True)


def hub_graph(m, k, rng, hubs=((11, 4000), (777, 600))):
    deg = rng.integers(0, 30, size=m)
    for r, d in hubs:
        deg[r] = d
    return deg


def counters(before, after):
    return {k: after[k] - before[k] for k in ("plans", "hits")}


@pytest.mark.parametrize("dtype,n,idx", [(torch.float32, 17, torch.int32),
                                         (torch.bfloat16, 47, torch.int32),
                                         (torch.float32, 128, torch.int32),
                                         (torch.float64, 16, torch.int32),
                                         (torch.float16, 64, torch.int32),
                                         (torch.float32, 32, torch.int64)])
def test_static_calls_plan_once_and_match_the_oracle(device, dtype, n, idx):
    rng = np.random.default_rng(600 + n)
    m, k = 60_000, 60_000
    rp, ci, v = random_csr(m, k, hub_graph(m, k, rng), rng, idx_dtype=idx)
    b = random_dense(k, n, rng)
    d = [rp.to(device), ci.to(device), v.to(device, dtype)]
    db = b.to(device, dtype)
    ref = fs.spmm(*d, m, k, db)  # the ordinary call: plans every time
    s0 = _C.static_plans()
    outs = [fs.spmm(*d, m, k, db, static_csr=True) for _ in range(4)]
    torch.cuda.synchronize()
    st = counters(s0, _C.static_plans())
    assert st == {"plans": 1, "hits": 3}, st
    for o in outs:
        assert torch.equal(o.view(torch.uint8), ref.view(torch.uint8))
    assert_bitwise(outs[-1].cpu(), oracle_spmm(rp, ci, v.to(dtype), b.to(dtype)), f"{dtype} N={n}")


def test_rewritten_row_ptr_replans_without_the_attribute(device):
    """Same addresses, same nnz, other structure: the ordinary call plans the new graph; a static
    call needs a new static_csr value to do so (the attribute is the caller's promise)."""
    rng = np.random.default_rng(610)
    m, k, n = 60_000, 60_000, 32
    rp_a, ci_a, v_a = random_csr(m, k, hub_graph(m, k, rng), rng)
    deg_b = rng.permutation(np.diff(rp_a.numpy()))  # the hubs move; nnz unchanged
    rp_b, ci_b, v_b = random_csr(m, k, deg_b, rng)
    b = random_dense(k, n, rng)
    rp, ci, v = rp_a.to(device), ci_a.to(device), v_a.to(device)
    db = b.to(device)
    out = fs.spmm(rp, ci, v, m, k, db, static_csr=5)
    assert_bitwise(out.cpu(), oracle_spmm(rp_a, ci_a, v_a, b), "graph A, static")
    rp.copy_(rp_b.to(device))
    ci.copy_(ci_b.to(device))
    v.copy_(v_b.to(device))
    out = fs.spmm(rp, ci, v, m, k, db)  # no attribute: plans graph B
    assert_bitwise(out.cpu(), oracle_spmm(rp_b, ci_b, v_b, b), "graph B, ordinary call")
    s0 = _C.static_plans()
    out = fs.spmm(rp, ci, v, m, k, db, static_csr=6)  # a new value: a new plan
    torch.cuda.synchronize()
    assert counters(s0, _C.static_plans()) == {"plans": 1, "hits": 0}
    assert_bitwise(out.cpu(), oracle_spmm(rp_b, ci_b, v_b, b), "graph B, new static value")


@pytest.mark.graph_capture
def test_static_call_captured_in_a_graph(device):
    rng = np.random.default_rng(620)
    m, k, n = 60_000, 60_000, 64
    rp, ci, v = random_csr(m, k, hub_graph(m, k, rng), rng)
    b = random_dense(k, n, rng)
    d = [rp.to(device), ci.to(device), v.to(device)]
    db = b.to(device)
    out = torch.empty((m, n), device=device)
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        fs.spmm(*d, m, k, db, out=out, static_csr=True)  # eager: plans (outside the capture)
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    s0 = _C.static_plans()
    with torch.cuda.graph(g, stream=s):  # captured on the stream whose plan the warm call built
        fs.spmm(*d, m, k, db, out=out, static_csr=True)
    assert counters(s0, _C.static_plans()) == {"plans": 0, "hits": 1}
    for i in range(3):
        b2 = random_dense(k, n, rng)
        db.copy_(b2.to(device))
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b2), f"replay {i}")


@pytest.mark.graph_capture
@pytest.mark.parametrize("graph", [False, True])
def test_compiled_job_static_plan(device, graph):
    rng = np.random.default_rng(630 + graph)
    m, k, n = 40_000, 40_000, 64
    rp, ci, v = random_csr(m, k, hub_graph(m, k, rng), rng)
    pl = ccl.PlacementSpec("hip", 1, 0, (0,), (device.index or 0,))
    job = ccl.SpmmJob(pl, m, k, n, ci.numel(), torch.int32, torch.float32, device, graph=graph,
                      static_csr=7)
    d = [rp.to(device), ci.to(device), v.to(device)]
    out = torch.empty((m, n), device=device)
    db = torch.empty((k, n), device=device)
    for i in range(4):
        b = random_dense(k, n, rng)
        db.copy_(b.to(device))
        out.fill_(float("nan"))
        job(*d, db, out=out)
        torch.cuda.synchronize()
        assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b), f"run {i}")
    st = job.static_stats
    assert st["plans"] == 1 and st["hits"] >= (1 if graph else 3), st
    if graph:
        assert job.graph_stats["replays"] >= 2
    job.close()


def test_autograd_cached_transpose_reuses_its_plan(device):
    rng = np.random.default_rng(640)
    m, k, n = 30_000, 20_000, 32
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 600_000, k, rng), rng)
    d_rp, d_ci, d_v = rp.to(device), ci.to(device), v.to(device)  # constant edge weights
    fs.autograd.TRANSPOSE_CACHE.__init__()
    grads = []
    s0 = None
    for step in range(4):
        b = random_dense(k, n, rng)
        db = b.to(device).requires_grad_(True)
        out = fs.spmm(d_rp, d_ci, d_v, m, k, db)
        g = random_dense(m, n, rng)
        out.backward(g.to(device))
        torch.cuda.synchronize()
        grads.append((g, db.grad.cpu()))
        if step == 1:
            s0 = _C.static_plans()  # steps 0-1: first sight of the values, then the gathered copy
    st = counters(s0, _C.static_plans())
    assert st["plans"] == 0 and st["hits"] == 2, st
    # d(b) = A^T @ g, against the oracle on the transposed CSR (rows of A ascending in each row)
    import scipy.sparse as sp
    at = sp.csr_matrix((v.numpy(), ci.numpy(), rp.numpy()), shape=(m, k)).T.tocsr()
    at.sort_indices()
    at_rp = torch.from_numpy(at.indptr.astype(np.int32))
    at_ci = torch.from_numpy(at.indices.astype(np.int32))
    at_v = torch.from_numpy(at.data.astype(np.float32))
    for g, gb in grads:
        assert_bitwise(gb, oracle_spmm(at_rp, at_ci, at_v, g), "d(b)")


def test_plans_past_the_cap_evict_the_least_recently_used(device):
    """The eager state keeps at most 8 plans (SpmmCsrPlanState::kMaxPlans): a ninth static CSR
    evicts the least recently used one, after the device drains; an evicted CSR plans again on
    its next call, and every call stays exact."""
    rng = np.random.default_rng(650)
    m, k, n = 40_000, 40_000, 16
    graphs = []
    for i in range(10):
        rp, ci, v = random_csr(m, k, hub_graph(m, k, rng, hubs=((i, 3000),)), rng)
        graphs.append((rp, ci, v, [rp.to(device), ci.to(device), v.to(device)]))
    b = random_dense(k, n, rng)
    db = b.to(device)
    s0 = _C.static_plans()
    for i, (rp, ci, v, d) in enumerate(graphs):
        out = fs.spmm(*d, m, k, db, static_csr=100 + i)
        assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b), f"graph {i}")
    st = _C.static_plans()
    assert counters(s0, st) == {"plans": 10, "hits": 0}
    assert st["entries"] == 8, st
    rp, ci, v, d = graphs[0]  # evicted: plans again
    out = fs.spmm(*d, m, k, db, static_csr=100)
    assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b), "graph 0 again")
    rp, ci, v, d = graphs[9]  # resident: a hit
    out = fs.spmm(*d, m, k, db, static_csr=109)
    torch.cuda.synchronize()
    assert counters(st, _C.static_plans()) == {"plans": 1, "hits": 1}
    assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b), "graph 9 again")


@pytest.mark.concurrent_streams
def test_each_stream_keeps_its_own_plan(device):
    """The hub reduce's arrival counters live in the plan workspace, so an eager static CSR used
    on two streams gets a plan per stream; both streams' results are exact."""
    rng = np.random.default_rng(660)
    m, k, n = 40_000, 40_000, 32
    rp, ci, v = random_csr(m, k, hub_graph(m, k, rng), rng)
    b = random_dense(k, n, rng)
    d = [rp.to(device), ci.to(device), v.to(device)]
    db = b.to(device)
    ref = oracle_spmm(rp, ci, v, b)
    streams = [torch.cuda.Stream(device) for _ in range(2)]
    s0 = _C.static_plans()
    outs = []
    for rep in range(2):
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                outs.append(fs.spmm(*d, m, k, db, static_csr=11))
    torch.cuda.synchronize()
    assert counters(s0, _C.static_plans()) == {"plans": 2, "hits": 2}
    for i, o in enumerate(outs):
        assert_bitwise(o.cpu(), ref, f"call {i}")


@pytest.mark.graph_capture
def test_a_captured_plan_outlives_eviction(device):
    """A graph that captured a static call holds the plan's workspace, so the state pins it: ten
    other static CSRs afterwards evict only unpinned plans, and the graph still replays exact."""
    rng = np.random.default_rng(670)
    m, k, n = 40_000, 40_000, 32
    rp, ci, v = random_csr(m, k, hub_graph(m, k, rng), rng)
    b = random_dense(k, n, rng)
    d = [rp.to(device), ci.to(device), v.to(device)]
    db = b.to(device)
    out = torch.empty((m, n), device=device)
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        fs.spmm(*d, m, k, db, out=out, static_csr=21)  # plans, outside the capture
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fs.spmm(*d, m, k, db, out=out, static_csr=21)  # a hit: the entry is pinned
    others = []
    for i in range(10):
        o_rp, o_ci, o_v = random_csr(m, k, hub_graph(m, k, rng, hubs=((i, 2500),)), rng)
        others.append([o_rp.to(device), o_ci.to(device), o_v.to(device)])
        fs.spmm(*others[-1], m, k, db, static_csr=300 + i)
    torch.cuda.synchronize()
    assert _C.static_plans()["entries"] == 8
    for i in range(2):
        b2 = random_dense(k, n, rng)
        db.copy_(b2.to(device))
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert_bitwise(out.cpu(), oracle_spmm(rp, ci, v, b2), f"replay {i} after evictions")
    del g
    torch.cuda.synchronize()


def test_autograd_learnable_values_reuse_the_transpose_plan(device):
    """Learnable edge weights (new values every step) take the gathered d(b) op over the cached
    A^T; its plan is kept across steps like the constant-values path's, and d(b) stays exact."""
    rng = np.random.default_rng(680)
    m, k, n = 30_000, 20_000, 32
    rp, ci, _ = random_csr(m, k, power_law_degrees(m, 600_000, k, rng), rng)
    d_rp, d_ci = rp.to(device), ci.to(device)
    fs.autograd.TRANSPOSE_CACHE.__init__()
    keep, grads, s0 = [], [], None
    for step in range(4):
        v = torch.from_numpy(rng.uniform(-1, 1, ci.numel()).astype(np.float32))
        dv = v.to(device).requires_grad_(True)  # new values each step: the gathered op
        keep.append(dv)  # distinct storage per step
        db = random_dense(k, n, rng).to(device).requires_grad_(True)
        out = fs.spmm(d_rp, d_ci, dv, m, k, db)
        g = random_dense(m, n, rng)
        out.backward(g.to(device))
        torch.cuda.synchronize()
        grads.append((v, g, db.grad.cpu()))
        if step == 0:
            s0 = _C.static_plans()  # step 0 built A^T and the gathered op's plan
    st = counters(s0, _C.static_plans())
    assert st["plans"] == 0 and st["hits"] == 3, st
    import scipy.sparse as sp
    for v, g, gb in grads:
        at = sp.csr_matrix((v.numpy(), ci.numpy(), rp.numpy()), shape=(m, k)).T.tocsr()
        at.sort_indices()
        assert_bitwise(gb, oracle_spmm(torch.from_numpy(at.indptr.astype(np.int32)),
                                       torch.from_numpy(at.indices.astype(np.int32)),
                                       torch.from_numpy(at.data.astype(np.float32)), g), "d(b)")


def test_sddmm_static_plans_once(device):
    """Op sddmm_csr with static_csr: its own kernel state plans the CSR once (hub rows: a real
    work list); every call keeps the oracle's bits."""
    from oracle import oracle
    rng = np.random.default_rng(690)
    m, k, n = 30_000, 20_000, 64
    rp, ci, _ = random_csr(m, k, power_law_degrees(m, 600_000, k, rng), rng)
    a = random_dense(m, n, rng)
    b = random_dense(k, n, rng)
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), a.numpy(), b.numpy())
    d_rp, d_ci, da, db = rp.to(device), ci.to(device), a.to(device), b.to(device)
    s0 = _C.static_plans()
    outs = [_C.sddmm_csr(d_rp, d_ci, da, db, m, k, static_csr=31) for _ in range(3)]
    torch.cuda.synchronize()
    assert counters(s0, _C.static_plans()) == {"plans": 1, "hits": 2}
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"call {i}"


def test_static_training_step_plans_each_op_once(device):
    """A training step of a static graph with learnable edge weights: the forward SpMM, the
    backward SDDMM (d values) and the gathered A^T SpMM (d b) each plan once, then reuse."""
    from oracle import oracle
    rng = np.random.default_rng(700)
    m, k, n = 30_000, 20_000, 32
    rp, ci, _ = random_csr(m, k, power_law_degrees(m, 600_000, k, rng), rng)
    d_rp, d_ci = rp.to(device), ci.to(device)
    fs.autograd.TRANSPOSE_CACHE.__init__()
    keep, s0 = [], None
    for step in range(4):
        v = torch.from_numpy(rng.uniform(-1, 1, ci.numel()).astype(np.float32))
        dv = v.to(device).requires_grad_(True)
        keep.append(dv)
        b = random_dense(k, n, rng)
        db = b.to(device).requires_grad_(True)
        out = fs.spmm(d_rp, d_ci, dv, m, k, db, static_csr=41)
        g = random_dense(m, n, rng)
        out.backward(g.to(device))
        torch.cuda.synchronize()
        if step == 0:
            s0 = _C.static_plans()
        ref_dv = oracle.sddmm(rp.numpy(), ci.numpy(), g.numpy(), b.numpy())
        assert np.array_equal(dv.grad.cpu().numpy().view(np.uint32), ref_dv.view(np.uint32)), \
            f"d(values) step {step}"
        assert_bitwise(out.detach().cpu(), oracle_spmm(rp, ci, v, b), f"forward step {step}")
    st = counters(s0, _C.static_plans())
    assert st == {"plans": 0, "hits": 9}, st  # 3 ops x 3 later steps
