"""The thin device layer of the C-ABI (ep::Device / Stream / Event and the
Memcpy / Memset primitives, include/ofx_spmm.h "thin device layer"), driven from the host the
way a OneFlow ep::hip backend or a non-Python host would: allocate, fill, copy both ways on a
created stream, order two streams with an event, time with events, an SpMM launched on the
shim's own stream with shim-allocated buffers, and the error paths."""
import ctypes

import numpy as np
import pytest
import torch

from oneflow_spmm._lib import LIB, OFX_OK

pytestmark = pytest.mark.gpu

H2D, D2H, D2D = 1, 2, 3
p = ctypes.c_void_p


def ok(rc):
    assert rc == OFX_OK, LIB.ofx_last_error().decode()


def test_device_stream_event_memcpy_memset(device):
    cnt, cur = ctypes.c_int(0), ctypes.c_int(-1)
    ok(LIB.ofx_device_count(ctypes.byref(cnt)))
    assert cnt.value >= 1
    ok(LIB.ofx_set_device(0))
    ok(LIB.ofx_get_device(ctypes.byref(cur)))
    assert cur.value == 0
    nbytes = 1 << 20
    d_a, d_b, h = p(), p(), p()
    ok(LIB.ofx_malloc(ctypes.byref(d_a), nbytes))
    ok(LIB.ofx_malloc(ctypes.byref(d_b), nbytes))
    ok(LIB.ofx_host_malloc(ctypes.byref(h), nbytes))
    assert d_a.value % 512 == 0 and d_b.value % 512 == 0  # ep::kMaxAlignmentRequirement
    s1, s2 = p(), p()
    ok(LIB.ofx_stream_create(ctypes.byref(s1)))
    ok(LIB.ofx_stream_create(ctypes.byref(s2)))
    e0, e1, ev = p(), p(), p()
    ok(LIB.ofx_event_create(ctypes.byref(e0), 1))
    ok(LIB.ofx_event_create(ctypes.byref(e1), 1))
    ok(LIB.ofx_event_create(ctypes.byref(ev), 0))
    host = (ctypes.c_uint8 * nbytes).from_address(h.value)
    src = np.random.default_rng(0).integers(0, 256, nbytes, dtype=np.uint8)
    np.frombuffer(host, dtype=np.uint8)[:] = src
    ok(LIB.ofx_event_record(e0, s1))
    ok(LIB.ofx_memcpy_async(s1, d_a, h, nbytes, H2D))        # host -> a
    ok(LIB.ofx_memset_async(s1, d_b, 0x5A, nbytes))          # b = 0x5A
    ok(LIB.ofx_event_record(ev, s1))
    ok(LIB.ofx_stream_wait_event(s2, ev))                    # s2 after a and b are written
    ok(LIB.ofx_memcpy_async(s2, d_b, d_a, nbytes // 2, D2D))  # first half of b = a
    ok(LIB.ofx_memcpy_async(s2, h, d_b, nbytes, D2H))
    ok(LIB.ofx_event_record(e1, s2))
    ok(LIB.ofx_stream_sync(s2))
    ok(LIB.ofx_event_sync(e1))
    got = np.frombuffer(host, dtype=np.uint8).copy()
    assert np.array_equal(got[: nbytes // 2], src[: nbytes // 2])
    assert (got[nbytes // 2:] == 0x5A).all()
    ms = ctypes.c_float(-1)
    ok(LIB.ofx_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
    assert ms.value >= 0
    ok(LIB.ofx_device_synchronize())
    for e in (e0, e1, ev):
        ok(LIB.ofx_event_destroy(e))
    for s in (s1, s2):
        ok(LIB.ofx_stream_destroy(s))
    ok(LIB.ofx_free(d_a))
    ok(LIB.ofx_free(d_b))
    ok(LIB.ofx_host_free(h))


def test_spmm_on_shim_stream_and_buffers(device):
    """ofx_spmm_csr with every buffer from ofx_malloc and the launch on an ofx_stream_create
    stream (no torch involved): bit-exact against the oracle."""
    from oracle import oracle
    from oneflow_spmm import ops
    rng = np.random.default_rng(3)
    m, k, n = 500, 400, 32
    deg = rng.integers(0, 30, size=m)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(k, d, replace=False)) for d in deg]).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1]).astype(np.float32)
    b = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    s = p()
    ok(LIB.ofx_stream_create(ctypes.byref(s)))
    bufs = {}
    for name, arr in (("rp", rp), ("ci", ci), ("v", v), ("b", b)):
        d = p()
        ok(LIB.ofx_malloc(ctypes.byref(d), max(arr.nbytes, 1)))
        ok(LIB.ofx_memcpy_async(s, d, arr.ctypes.data, arr.nbytes, H2D))
        bufs[name] = d
    d_c = p()
    ok(LIB.ofx_malloc(ctypes.byref(d_c), m * n * 4))
    ws_bytes = ops.workspace_size(torch.int32, torch.float32, m, k, n, len(ci))
    d_ws = p()
    ok(LIB.ofx_malloc(ctypes.byref(d_ws), max(ws_bytes, 1)))
    ok(LIB.ofx_spmm_csr(s, 5, 2, m, k, n, len(ci), bufs["rp"], bufs["ci"], bufs["v"], bufs["b"], n,
                        d_c, n, 0, m, d_ws, ws_bytes, None))
    out = np.empty((m, n), dtype=np.float32)
    ok(LIB.ofx_memcpy_async(s, out.ctypes.data, d_c, out.nbytes, D2H))
    ok(LIB.ofx_stream_sync(s))
    ref = oracle.spmm(rp, ci, v, b)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    for d in list(bufs.values()) + [d_c, d_ws]:
        ok(LIB.ofx_free(d))
    ok(LIB.ofx_stream_destroy(s))


def test_shim_errors(device):
    assert LIB.ofx_set_device(1 << 20) != OFX_OK
    assert LIB.ofx_malloc(None, 16) != OFX_OK
    assert LIB.ofx_memcpy_async(None, None, None, 16, 99) != OFX_OK
    assert len(LIB.ofx_last_error()) > 0
    # a reported HIP failure does not resurface at the next launch's error check
    from oneflow_spmm import _C
    x = torch.ones(4, 8, device=device)
    rp = torch.tensor([0, 1, 1, 2, 2], dtype=torch.int32, device=device)
    ci = torch.tensor([0, 3], dtype=torch.int32, device=device)
    v = torch.tensor([2.0, 3.0], device=device)
    assert LIB.ofx_set_device(1 << 20) != OFX_OK
    out = _C.spmm_csr(rp, ci, v, 4, 4, x)
    torch.cuda.synchronize()
    assert out[0].eq(2).all() and out[2].eq(3).all() and out[1].eq(0).all()
