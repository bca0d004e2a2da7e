import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "of-spmm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: full BASELINE-size problems")
    config.addinivalue_line("markers", "graph_capture: captures launches into a hipGraph (not run "
                                       "under the bounds-checked library)")
    config.addinivalue_line("markers", "concurrent_streams: launches run concurrently on several "
                                       "streams (not run under the bounds-checked library)")
    # GPU calls (scripts/gpu_run.sh): a fatal signal's thread dump also goes to a file that
    # survives pytest's output capture (the r03ai abort's messages were lost)
    path = os.environ.get("OFX_FAULTHANDLER_FILE")
    if path:
        import faulthandler
        global _FAULT_FILE
        _FAULT_FILE = open(path, "a")
        faulthandler.enable(file=_FAULT_FILE, all_threads=True)


_FAULT_FILE = None


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _debug_bounds_guard(request):
    """With OFX_DEBUG_BOUNDS_CHECK=1 and a bounds-checked library (OFX_SPMM_LIB=...libofx_spmm_dbg.so,
    csrc/dbg_bounds.h), every test fails if any forward launch it made touched memory outside its
    allocations (the access itself was skipped, so nothing faulted): the site, address, block and
    launch configuration are in the message."""
    if os.environ.get("OFX_DEBUG_BOUNDS_CHECK") != "1" or "gpu" not in request.keywords:
        yield
        return
    if "graph_capture" in request.keywords:
        # csrc/dbg_bounds.h publishes each launch's allocation table with a host-to-device copy
        # of a host stack object; a graph capture records that copy and replays it from memory
        # that is gone, so captured launches are outside what this instrument can check
        pytest.skip("graph capture: the bounds-checked library's per-launch table is not capturable")
    if "concurrent_streams" in request.keywords:
        # the table is one device global per translation unit, rewritten before every launch:
        # launches overlapping on two streams would read each other's allocations
        pytest.skip("concurrent streams: the bounds-checked library keeps one launch table")
    import ctypes
    from oneflow_spmm import _lib
    out = (ctypes.c_uint64 * 8)()
    _lib.LIB.ofx_debug_bounds_read(out, 1)  # clear
    yield
    rc = _lib.LIB.ofx_debug_bounds_read(out, 1)
    assert rc == _lib.OFX_OK, _lib.last_error()
    if out[0]:
        site = int(out[1])
        raise AssertionError(
            f"out-of-allocation access ({int(out[0])} in this test): site "
            f"{['?', 'spmm_csr_impl.h', 'spmm_plan.h'][site // 100000]}:{site % 100000}, address "
            f"{int(out[2]):#x}, {int(out[3])} B, block {int(out[4])}, thread {int(out[5])}, "
            f"launch tag {int(out[6]):#x}")
