"""The kHIP collectives of the OneFlow mirror on the GPU (world size 1 on the one-GPU box; RCCL
refuses two ranks on one GPU): eager boxing ccl-s-to-b through op eager_ccl_all_gather and
HipAllGather (RCCL communicator from EagerRcclCommMgr), the lazy graph's
_nccl_logical_all_gather kernel, and the compiled row-split job (bit-exact vs the oracle, and
replayed from a hipGraph capture)."""
import numpy as np
import pytest
import torch

from oneflow_spmm import ccl
from oneflow_spmm.ccl import PlacementSpec
from tests.helpers import assert_bitwise, oracle_spmm, power_law_degrees, random_csr, random_dense

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip_placement(device):
    ccl.install_control_plane()
    return PlacementSpec("hip", 1, 0, (0,), (device.index or 0,))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.int64])
def test_eager_ccl_s2b_on_hip(device, hip_placement, dt):
    x = (torch.arange(77 * 9, dtype=torch.float64).reshape(77, 9) - 100).to(dt).to(device)
    out = ccl.ccl_s2b(x, hip_placement, 77)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().view(torch.uint8), x.cpu().view(torch.uint8))


def test_nccl_logical_all_gather_on_hip(device, hip_placement):
    x = torch.randn(123, 64, device=device)
    out = ccl.nccl_logical_all_gather(x, hip_placement, stream_name="spmm")
    torch.cuda.synchronize()
    assert torch.equal(out, x)


@pytest.mark.graph_capture
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_spmm_job_on_hip_bitexact_and_graph_replay(device, hip_placement, dt):
    rng = np.random.default_rng(31)
    m, k, n = 5000, 4000, 128
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 150000, k, rng), rng, val_dtype=dt)
    b1, b2 = random_dense(k, n, rng, dt), random_dense(k, n, rng, dt)
    job = ccl.SpmmJob(hip_placement, m, k, n, ci.numel(), torch.int32, dt, device)
    assert "no boxing" in job.plan
    d = (rp.to(device), ci.to(device), v.to(device))
    b = b1.to(device)
    out = job(*d, b)
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b1), "job run")
    # compile once, capture the run into a hipGraph, replay on a new b
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        job(*d, b, out=out)
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        job(*d, b, out=out)
    b.copy_(b2.to(device))
    out.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b2), "graph replay")


@pytest.mark.graph_capture
@pytest.mark.parametrize("stream_kind", ["default", "side"])
def test_spmm_job_native_graph_mode(device, hip_placement, stream_kind):
    """The job's own graph mode (UserKernel::ForwardUserKernel's CUDA-graph branch,
    user_kernel.cpp:676-707, over the C-ABI's hipGraph executable): run 1 eager, run 2 captured
    and launched, later runs with the same tensors one graph launch each, new tensors re-capture
    (an in-place executable update); every result bit-exact vs the oracle, on the null stream
    and on a side stream."""
    rng = np.random.default_rng(37)
    m, k, n = 3000, 2500, 64
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 60000, k, rng), rng)
    bs = [random_dense(k, n, rng) for _ in range(3)]
    job = ccl.SpmmJob(hip_placement, m, k, n, ci.numel(), torch.int32, torch.float32, device,
                      graph=True)
    d = (rp.to(device), ci.to(device), v.to(device))
    b = bs[0].to(device)
    out = torch.empty((m, n), device=device)
    stream = torch.cuda.current_stream(device) if stream_kind == "default" \
        else torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        job(*d, b, out=out)                      # eager (IsReadyForCapture after the first run)
        assert job.graph_stats["captures"] == 0
        job(*d, b, out=out)                      # captured + launched
        stream.synchronize()
        assert_bitwise(out, oracle_spmm(rp, ci, v, bs[0]), "captured run")
        for i in (1, 2):                         # replays read the new contents of b
            b.copy_(bs[i].to(device))
            out.fill_(float("nan"))
            job(*d, b, out=out)
            stream.synchronize()
            assert_bitwise(out, oracle_spmm(rp, ci, v, bs[i]), f"replay {i}")
        assert job.graph_stats == {"captures": 1, "replays": 2, "updates": 0}
        out2 = torch.empty_like(out)             # new address: re-capture, executable updated
        job(*d, b, out=out2)
        job(*d, b, out=out2)
        stream.synchronize()
        assert_bitwise(out2, oracle_spmm(rp, ci, v, bs[2]), "re-captured run")
        assert job.graph_stats == {"captures": 2, "replays": 3, "updates": 1}
