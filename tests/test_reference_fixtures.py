"""Parity against the reference's OWN golden vectors (tests/golden/ref_embedding_scale_by_freq.npz,
extracted from python/oneflow/test/modules/test_sparse.py:76-134 by
tests/golden/make_reference_fixtures.py).

The reference has no SpMM, but its embedding test pins the two CPU building blocks the SpMM
composition is made of, with literal inputs and expected outputs:
  * forward = EmbeddingFunctor<kCPU> (oneflow/user/kernels/embedding_kernel_util.cpp:48-60), the
    row gather of gather_kernel_util.cpp:72-92.  As an SpMM: A is the [8 x 10] one-hot CSR of
    the indices (values 1), and A @ weight must be the test's expected output.
  * backward = EmbeddingGradFunctor<kCPU> (:63-88): dx[indices[i]] = dy[i] + dx[indices[i]] for i
    ascending (std::plus: the segment sum of unsorted_segment_sum_kernel_util.cpp:29-45), then
    each row divided by its index's frequency when > 1 (scale_grad_by_freq).  As an SpMM: A^T
    @ dy with A^T's rows listing i ascending (the stable transpose), dy = ones (the gradient of
    y.sum()); the frequency division is the test's own step, applied here as the reference does.
Checked for the oracle, the kCPU kernel, the op layer's autograd and (on a GPU) the HIP kernel,
bit for bit, and with the reference test's tolerance (allclose 1e-5).  The fixture's values make
every sum exact, so it pins WHICH rows are gathered and summed where; the rounding order of
longer sums is pinned by the restatement (tests/test_oracle.py) and the scipy fixtures."""
import os

import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import ops
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "ref_embedding_scale_by_freq.npz")


@pytest.fixture(scope="module")
def fx():
    d = np.load(GOLDEN)  # allow_pickle=False: plain arrays only
    idx = d["indices"].reshape(-1).astype(np.int64)
    n_rows, emb = d["weight"].shape
    rp = np.arange(idx.size + 1, dtype=np.int32)  # one nonzero per output row
    return dict(weight=d["weight"], idx=idx, output=d["output"].reshape(idx.size, -1),
                weight_grad=d["weight_grad"], rp=rp, ci=idx.astype(np.int32),
                vals=np.ones(idx.size, np.float32), m=idx.size, k=n_rows, emb=emb)


def scale_by_freq(grad: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """The reference's frequency step (embedding_kernel_util.cpp:77-86): rows whose index occurs
    more than once are divided by the count, in T."""
    out = grad.copy()
    freq = np.bincount(idx, minlength=grad.shape[0])
    for r in range(grad.shape[0]):
        if freq[r] > 1:
            out[r] = (out[r] / np.float32(freq[r])).astype(np.float32)
    return out


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                                                 np.ascontiguousarray(b).view(np.uint32))


def test_fixture_is_the_reference_test():
    """The arrays are the test's literals: the expected forward is the gathered rows of weight,
    and the expected gradient counts each index once after the frequency scale."""
    d = np.load(GOLDEN)
    assert d["weight"].shape == (10, 3) and d["indices"].shape == (2, 4)
    assert d["output"].shape == (2, 4, 3) and d["weight_grad"].shape == (10, 3)
    assert "test_sparse.py:76" in str(d["source"])


def test_oracle_gather_matches_reference_forward(fx):
    c = oracle.spmm(fx["rp"], fx["ci"], fx["vals"], fx["weight"])
    assert same_bits(c, fx["output"])
    assert np.allclose(c, fx["output"], 1e-5, 1e-5)


def test_oracle_segment_sum_matches_reference_backward(fx):
    rp_t, ci_t, perm = oracle.transpose(fx["rp"], fx["ci"], fx["k"])
    dy = np.ones((fx["m"], fx["emb"]), np.float32)  # d(y.sum()) / dy
    seg = oracle.spmm(rp_t, ci_t, fx["vals"][perm], dy)  # dx[idx[i]] += dy[i], i ascending
    got = scale_by_freq(seg, fx["idx"])
    assert same_bits(got, fx["weight_grad"])
    assert np.allclose(got, fx["weight_grad"], 1e-5, 1e-5)


def _devices():
    yield "cpu"
    yield pytest.param("cuda", marks=pytest.mark.gpu)


@pytest.mark.parametrize("dev", list(_devices()))
def test_operator_matches_reference_forward_and_backward(fx, dev):
    """The op (kCPU or HIP kernel) and its autograd reproduce the reference's embedding test:
    out = A @ weight is its forward; d(weight) of out.sum() is its backward before the
    frequency scale."""
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    rp = torch.from_numpy(fx["rp"]).to(dev)
    ci = torch.from_numpy(fx["ci"]).to(dev)
    v = torch.from_numpy(fx["vals"]).to(dev)
    w = torch.from_numpy(fx["weight"]).to(dev).requires_grad_(True)
    out = fs.spmm(rp, ci, v, fx["m"], fx["k"], w)
    out.sum().backward()
    if dev == "cuda":
        torch.cuda.synchronize()
    got_out = out.detach().cpu().numpy()
    got_grad = scale_by_freq(w.grad.cpu().numpy(), fx["idx"])
    assert same_bits(got_out, fx["output"])
    assert same_bits(got_grad, fx["weight_grad"])
    # the device kernel without the op layer, too
    if dev == "cuda":
        c = ops.spmm_csr_device(rp, ci, v, w.detach(), fx["m"], fx["k"])
        torch.cuda.synchronize()
        assert same_bits(c.cpu().numpy(), fx["output"])
