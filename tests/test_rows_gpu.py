"""ofx_gather_rows (the halo pack kernel, csrc/rows.hip): dst[i] = src[idx[i]] byte-exact against
torch.index_select, for 16-B, 4-B and 1-B word paths, strided rows and both index dtypes."""
import numpy as np
import pytest
import torch

from oneflow_spmm._C import current_stream_handle, dtype_code
from oneflow_spmm._lib import LIB, check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("n,dtype,pad", [(128, torch.float32, 0), (3, torch.float32, 0),
                                         (7, torch.bfloat16, 0), (64, torch.float32, 5),
                                         (1, torch.bfloat16, 3), (300, torch.float64, 0)])
def test_gather_rows_matches_index_select(device, idx_dtype, n, dtype, pad):
    rng = np.random.default_rng(n + pad)
    k, count = 5000, 3333
    src_full = torch.from_numpy(rng.standard_normal((k, n + pad))).to(dtype).to(device)
    src = src_full[:, :n]
    idx = torch.from_numpy(rng.integers(0, k, count)).to(idx_dtype).to(device)
    dst_full = torch.full((count, n + pad), 7, dtype=dtype, device=device)
    dst = dst_full[:, :n]
    esz = src.element_size()
    check(LIB.ofx_gather_rows(current_stream_handle(src), dtype_code(idx_dtype), count, n * esz,
                              idx.data_ptr(), src.data_ptr(), src.stride(0) * esz, dst.data_ptr(),
                              dst.stride(0) * esz), "gather_rows")
    torch.cuda.synchronize()
    want = torch.index_select(src, 0, idx.long())
    assert torch.equal(dst.contiguous().view(torch.uint8), want.contiguous().view(torch.uint8))
    if pad:
        assert (dst_full[:, n:] == 7).all()  # row padding untouched


def test_gather_rows_empty_and_errors(device):
    x = torch.zeros(4, 4, device=device)
    check(LIB.ofx_gather_rows(None, dtype_code(torch.int64), 0, 16, None, None, 16, None, 16), "empty")
    assert LIB.ofx_gather_rows(None, dtype_code(torch.float32), 1, 16, x.data_ptr(), x.data_ptr(),
                               16, x.data_ptr(), 16) != 0
    assert LIB.ofx_gather_rows(None, dtype_code(torch.int64), 1, 32, x.data_ptr(), x.data_ptr(),
                               16, x.data_ptr(), 16) != 0  # stride < row


@pytest.mark.parametrize("k,world", [(2449029, 8), (999, 2), (1000, 4), (7, 3), (5, 8)])
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
def test_device_padded_remap_matches_host(device, k, world, idx_dtype):
    from oneflow_spmm.distributed import padded_owner_remap
    rng = np.random.default_rng(k)
    col = torch.from_numpy(rng.integers(0, k, 20000)).to(idx_dtype)
    out = torch.empty_like(col, device=device)
    d = col.to(device)
    check(LIB.ofx_padded_owner_remap(None, dtype_code(idx_dtype), col.numel(), k, world,
                                     d.data_ptr(), out.data_ptr()), "remap")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), padded_owner_remap(col, k, world))


@pytest.mark.parametrize("S,C,rows,w,dtype", [(1, 1, 7, 16, torch.float32), (2, 4, 33, 8, torch.float32),
                                             (2, 2, 100, 3, torch.float32), (3, 2, 5, 5, torch.bfloat16),
                                             (1, 8, 1000, 16, torch.float64), (2, 3, 0, 4, torch.float32)])
def test_copy_blocks_pack_and_unpack(device, S, C, rows, w, dtype):
    """ofx_copy_blocks as the grid exchange uses it: a shard [rows, S*C*w] packed into
    [S][C][rows][w] (block b, sub-block s = columns b*S*w + s*w), then unpacked back into a
    row-major [rows, N] output with a padded leading dimension; 16-B, 4-B and 1-B word paths."""
    import ctypes
    from oneflow_spmm._C import current_stream_handle
    from oneflow_spmm._lib import LIB, check
    n = S * C * w
    e = torch.empty(0, dtype=dtype).element_size()
    shard = torch.randn(rows, n + 3, device=device).to(dtype)[:, :n]  # leading dim n + 3
    packed = torch.full((S, C, rows, w), 7, dtype=dtype, device=device)
    st = current_stream_handle(shard)
    check(LIB.ofx_copy_blocks(st, S, C, rows, w * e, shard.data_ptr(), w * e, S * w * e,
                              shard.stride(0) * e, packed.data_ptr(), C * rows * w * e,
                              rows * w * e, w * e), "copy_blocks")
    ref = torch.stack([torch.stack([shard[:, b * S * w + s * w: b * S * w + (s + 1) * w]
                                    for b in range(C)]) for s in range(S)])
    assert torch.equal(packed, ref)
    out = torch.zeros(rows, n + 5, dtype=dtype, device=device)
    check(LIB.ofx_copy_blocks(st, S, C, rows, w * e, packed.data_ptr(), C * rows * w * e,
                              rows * w * e, w * e, out.data_ptr(), w * e, S * w * e,
                              out.stride(0) * e), "copy_blocks")
    torch.cuda.synchronize()
    assert torch.equal(out[:, :n], shard) and (out[:, n:] == 0).all()
