"""oracle.py — ctypes/numpy front end of the CPU SpMM restatement (spmm_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the *checker*; the product package (of-spmm_amd/oneflow_spmm) never imports
it.  Parity status: the reference has no SpMM and no test pinning one.  Its
two building blocks ARE pinned by the reference's own golden vectors: the embedding test
python/oneflow/test/modules/test_sparse.py:76-134 holds literal inputs and expected outputs of
EmbeddingFunctor<kCPU> (the row gather) and EmbeddingGradFunctor<kCPU> (the index-order segment
sum), oneflow/user/kernels/embedding_kernel_util.cpp:48-88, and tests/test_reference_fixtures.py
checks this oracle (and the kernels) against them bit for bit
(tests/golden/ref_embedding_scale_by_freq.npz, extracted by make_reference_fixtures.py).  Those
sums are exact, so the rounding order of longer sums is pinned by restatement only, and
cross-validated against scipy.sparse and torch.sparse_csr (tests/golden/make_golden.py,
tests/test_oracle.py): "parity partially pinned".

Semantics (see spmm_oracle.c header for the reference file:line anchors):
  C[r, :] = sum_{j in row r, ascending} val[j] * B[col[j], :]   from +0, multiply then add.
16-bit types are carried as numpy uint16 bit patterns (bf16) / float16.  Each product is rounded
to the 16-bit type (the multiply's output tensor has that dtype: BinaryFunctor<kMul> is
`static_cast<Dst>(src0 * src1)`, oneflow/core/ep/common/primitive/binary_functor.h:46-51), the
products are summed in fp32 and the sum is rounded once at the end
(oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:146-205).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
INT64_MAX = (1 << 63) - 1


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "spmm_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        i64, p, c_int = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
        base = [i64, i64, i64, p, p, p, p, i64, p, i64, i64, i64, i64, i64, c_int]
        _LIB.orc_spmm_f64.argtypes = base + [c_int]  # + neg_zero
        _LIB.orc_spmm_f32.argtypes = base + [c_int, c_int]  # + round16, neg_zero
        _LIB.orc_round16.argtypes = [p, i64, c_int]
        _LIB.orc_spmm_f32_ref64.argtypes = [i64, p, p, p, p, i64, p, p, i64, i64, c_int, i64]
        _LIB.orc_balanced_range.argtypes = [i64, i64, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    return _LIB


def default_split(n: int) -> int:
    """Restates the operator's documented default hub-row threshold:
    T = clamp(65536 // n, 128, 512) rounded down to a power of two (the cap was 8192 before
    round 3)."""
    t = 65536 // n if n > 0 else 512
    t = min(max(t, 128), 512)
    p = 128
    while p * 2 <= t:
        p *= 2
    return p


def balanced_range(total: int, parts: int, idx: int) -> tuple[int, int]:
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    lib().orc_balanced_range(total, parts, idx, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


# ---- 16-bit helpers ------------------------------------------------------------------------
def bf16_bits_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even; NaN stays NaN."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


_ROUND16 = {"f32": 0, "bf16": 1, "f16": 2}


def round16(x: np.ndarray, dtype: str) -> np.ndarray:
    """fp32 values rounded to bf16/f16 as the multiply rounds its products (returned as fp32)."""
    y = np.array(x, dtype=np.float32, copy=True, order="C")
    lib().orc_round16(_p(y), y.size, _ROUND16[dtype])
    return y


def _schedule(n, split, chunk, ordered):
    if ordered:
        return INT64_MAX, INT64_MAX
    s = split if split and split > 0 else default_split(n)
    c = chunk if chunk and chunk > 0 else s
    return s, min(c, s)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def spmm(row_ptr, col_idx, values, b, *, dtype="f32", row_begin=0, row_end=None, split=0, chunk=0,
         ordered=False, nthreads=None, k=None, negative="error"):
    """Oracle SpMM.  dtype in {"f32","f64","bf16","f16"}; bf16 arrays are uint16 bit patterns.
    Returns C rows [row_begin, row_end) in the storage dtype (bf16 -> uint16 bits).
    A column >= k gathers a zero-filled row (gather_kernel_util.cpp:84-89: the nonzero adds
    val * 0).  A negative column raises (the CPU gather's CHECK_GE, :80) unless
    negative="zero": the CUDA gather's semantics (gather_kernel_util.cu:36), the device kernel's."""
    m = len(row_ptr) - 1
    row_end = m if row_end is None else row_end
    n = b.shape[1]
    k = b.shape[0] if k is None else k
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    ci = np.ascontiguousarray(col_idx, dtype=np.int64)
    s, c = _schedule(n, split, chunk, ordered)
    nt = nthreads or min(os.cpu_count() or 1, 16)
    rows = row_end - row_begin
    if dtype == "f64":
        v = np.ascontiguousarray(values, dtype=np.float64)
        bb = np.ascontiguousarray(b, dtype=np.float64)
        out = np.zeros((rows, n), dtype=np.float64)
        rc = lib().orc_spmm_f64(m, k, n, _p(rp), _p(ci), _p(v), _p(bb), n, _p(out), n,
                                row_begin, row_end, s, c, nt, int(negative == "zero"))
    else:
        if dtype == "bf16":
            v, bb = bf16_bits_to_f32(np.asarray(values)), bf16_bits_to_f32(np.asarray(b))
        else:
            v = np.asarray(values).astype(np.float32)
            bb = np.asarray(b).astype(np.float32)
        v, bb = np.ascontiguousarray(v), np.ascontiguousarray(bb)
        out = np.zeros((rows, n), dtype=np.float32)
        rc = lib().orc_spmm_f32(m, k, n, _p(rp), _p(ci), _p(v), _p(bb), n, _p(out), n,
                                row_begin, row_end, s, c, nt, _ROUND16.get(dtype, 0),
                                int(negative == "zero"))
    if rc != 0:
        raise ValueError("oracle: negative column index (CHECK_GE(idx, 0))")
    if dtype == "bf16":
        return f32_to_bf16_bits(out)
    if dtype == "f16":
        return out.astype(np.float16)
    return out


def bias_act(out, bias=None, activation="none", *, dtype="f32"):
    """The composition spmm_csr -> bias_add -> relu applied to an oracle SpMM result, each op
    rounding to the storage dtype as the separate OneFlow kernels do:
      bias_add  BroadcastElementwiseBinary kAdd of out[M,N] and bias[1,N,1]-broadcast
                (oneflow/user/kernels/bias_add_kernel.cpp:25-53): one add, one rounding;
      relu      UnaryFunctor<kRelu> (oneflow/core/ep/common/primitive/unary_functor.h:146-156):
                src <= 0 -> 0 (so -0 -> +0), otherwise src (NaN passes).
    bf16 arrays are uint16 bit patterns; the add is done in fp32 and rounded once (exact for
    two 16-bit operands: fp32 holds >= 2p+2 bits, so the double rounding is innocuous)."""
    y = np.array(out, copy=True)
    if bias is not None:
        bias = np.asarray(bias)
        if dtype == "bf16":
            y = f32_to_bf16_bits(bf16_bits_to_f32(y) + bf16_bits_to_f32(bias)[None, :])
        elif dtype == "f16":
            y = (y.astype(np.float32) + bias.astype(np.float32)[None, :]).astype(np.float16)
        else:
            y = y + bias.astype(y.dtype)[None, :]
    if activation == "relu":
        f = bf16_bits_to_f32(y) if dtype == "bf16" else y
        y = np.where(f <= 0, np.zeros_like(y), y)
    elif activation != "none":
        raise ValueError(f"oracle: unknown activation {activation!r}")
    return y


def relu_bias_grad(y, dy, *, relu: bool, dtype="f32"):
    """Backward of the fused epilogue, restating csrc/epilogue_grad.hip (TEST INFRASTRUCTURE):
    dx = relu ? (y > 0 ? dy : 0) : dy   (ReluGrad from the output,
         oneflow/core/autograd/gradient_funcs/activation.cpp:195-205),
    d_bias[j] = sum_i dx[i, j]           (bias_add grad, gradient_funcs/bias_add.cpp:62) in the
    operator's stated order: chunks of 2048 rows summed in row order from +0 in the
    accumulation type, chunk partials in 8 interleaved lanes, lanes combined
    ((l0+l4)+(l2+l6))+((l1+l5)+(l3+l7)), one rounding.  The reference's reduce_sum order is
    its device reduction's, so only this restatement pins the bits.  bf16 = uint16 bits."""
    def to_acc(a):
        if dtype == "bf16":
            return bf16_bits_to_f32(np.asarray(a))
        return np.asarray(a).astype(np.float64 if dtype == "f64" else np.float32)
    acc_t = np.float64 if dtype == "f64" else np.float32
    g = to_acc(dy)
    if relu:
        g = np.where(to_acc(y) > 0, g, acc_t(0)).astype(acc_t)
    m, n = g.shape
    rows, lanes = 2048, 8
    nch = (m + rows - 1) // rows
    part = np.zeros((nch, n), dtype=acc_t)
    for c in range(nch):
        blk = g[c * rows:(c + 1) * rows]
        part[c] = np.cumsum(blk, axis=0, dtype=acc_t)[-1]  # sequential, rounded each step
    lane = np.zeros((lanes, n), dtype=acc_t)
    for l in range(lanes):
        sel = part[l::lanes]
        if len(sel):
            lane[l] = np.cumsum(sel, axis=0, dtype=acc_t)[-1]
    s = lanes // 2
    while s >= 1:
        lane[:s] = (lane[:s] + lane[s:2 * s]).astype(acc_t)
        s //= 2
    def store(a):
        if dtype == "bf16":
            return f32_to_bf16_bits(a.astype(np.float32))
        if dtype == "f16":
            return a.astype(np.float16)
        return a.astype(acc_t)
    return store(g), store(lane[0])


def ref64(row_ptr, col_idx, values_f32, b_f32, *, row_begin=0, row_end=None, nthreads=None):
    """fp64 product C64 and |.|-sum bound of an fp32 (or upcast 16-bit) problem (columns outside
    [0, K) gather a zero row)."""
    m = len(row_ptr) - 1
    row_end = m if row_end is None else row_end
    n = b_f32.shape[1]
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    ci = np.ascontiguousarray(col_idx, dtype=np.int64)
    v = np.ascontiguousarray(values_f32, dtype=np.float32)
    bb = np.ascontiguousarray(b_f32, dtype=np.float32)
    rows = row_end - row_begin
    c64 = np.zeros((rows, n))
    ab = np.zeros((rows, n))
    lib().orc_spmm_f32_ref64(n, _p(rp), _p(ci), _p(v), _p(bb), n, _p(c64), _p(ab), row_begin,
                             row_end, nthreads or min(os.cpu_count() or 1, 16), bb.shape[0])
    return c64, ab


def within_tolerance(c, c64, absum, rtol):
    """|C - C64| <= rtol * absum + 1e-30 elementwise (SURVEY.md §8c acceptance)."""
    err = np.abs(np.asarray(c, dtype=np.float64) - c64)
    bound = rtol * absum + 1e-30
    ok = err <= bound
    return bool(ok.all()), float((err / (absum + 1e-30)).max(initial=0.0))


# ---- backward -----------------------------------------------------------
def _lib_sddmm():
    L = lib()
    if not getattr(L, "_sddmm_set", False):
        i64, p, c_int = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
        L.orc_sddmm_f32.argtypes = [i64, p, p, p, i64, p, i64, p, i64, i64, c_int, i64]
        L.orc_sddmm_f64.argtypes = L.orc_sddmm_f32.argtypes
        L._sddmm_set = True
    return L


def sddmm(row_ptr, col_idx, a, b, *, dtype="f32", row_begin=0, row_end=None, nthreads=None):
    """out[j] = <a[row(j)-row_begin], b[col[j]]> in the operator's pairwise-leaf order (a column
    outside [0, K) reads the forward's zero-filled row).
    a holds rows [row_begin, row_end); bf16 arrays are uint16 bit patterns."""
    m = len(row_ptr) - 1
    row_end = m if row_end is None else row_end
    n = b.shape[1]
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    ci = np.ascontiguousarray(col_idx, dtype=np.int64)
    nnz = int(rp[-1])
    nt = nthreads or min(os.cpu_count() or 1, 16)
    if dtype == "f64":
        aa = np.ascontiguousarray(a, dtype=np.float64)
        bb = np.ascontiguousarray(b, dtype=np.float64)
        out = np.zeros(nnz, dtype=np.float64)
        _lib_sddmm().orc_sddmm_f64(n, _p(rp), _p(ci), _p(aa), n, _p(bb), n, _p(out), row_begin,
                                   row_end, nt, bb.shape[0])
        return out
    if dtype == "bf16":
        aa, bb = bf16_bits_to_f32(np.asarray(a)), bf16_bits_to_f32(np.asarray(b))
    else:
        aa, bb = np.asarray(a).astype(np.float32), np.asarray(b).astype(np.float32)
    aa, bb = np.ascontiguousarray(aa), np.ascontiguousarray(bb)
    out = np.zeros(nnz, dtype=np.float32)
    _lib_sddmm().orc_sddmm_f32(n, _p(rp), _p(ci), _p(aa), n, _p(bb), n, _p(out), row_begin, row_end, nt,
                               bb.shape[0])
    if dtype == "bf16":
        return f32_to_bf16_bits(out)
    if dtype == "f16":
        return out.astype(np.float16)
    return out


def transpose(row_ptr, col_idx, k):
    """CSR -> CSR of the transpose by a stable sort on the column (entries of each new row keep
    ascending original row order).  Returns (row_ptr_T, col_idx_T = original rows, perm).
    A column outside [0, k) sorts as k: after row_ptr_T[k], in no row (the forward's zero-filled
    gather reads no row of b, so d b gets nothing from it)."""
    rp = np.asarray(row_ptr, dtype=np.int64)
    ci = np.asarray(col_idx, dtype=np.int64)
    rows = np.repeat(np.arange(len(rp) - 1, dtype=np.int64), np.diff(rp))
    key = np.where((ci >= 0) & (ci < k), ci, k)
    perm = np.argsort(key, kind="stable")
    rp_t = np.zeros(k + 1, dtype=np.int64)
    rp_t[1:] = np.cumsum(np.bincount(key, minlength=k + 1)[:k])
    return rp_t, rows[perm], perm


# ---- COO -> CSR -----------------------------------------------------------
def coo_to_csr(row, col, values, m, k, merge=True, dtype="f32"):
    """Canonical CSR from COO by a stable sort on (row, col); duplicates summed sequentially in
    input order (fp32 for 16-bit types; bf16 as uint16 bits)."""
    row = np.asarray(row, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    key = row * k + col
    perm = np.argsort(key, kind="stable")
    sk = key[perm]
    heads = np.ones(len(sk), dtype=bool)
    if merge and len(sk):
        heads[1:] = sk[1:] != sk[:-1]
    starts = np.nonzero(heads)[0]
    ends = np.append(starts[1:], len(sk))
    out_col = col[perm][starts]
    out_row = row[perm][starts]
    rp = np.zeros(m + 1, dtype=np.int64)
    rp[1:] = np.cumsum(np.bincount(out_row, minlength=m))
    out_val = None
    if values is not None:
        if dtype == "bf16":
            v = bf16_bits_to_f32(np.asarray(values))
        elif dtype == "f64":
            v = np.asarray(values, dtype=np.float64)
        else:
            v = np.asarray(values).astype(np.float32)
        acc_t = np.float64 if dtype == "f64" else np.float32
        out = np.zeros(len(starts), dtype=acc_t)
        vp = v[perm]
        for i, (s, e) in enumerate(zip(starts, ends)):
            a = acc_t(0)
            for q in range(s, e):
                a = acc_t(a + vp[q])
            out[i] = a
        if dtype == "bf16":
            out_val = f32_to_bf16_bits(out)
        elif dtype == "f16":
            out_val = out.astype(np.float16)
        else:
            out_val = out
    return rp, out_col, out_val
