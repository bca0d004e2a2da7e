// rows.hip — row gather for the halo exchange: dst[i, :] = src[idx[i], :].
//
// Packs the B rows a peer asked for into one contiguous send buffer per step (the pack step of
// ShuffleData's callers, oneflow/user/kernels/data_shuffle_kernel.cu:356-497, which gather
// embedding rows by id before the grouped send).  HBM-bound: row_bytes read + written per row.
// Lane groups of LPR lanes copy one row with the widest aligned word (16 B when the row size,
// strides and base pointers allow it, else 4 B, else 1 B); groups stride over the rows.
#include <hip/hip_runtime.h>

#include "ofx_internal.h"
#include "spmm_common.h"

namespace ofx {
namespace {

constexpr int kBlock = 256;

template <typename W, int LPR, typename I>
__global__ void __launch_bounds__(kBlock)
    gather_rows_kernel(const I* __restrict__ idx, int64_t count, int64_t words,
                       const char* __restrict__ src, int64_t src_stride, char* __restrict__ dst,
                       int64_t dst_stride) {
  constexpr int GPB = kBlock / LPR;
  const int gl = threadIdx.x % LPR;
  for (int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; i < count;
       i += (int64_t)gridDim.x * GPB) {
    const int64_t r = idx ? (int64_t)idx[i] : i;  // NULL index: a plain strided row copy
    const W* s = reinterpret_cast<const W*>(src + r * src_stride);
    W* d = reinterpret_cast<W*>(dst + i * dst_stride);
    for (int64_t w = gl; w < words; w += LPR) d[w] = s[w];
  }
}

template <typename W, typename I>
int launch(hipStream_t s, const I* idx, int64_t count, int64_t row_bytes, const void* src,
           int64_t src_stride, void* dst, int64_t dst_stride) {
  const int64_t words = row_bytes / (int64_t)sizeof(W);
  int lpr = 1;
  while (lpr < 64 && lpr < words) lpr *= 2;
  const int64_t gpb = kBlock / lpr;
  const unsigned grid = (unsigned)std::min<int64_t>((count + gpb - 1) / gpb, 65536);
  auto go = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, s, idx, count, words,
                       static_cast<const char*>(src), src_stride, static_cast<char*>(dst),
                       dst_stride);
  };
  switch (lpr) {
    case 1: go(gather_rows_kernel<W, 1, I>); break;
    case 2: go(gather_rows_kernel<W, 2, I>); break;
    case 4: go(gather_rows_kernel<W, 4, I>); break;
    case 8: go(gather_rows_kernel<W, 8, I>); break;
    case 16: go(gather_rows_kernel<W, 16, I>); break;
    case 32: go(gather_rows_kernel<W, 32, I>); break;
    default: go(gather_rows_kernel<W, 64, I>); break;
  }
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

template <typename I>
int dispatch(hipStream_t s, const I* idx, int64_t count, int64_t row_bytes, const void* src,
             int64_t src_stride, void* dst, int64_t dst_stride) {
  auto aligned = [&](int64_t a) {
    return row_bytes % a == 0 && src_stride % a == 0 && dst_stride % a == 0 &&
           (uintptr_t)src % a == 0 && (uintptr_t)dst % a == 0;
  };
  if (aligned(16)) return launch<uint4>(s, idx, count, row_bytes, src, src_stride, dst, dst_stride);
  if (aligned(4)) return launch<uint32_t>(s, idx, count, row_bytes, src, src_stride, dst, dst_stride);
  return launch<unsigned char>(s, idx, count, row_bytes, src, src_stride, dst, dst_stride);
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_gather_rows(void* stream, int idx_dtype, int64_t count, int64_t row_bytes,
                               const void* idx, const void* src, int64_t src_stride_bytes,
                               void* dst, int64_t dst_stride_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "gather_rows: bad index dtype %d",
                idx_dtype);
    OFX_REQUIRE(count >= 0 && row_bytes >= 0 && src_stride_bytes >= row_bytes &&
                    dst_stride_bytes >= row_bytes,
                OFX_EINVAL, "gather_rows: bad sizes");
    if (count == 0 || row_bytes == 0) return OFX_OK;
    OFX_REQUIRE(src && dst, OFX_EINVAL, "gather_rows: NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (idx_dtype == OFX_DT_INT32)
      return dispatch(s, static_cast<const int32_t*>(idx), count, row_bytes, src, src_stride_bytes,
                      dst, dst_stride_bytes);
    return dispatch(s, static_cast<const int64_t*>(idx), count, row_bytes, src, src_stride_bytes, dst,
                    dst_stride_bytes);
  });
}

// ---- 3-level strided block copy (grid exchange pack / unpack) ---------------
// Row q = (o, i, r) of an nouter x ninner x rows set of rows, each row_bytes long:
//   dst + o*dst_outer + i*dst_inner + r*dst_row  <-  src + o*src_outer + i*src_inner + r*src_row
// One launch replaces the C x S per-block copies of a grid step (pack the shard into column
// blocks, unpack the received blocks into the output rows).
namespace ofx {
namespace {
template <typename W, int LPR>
__global__ void __launch_bounds__(kBlock)
    copy_blocks_kernel(int64_t count, int64_t ninner, int64_t rows, int64_t words,
                       const char* __restrict__ src, int64_t so, int64_t si, int64_t sr,
                       char* __restrict__ dst, int64_t dout, int64_t di, int64_t dr) {
  constexpr int GPB = kBlock / LPR;
  const int gl = threadIdx.x % LPR;
  for (int64_t q = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; q < count;
       q += (int64_t)gridDim.x * GPB) {
    const int64_t r = q % rows, oi = q / rows;
    const int64_t i = oi % ninner, o = oi / ninner;
    const W* s = reinterpret_cast<const W*>(src + o * so + i * si + r * sr);
    W* d = reinterpret_cast<W*>(dst + o * dout + i * di + r * dr);
    for (int64_t w = gl; w < words; w += LPR) d[w] = s[w];
  }
}

template <typename W>
int launch_blocks(hipStream_t s, int64_t nouter, int64_t ninner, int64_t rows, int64_t row_bytes,
                  const void* src, int64_t so, int64_t si, int64_t sr, void* dst, int64_t dout,
                  int64_t di, int64_t dr) {
  const int64_t words = row_bytes / (int64_t)sizeof(W);
  const int64_t count = nouter * ninner * rows;
  int lpr = 1;
  while (lpr < 64 && lpr < words) lpr *= 2;
  const int64_t gpb = kBlock / lpr;
  const unsigned grid = (unsigned)std::min<int64_t>((count + gpb - 1) / gpb, 65536);
  auto go = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, s, count, ninner, rows, words,
                       static_cast<const char*>(src), so, si, sr, static_cast<char*>(dst), dout,
                       di, dr);
  };
  switch (lpr) {
    case 1: go(copy_blocks_kernel<W, 1>); break;
    case 2: go(copy_blocks_kernel<W, 2>); break;
    case 4: go(copy_blocks_kernel<W, 4>); break;
    case 8: go(copy_blocks_kernel<W, 8>); break;
    case 16: go(copy_blocks_kernel<W, 16>); break;
    case 32: go(copy_blocks_kernel<W, 32>); break;
    default: go(copy_blocks_kernel<W, 64>); break;
  }
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_copy_blocks(void* stream, int64_t nouter, int64_t ninner, int64_t rows,
                               int64_t row_bytes, const void* src, int64_t src_outer,
                               int64_t src_inner, int64_t src_row, void* dst, int64_t dst_outer,
                               int64_t dst_inner, int64_t dst_row) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(nouter >= 0 && ninner >= 0 && rows >= 0 && row_bytes >= 0, OFX_EINVAL,
                "copy_blocks: negative size");
    if (nouter == 0 || ninner == 0 || rows == 0 || row_bytes == 0) return OFX_OK;
    OFX_REQUIRE(src && dst, OFX_EINVAL, "copy_blocks: NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto aligned = [&](int64_t a) {
      return row_bytes % a == 0 && src_outer % a == 0 && src_inner % a == 0 && src_row % a == 0 &&
             dst_outer % a == 0 && dst_inner % a == 0 && dst_row % a == 0 &&
             (uintptr_t)src % a == 0 && (uintptr_t)dst % a == 0;
    };
    if (aligned(16))
      return launch_blocks<uint4>(s, nouter, ninner, rows, row_bytes, src, src_outer, src_inner,
                                  src_row, dst, dst_outer, dst_inner, dst_row);
    if (aligned(4))
      return launch_blocks<uint32_t>(s, nouter, ninner, rows, row_bytes, src, src_outer, src_inner,
                                     src_row, dst, dst_outer, dst_inner, dst_row);
    return launch_blocks<unsigned char>(s, nouter, ninner, rows, row_bytes, src, src_outer,
                                        src_inner, src_row, dst, dst_outer, dst_inner, dst_row);
  });
}

// ---- padded-owner column remap (row split) -----------------------------------
// Column c of B lives in shard owner(c) = BalancedSplitter(k, world) and, in the padded gathered
// buffer [world * P, n] (P = ceil(k / world)), at row c + max(owner(c) - extra, 0) where
// extra = k % world > 0 (the first `extra` shards hold P rows, the rest P - 1, each padded to
// P); with extra == 0 every shard holds exactly P rows and c stays.
namespace ofx {
namespace {
template <typename I>
__global__ void padded_remap_kernel(const I* __restrict__ in, I* __restrict__ out, int64_t nnz,
                                    int64_t base, int64_t extra) {
  const int64_t big = extra * (base + 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz; j += stride) {
    const int64_t c = (int64_t)in[j];
    const int64_t owner = c < big ? c / (base + 1) : extra + (c - big) / (base > 0 ? base : 1);
    // extra == 0: P == base, every shard fills its slot, nothing moves
    out[j] = (I)(c + (extra > 0 && owner > extra ? owner - extra : 0));
  }
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_padded_owner_remap(void* stream, int idx_dtype, int64_t nnz, int64_t k,
                                      int64_t world, const void* col_in, void* col_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "padded_owner_remap: bad index dtype");
    OFX_REQUIRE(nnz >= 0 && k >= 0 && world > 0, OFX_EINVAL, "padded_owner_remap: bad sizes");
    if (nnz == 0) return OFX_OK;
    OFX_REQUIRE(col_in && col_out, OFX_EINVAL, "padded_owner_remap: NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t base = k / world, extra = k % world;
    const unsigned grid = (unsigned)std::min<int64_t>((nnz + kBlock - 1) / kBlock, 65536);
    if (idx_dtype == OFX_DT_INT32)
      hipLaunchKernelGGL(padded_remap_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, s,
                         static_cast<const int32_t*>(col_in), static_cast<int32_t*>(col_out), nnz,
                         base, extra);
    else
      hipLaunchKernelGGL(padded_remap_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, s,
                         static_cast<const int64_t*>(col_in), static_cast<int64_t*>(col_out), nnz,
                         base, extra);
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}
