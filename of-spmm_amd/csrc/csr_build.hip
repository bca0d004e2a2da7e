// csr_build.hip — COO (edge_index) -> CSR on the device, gfx950.
//
// GNN inputs arrive as COO pairs; the reference keeps the building blocks for this on CUDA
// (oneflow/user/kernels/radix_sort.cuh, core/cuda/unique.cuh, search_sorted_kernel.cu) but no
// SpMM to feed.  Here:
//   key = row * k + col (64-bit)  ->  stable LSD radix sort of (key, entry id) (hipCUB / rocPRIM)
//   ->  optional duplicate merge: entries with equal (row, col) are summed in input order
//       (deterministic: one thread walks each run sequentially, fp32 accumulation for 16-bit)
//   ->  col_idx = key % k, values gathered / summed, row_ptr[r] = lower_bound(keys, r * k).
// Output is canonical CSR (rows ascending, columns ascending and unique when merging).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <climits>

#include "ofx_internal.h"
#include "spmm_common.h"
#include "spmm_plan.h"

namespace ofx {
namespace {

constexpr int kBlock = 256;

unsigned grid_for(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g > 65536) g = 65536;
  return (unsigned)(g < 1 ? 1 : g);
}

int key_bits(int64_t m, int64_t k) {
  const unsigned __int128 top = (unsigned __int128)(m > 0 ? m : 1) * (unsigned __int128)(k > 0 ? k : 1);
  int b = 1;
  while (b < 64 && ((unsigned __int128)1 << b) < top) ++b;
  return b;
}

template <typename I>
__global__ void make_keys_kernel(const I* __restrict__ row, const I* __restrict__ col, int64_t nnz,
                                 int64_t k, uint64_t* __restrict__ keys, int64_t* __restrict__ ids,
                                 unsigned int* __restrict__ bad, int64_t m) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
    const int64_t r = (int64_t)row[i], c = (int64_t)col[i];
    if (r < 0 || r >= m || c < 0 || c >= k) atomicOr(bad, 1u);
    keys[i] = (uint64_t)(r < 0 ? 0 : r) * (uint64_t)k + (uint64_t)(c < 0 ? 0 : c);
    ids[i] = i;
  }
}

// head[i] = 1 if sorted key i starts a run of equal keys (or merging is off).
__global__ void heads_kernel(const uint64_t* __restrict__ keys, int64_t nnz, int merge,
                             int64_t* __restrict__ head) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride)
    head[i] = (!merge || i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// pos = inclusive scan of head; the run starting at sorted position i (head) lands at pos[i]-1.
template <typename T, typename I>
__global__ void emit_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ perm,
                            const int64_t* __restrict__ pos, int64_t nnz, int64_t k,
                            const T* __restrict__ val, I* __restrict__ out_col,
                            T* __restrict__ out_val, uint64_t* __restrict__ out_keys) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
    const bool head = i == 0 || pos[i] != pos[i - 1];
    if (!head) continue;
    const int64_t o = pos[i] - 1;
    out_col[o] = (I)(keys[i] % (uint64_t)k);
    out_keys[o] = keys[i];
    if (val != nullptr) {
      A acc = A(0);
      int64_t e = i;
      do {  // the run of equal keys, in input (stable) order
        acc = acc + Num<T>::load(val[perm[e]]);
        ++e;
      } while (e < nnz && pos[e] == pos[i]);
      out_val[o] = Num<T>::store(acc);
    }
  }
}

template <typename I>
__global__ void row_ptr_kernel(const uint64_t* __restrict__ ukeys,
                               const int64_t* __restrict__ pos_last, int64_t m, int64_t k,
                               I* __restrict__ out_rp) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > m) return;
  const int64_t n = *pos_last;
  const uint64_t target = (uint64_t)r * (uint64_t)k;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ukeys[mid] < target) lo = mid + 1; else hi = mid;
  }
  out_rp[r] = (I)lo;
}

__global__ void copy_count_kernel(const int64_t* __restrict__ pos_last, int64_t* __restrict__ out) {
  *out = *pos_last;
}

struct BuildWs {
  size_t keys_in, keys_out, ids_in, ids_out, head, pos, ukeys, bad, cub, total, cub_bytes,
      scan_bytes;
};

int build_ws(int64_t m, int64_t k, int64_t nnz, BuildWs* w) {
  *w = BuildWs{};
  if (nnz == 0) return OFX_OK;
  size_t cub = 0, scan = 0;
  OFX_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const uint64_t*)nullptr,
                                                   (uint64_t*)nullptr, (const int64_t*)nullptr,
                                                   (int64_t*)nullptr, (int)nnz, 0, key_bits(m, k)));
  OFX_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, scan, (const int64_t*)nullptr,
                                                 (int64_t*)nullptr, (int)nnz));
  size_t off = 0;
  const size_t e8 = plan::align_up((size_t)nnz * 8, 256);
  w->keys_in = off; off += e8;
  w->keys_out = off; off += e8;
  w->ids_in = off; off += e8;
  w->ids_out = off; off += e8;
  w->head = off; off += e8;
  w->pos = off; off += e8;
  w->ukeys = off; off += e8;
  w->bad = off; off += 256;
  w->cub = off;
  w->cub_bytes = cub > scan ? cub : scan;
  w->scan_bytes = scan;
  off += plan::align_up(w->cub_bytes, 256);
  w->total = off;
  return OFX_OK;
}

template <typename T, typename I>
int build(hipStream_t s, int64_t m, int64_t k, int64_t nnz, const I* row, const I* col,
          const T* val, int merge, I* out_rp, I* out_col, T* out_val, int64_t* out_nnz,
          unsigned int* bad_out, char* ws, size_t ws_bytes) {
  BuildWs w;
  int rc = build_ws(m, k, nnz, &w);
  if (rc) return rc;
  if (nnz == 0) {
    OFX_HIP_CHECK(hipMemsetAsync(out_rp, 0, (size_t)(m + 1) * sizeof(I), s));
    OFX_HIP_CHECK(hipMemsetAsync(out_nnz, 0, sizeof(int64_t), s));
    if (bad_out) OFX_HIP_CHECK(hipMemsetAsync(bad_out, 0, sizeof(unsigned int), s));
    return OFX_OK;
  }
  OFX_REQUIRE(ws && ws_bytes >= w.total, OFX_EWORKSPACE,
              "coo_to_csr: workspace of %zu bytes < %zu required", ws_bytes, w.total);
  auto* keys_in = reinterpret_cast<uint64_t*>(ws + w.keys_in);
  auto* keys_out = reinterpret_cast<uint64_t*>(ws + w.keys_out);
  auto* ids_in = reinterpret_cast<int64_t*>(ws + w.ids_in);
  auto* ids_out = reinterpret_cast<int64_t*>(ws + w.ids_out);
  auto* head = reinterpret_cast<int64_t*>(ws + w.head);
  auto* pos = reinterpret_cast<int64_t*>(ws + w.pos);
  auto* ukeys = reinterpret_cast<uint64_t*>(ws + w.ukeys);
  auto* bad = bad_out ? bad_out : reinterpret_cast<unsigned int*>(ws + w.bad);
  void* cub_tmp = ws + w.cub;
  const unsigned g = grid_for(nnz);
  OFX_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(unsigned int), s));
  hipLaunchKernelGGL((make_keys_kernel<I>), dim3(g), dim3(kBlock), 0, s, row, col, nnz, k, keys_in,
                     ids_in, bad, m);
  OFX_HIP_CHECK(hipGetLastError());
  size_t cb = w.cub_bytes;
  OFX_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cb, keys_in, keys_out, ids_in, ids_out,
                                                   (int)nnz, 0, key_bits(m, k), s));
  hipLaunchKernelGGL(heads_kernel, dim3(g), dim3(kBlock), 0, s, keys_out, nnz, merge, head);
  OFX_HIP_CHECK(hipGetLastError());
  cb = w.cub_bytes;
  OFX_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(cub_tmp, cb, head, pos, (int)nnz, s));
  hipLaunchKernelGGL((emit_kernel<T, I>), dim3(g), dim3(kBlock), 0, s, keys_out, ids_out, pos, nnz, k,
                     val, out_col, out_val, ukeys);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((row_ptr_kernel<I>), dim3((unsigned)((m + 1 + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, s, ukeys, pos + (nnz - 1), m, k, out_rp);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(copy_count_kernel, dim3(1), dim3(1), 0, s, pos + (nnz - 1), out_nnz);
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

template <typename I>
int build_typed(int val_dtype, hipStream_t s, int64_t m, int64_t k, int64_t nnz, const I* row,
                const I* col, const void* val, int merge, I* out_rp, I* out_col, void* out_val,
                int64_t* out_nnz, unsigned int* bad, char* ws, size_t ws_bytes) {
  switch (val_dtype) {
    case OFX_DT_FLOAT:
      return build<float, I>(s, m, k, nnz, row, col, (const float*)val, merge, out_rp, out_col,
                             (float*)out_val, out_nnz, bad, ws, ws_bytes);
    case OFX_DT_DOUBLE:
      return build<double, I>(s, m, k, nnz, row, col, (const double*)val, merge, out_rp, out_col,
                              (double*)out_val, out_nnz, bad, ws, ws_bytes);
    case OFX_DT_BFLOAT16:
      return build<bf16, I>(s, m, k, nnz, row, col, (const bf16*)val, merge, out_rp, out_col,
                            (bf16*)out_val, out_nnz, bad, ws, ws_bytes);
    case OFX_DT_FLOAT16:
      return build<f16, I>(s, m, k, nnz, row, col, (const f16*)val, merge, out_rp, out_col,
                           (f16*)out_val, out_nnz, bad, ws, ws_bytes);
    default: return fail(OFX_EUNSUPPORTED, "coo_to_csr: unsupported value dtype %d", val_dtype);
  }
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_coo_to_csr_workspace_size(int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                             size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes && m >= 0 && k >= 0 && nnz >= 0 && nnz <= INT32_MAX, OFX_EINVAL,
                "coo_to_csr: bad sizes (nnz must be < 2^31)");
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "coo_to_csr: bad index dtype %d",
                idx_dtype);
    BuildWs w;
    const int rc = build_ws(m, k, nnz, &w);
    *bytes = w.total;
    return rc;
  });
}

extern "C" int ofx_coo_to_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                              int64_t nnz, const void* row, const void* col, const void* values,
                              int merge_duplicates, void* out_row_ptr, void* out_col_idx,
                              void* out_values, void* out_nnz, void* bad_flag, void* workspace,
                              size_t workspace_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(m >= 0 && k >= 0 && nnz >= 0 && nnz <= INT32_MAX, OFX_EINVAL,
                "coo_to_csr: bad sizes (nnz must be < 2^31)");
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "coo_to_csr: bad index dtype %d",
                idx_dtype);
    OFX_REQUIRE(out_row_ptr && out_nnz && (nnz == 0 || (row && col && out_col_idx)), OFX_EINVAL,
                "coo_to_csr: NULL pointer");
    OFX_REQUIRE((values == nullptr) == (out_values == nullptr), OFX_EINVAL,
                "coo_to_csr: values and out_values must both be given or both be NULL");
    const int vdt = values ? val_dtype : OFX_DT_FLOAT;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (idx_dtype == OFX_DT_INT32)
      return build_typed<int32_t>(vdt, s, m, k, nnz, (const int32_t*)row, (const int32_t*)col, values,
                                  merge_duplicates, (int32_t*)out_row_ptr, (int32_t*)out_col_idx,
                                  out_values, (int64_t*)out_nnz, (unsigned int*)bad_flag,
                                  (char*)workspace, workspace_bytes);
    return build_typed<int64_t>(vdt, s, m, k, nnz, (const int64_t*)row, (const int64_t*)col, values,
                                merge_duplicates, (int64_t*)out_row_ptr, (int64_t*)out_col_idx,
                                out_values, (int64_t*)out_nnz, (unsigned int*)bad_flag,
                                (char*)workspace, workspace_bytes);
  });
}
