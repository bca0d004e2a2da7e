// spmm_backward.hip — the gradient path of op "spmm_csr" (SURVEY.md §8f row 1), gfx950.
//
// For C = A @ B with A in CSR (values v):
//   dB = A^T @ dC       -> ofx_csr_transpose (structure, once per graph) + ofx_gather_values
//                          (A^T values = v[perm]) + the forward SpMM kernel on A^T
//   dv[j] = <dC[row(j),:], B[col(j),:]>  (SDDMM on A's pattern) -> ofx_sddmm_csr
// Reference anchors: the gradient-function pattern of matrix_vector_product
// (oneflow/core/autograd/gradient_funcs/matrix_vector_product.cpp:26-91: dA = dy x b^T restricted,
// db = a^T x dy) and the transpose-by-sort building blocks the reference keeps for CUDA
// (oneflow/user/kernels/radix_sort.cuh, arg_sort_kernel.cu).
//
// Numeric contract of ofx_sddmm_csr (also restated by oracle/spmm_oracle.c):
//   p_n = dC[r,n] * B[c,n] (one rounding); leaf i = sequential sum of p_n over n in [8i, 8i+8)
//   from +0; the leaves (padded with +0 to a power of two) are added pairwise, level by level
//   ((l0+l1)+(l2+l3))+...; one rounding to T at the end.  fp32 accumulation for f32/f16/bf16.
// The transpose is a stable LSD radix sort by column, so A^T rows hold their entries in
// ascending row order and dB = A^T @ dC follows the forward contract exactly.
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

template <typename I>
__global__ void iota_kernel(I* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (I)i;
}

// row_of[j] = r for j in [rp[r], rp[r+1]): one wave per row, lanes stride the row (a hub row
// of 10^5-10^6 nonzeros must not be written by a single thread).
template <typename I>
__global__ void __launch_bounds__(kBlock) expand_rows_kernel(const I* __restrict__ rp, int64_t m,
                                                             I* __restrict__ row_of) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); r < m; r += stride)
    for (int64_t j = (int64_t)rp[r] + lane; j < (int64_t)rp[r + 1]; j += 64) row_of[j] = (I)r;
}

// Sort keys of the transpose: the column, or k for a column outside [0, k) (the forward zero-fills
// its gathered row, so such a nonzero touches no row of B and belongs to no row of A^T; sorted
// past row_ptr_T[k], it is never read).
template <typename I>
__global__ void transpose_keys_kernel(const I* __restrict__ col, int64_t nnz, int64_t k,
                                      I* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz; j += stride) {
    const int64_t c = (int64_t)col[j];
    keys[j] = (I)((uint64_t)c < (uint64_t)k ? c : k);
  }
}

// out_rp[c] = first position of column >= c in the sorted keys (binary search).
template <typename I>
__global__ void col_ptr_kernel(const I* __restrict__ keys, int64_t nnz, int64_t k,
                               I* __restrict__ out_rp) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > k) return;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)keys[mid] < c) lo = mid + 1; else hi = mid;
  }
  out_rp[c] = (I)lo;
}

template <typename I>
__global__ void gather_rows_kernel(const I* __restrict__ perm, const I* __restrict__ row_of,
                                   int64_t nnz, I* __restrict__ out_col) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nnz; t += stride)
    out_col[t] = row_of[perm[t]];
}

template <typename T, typename I>
__global__ void gather_values_kernel(const I* __restrict__ perm, const T* __restrict__ src,
                                     int64_t nnz, T* __restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nnz; t += stride)
    dst[t] = src[perm[t]];
}

int bits_for(int64_t k) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < k) ++b;
  return b;
}

// Workspace: keys_in, vals_in (iota), keys_out, row_of, then hipcub temp storage.
template <typename I>
int transpose_ws(int64_t nnz, int64_t k, size_t* bytes, size_t* cub_bytes) {
  size_t cub = 0;
  if (nnz > 0) {
    OFX_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const I*)nullptr, (I*)nullptr,
                                                     (const I*)nullptr, (I*)nullptr, (int)nnz, 0,
                                                     bits_for(k + 1)));
  }
  *cub_bytes = cub;
  *bytes = plan::align_up(4 * (size_t)nnz * sizeof(I), 256) + plan::align_up(cub, 256);
  return OFX_OK;
}

template <typename I>
int transpose(hipStream_t s, int64_t m, int64_t k, int64_t nnz, const I* rp, const I* col,
              I* out_rp, I* out_col, I* out_perm, void* ws, size_t ws_bytes) {
  size_t need = 0, cub = 0;
  int rc = transpose_ws<I>(nnz, k, &need, &cub);
  if (rc) return rc;
  OFX_REQUIRE(ws_bytes >= need && (need == 0 || ws), OFX_EWORKSPACE,
              "csr_transpose: workspace of %zu bytes < %zu required", ws_bytes, need);
  const unsigned g_nnz = (unsigned)std::min<int64_t>((nnz + kBlock - 1) / kBlock, 65536);
  if (nnz == 0) {
    OFX_HIP_CHECK(hipMemsetAsync(out_rp, 0, (size_t)(k + 1) * sizeof(I), s));
    return OFX_OK;
  }
  I* keys_out = static_cast<I*>(ws);
  I* vals_in = keys_out + nnz;
  I* row_of = vals_in + nnz;
  I* keys_in = row_of + nnz;
  void* cub_tmp = static_cast<char*>(ws) + plan::align_up(4 * (size_t)nnz * sizeof(I), 256);
  hipLaunchKernelGGL((iota_kernel<I>), dim3(g_nnz), dim3(kBlock), 0, s, vals_in, nnz);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((expand_rows_kernel<I>), dim3((unsigned)std::min<int64_t>((m + 3) / 4, 1 << 20)),
                     dim3(kBlock), 0, s,
                     rp, m, row_of);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((transpose_keys_kernel<I>), dim3(g_nnz), dim3(kBlock), 0, s, col, nnz, k,
                     keys_in);
  OFX_HIP_CHECK(hipGetLastError());
  // stable LSD radix sort of (col, j): entries of one column keep ascending j == ascending row
  OFX_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub, keys_in, keys_out, vals_in, out_perm,
                                                   (int)nnz, 0, bits_for(k + 1), s));
  hipLaunchKernelGGL((col_ptr_kernel<I>), dim3((unsigned)((k + 1 + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, s, keys_out, nnz, k, out_rp);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((gather_rows_kernel<I>), dim3(g_nnz), dim3(kBlock), 0, s, out_perm, row_of,
                     nnz, out_col);
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

// ---- SDDMM -------------------------------------------------------------------------------
// One lane-group of LG lanes per work item (a row, or a chunk of a hub row, from the shared
// planner: the per-nonzero results do not depend on the grouping).  Lane t of a group owns the
// L contiguous 8-element leaves [t*L, (t+1)*L) of the N-vector: it keeps dC[row] in registers
// for the whole row and streams B[col] rows, U nonzeros in flight.  In-lane pairwise over its L
// leaves, then an xor butterfly over the LG lanes = the pairwise tree over LG*L leaves.
constexpr int kLeaf = 8;

template <typename T, bool ALIGNED>
__device__ __forceinline__ void load_leaf(const T* __restrict__ p, int64_t base, int64_t n,
                                          typename Num<T>::acc (&x)[kLeaf]) {
  using A = typename Num<T>::acc;
  if constexpr (ALIGNED) {  // n % 8 == 0, rows 16-B aligned: a leaf is all in or all out
    if (base >= n) {
#pragma unroll
      for (int e = 0; e < kLeaf; ++e) x[e] = A(0);
      return;
    }
    struct alignas(16) P16 {
      T v[16 / sizeof(T) < kLeaf ? 16 / sizeof(T) : kLeaf];
    };
    constexpr int per = sizeof(P16) / sizeof(T);
#pragma unroll
    for (int q = 0; q < kLeaf / per; ++q) {
      const P16 v = *reinterpret_cast<const P16*>(p + base + q * per);
#pragma unroll
      for (int e = 0; e < per; ++e) x[q * per + e] = Num<T>::load(v.v[e]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < kLeaf; ++e) x[e] = base + e < n ? Num<T>::load(p[base + e]) : A(0);
  }
}

// Work item of lane-group g: (local row, nonzero range) of a row or hub chunk; false if none.
template <typename I>
__device__ __forceinline__ bool sddmm_item(const I* __restrict__ rp, int64_t g, int64_t row_begin,
                                           int64_t nrows, int64_t chunk,
                                           const unsigned long long* __restrict__ counters,
                                           const int64_t* __restrict__ items,
                                           const int64_t* __restrict__ order, int64_t* lr_out,
                                           int64_t* j0_out, int64_t* j1_out) {
  int64_t lr, c = -1;
  if (order == nullptr) {
    if (g >= nrows) return false;
    lr = g;
  } else {
    const int64_t nchunks = (int64_t)counters[0];
    if (g < nchunks) {
      lr = items[2 * g];
      c = items[2 * g + 1];
    } else {
      const int64_t q = g - nchunks;
      if (q >= nrows - (int64_t)counters[1]) return false;
      lr = plan::order_row(order, nrows, (int64_t)counters[3] - (int64_t)counters[2], q);
    }
  }
  const int64_t r = row_begin + lr;
  const int64_t rs = (int64_t)rp[r], re = (int64_t)rp[r + 1];
  int64_t j0 = rs, j1 = re;
  if (c >= 0) {  // chunk c of len / chunk; the last takes the remainder
    j0 = rs + c * chunk;
    j1 = (re - j0 - chunk < chunk) ? re : j0 + chunk;
  }
  *lr_out = lr;
  *j0_out = j0;
  *j1_out = j1;
  return j0 < j1;
}

// A work list from a failed, superseded or never-built plan: the launch fills its output (the
// nonzeros of its rows, out[rp[row_begin] .. rp[row_begin + nrows])) with the canonical quiet NaN
// and reports it (spmm_plan.h plan_valid; the host's next entry returns OFX_EPLAN).  Every launch
// of a cut grid poisons the whole range (idempotent).
template <typename T, typename I>
__device__ __forceinline__ bool sddmm_plan_invalid(const unsigned long long* __restrict__ counters,
                                                   int64_t block_base, unsigned* err,
                                                   const I* __restrict__ rp, int64_t row_begin,
                                                   int64_t nrows, T* __restrict__ out) {
  if (counters == nullptr || plan::plan_valid(counters)) return false;
  if (block_base + blockIdx.x == 0 && threadIdx.x == 0)
    plan::raise_device_error(err, plan::kErrPlanInvalid);
  const int64_t j0 = (int64_t)rp[row_begin], j1 = (int64_t)rp[row_begin + nrows];
  const T p = poison_value<T>();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < j1; j += stride) out[j] = p;
  return true;
}

// Grid pieces: a launch holds fewer than 2^32 threads (papers-scale row counts would not).
constexpr int64_t kLaunchBlocks = ((int64_t)1 << 31) / kBlock;

template <typename T, typename I, int LG, int L, int U, bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
    sddmm_kernel(const I* __restrict__ rp, const I* __restrict__ col, const T* __restrict__ dC,
                 int64_t ldc, const T* __restrict__ B, int64_t ldb, int64_t kb,
                 T* __restrict__ out, int64_t row_begin, int64_t nrows, int64_t n, int64_t chunk,
                 const unsigned long long* __restrict__ counters, const int64_t* __restrict__ items,
                 const int64_t* __restrict__ order, int64_t block_base, unsigned* err) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  constexpr int GPW = 64 / LG;
  if (sddmm_plan_invalid(counters, block_base, err, rp, row_begin, nrows, out)) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gl = lane & (LG - 1);
  const int64_t g = ((block_base + (int64_t)blockIdx.x) * (kBlock / 64) + wave) * GPW + lane / LG;
  int64_t lr, j0, j1;
  if (!sddmm_item<I>(rp, g, row_begin, nrows, chunk, counters, items, order, &lr, &j0, &j1)) return;
  // dC row, this lane's leaves
  A a[L][kLeaf];
  const T* arow = dC + lr * ldc;
#pragma unroll
  for (int l = 0; l < L; ++l) load_leaf<T, ALIGNED>(arow, (int64_t)(gl * L + l) * kLeaf, n, a[l]);
  const int gbase = lane & ~(LG - 1);
  // Column indices come LG at a time (one coalesced load per group, then ds_bpermute), so the
  // B-row loads of a batch never wait behind a dependent index load; lane t keeps the result of
  // the batch's t-th nonzero and the group stores LG results with one coalesced store.
  for (int64_t jb = j0; jb < j1; jb += LG) {
    const int cnt = (int)((j1 - jb) < LG ? (j1 - jb) : LG);
    const I myc = gl < cnt ? col[jb + gl] : I(0);
    A res = A(0);
    for (int k = 0; k < cnt; k += U) {
      A bv[U][L][kLeaf];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t cu = (int64_t)__shfl((int64_t)myc, gbase + ((k + u) & (LG - 1)), 64);
        if (k + u < cnt) {
          // a column outside [0, k): the forward gathered a zero row (zero_row_leaves)
          const T* brow = B + cu * ldb;
          const bool in = (uint64_t)cu < (uint64_t)kb;
#pragma unroll
          for (int l = 0; l < L; ++l) load_leaf<T, ALIGNED>(brow, in ? (int64_t)(gl * L + l) * kLeaf : n, n, bv[u][l]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u < cnt) {
          A leaf[L];
#pragma unroll
          for (int l = 0; l < L; ++l) {
            A s = A(0);
#pragma unroll
            for (int e = 0; e < kLeaf; ++e) s = s + a[l][e] * bv[u][l][e];
            leaf[l] = s;
          }
#pragma unroll
          for (int w = 1; w < L; w <<= 1)
#pragma unroll
            for (int l = 0; l < L; l += 2 * w) leaf[l] = leaf[l] + leaf[l + w];
          A t = leaf[0];
#pragma unroll
          for (int w = 1; w < LG; w <<= 1) t = t + __shfl_xor(t, w, 64);
          if (gl == k + u) res = t;
        }
      }
    }
    if (gl < cnt) out[jb + gl] = Num<T>::store(res);
  }
}

// n > 2048: the padded leaves are cut into tiles of kWideLeaves (one wave, 4 leaves per lane);
// each tile's value is its 256-leaf pairwise tree (the butterfly of the narrow kernel) and the
// tile values are added pairwise in tile order through a binary-counter stack.  The pairwise tree
// over all padded leaves is exactly the tree over its 256-leaf subtrees, so the contract's order
// (8-element leaves, zero-padded to a power of two, pairwise) is unchanged.  One wave per row or
// hub chunk; the dC tile is reloaded per batch of 64 nonzeros (only for these wide rows).
constexpr int kWideLeaves = 256;
constexpr int kMaxTilesLog = 6;  // n <= 2048 * 64 = 131072

template <typename T, typename I, bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
    sddmm_wide_kernel(const I* __restrict__ rp, const I* __restrict__ col, const T* __restrict__ dC,
                      int64_t ldc, const T* __restrict__ B, int64_t ldb, int64_t kb,
                      T* __restrict__ out, int64_t row_begin, int64_t nrows, int64_t n,
                      int64_t chunk, int tiles,
                      const unsigned long long* __restrict__ counters,
                      const int64_t* __restrict__ items, const int64_t* __restrict__ order,
                      int64_t block_base, unsigned* err) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  constexpr int L = kWideLeaves / 64, U = 2;
  if (sddmm_plan_invalid(counters, block_base, err, rp, row_begin, nrows, out)) return;
  const int lane = threadIdx.x & 63;
  const int64_t g = (block_base + (int64_t)blockIdx.x) * (kBlock / 64) +
                    __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t lr, j0, j1;
  if (!sddmm_item<I>(rp, g, row_begin, nrows, chunk, counters, items, order, &lr, &j0, &j1)) return;
  const T* arow = dC + lr * ldc;
  for (int64_t jb = j0; jb < j1; jb += 64) {
    const int cnt = (int)((j1 - jb) < 64 ? (j1 - jb) : 64);
    const I myc = lane < cnt ? col[jb + lane] : I(0);
    A stk[kMaxTilesLog + 1];
#pragma unroll
    for (int l = 0; l <= kMaxTilesLog; ++l) stk[l] = A(0);
    for (int t = 0; t < tiles; ++t) {
      const int64_t leaf0 = (int64_t)t * kWideLeaves + (int64_t)lane * L;
      A a[L][kLeaf];
#pragma unroll
      for (int l = 0; l < L; ++l) load_leaf<T, ALIGNED>(arow, (leaf0 + l) * kLeaf, n, a[l]);
      A tv = A(0);
      for (int k = 0; k < cnt; k += U) {
        A bv[U][L][kLeaf];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t cu = (int64_t)__shfl((int64_t)myc, (k + u) & 63, 64);
          if (k + u < cnt) {
            const T* brow = B + cu * ldb;
            const bool in = (uint64_t)cu < (uint64_t)kb;  // else a zero row
#pragma unroll
            for (int l = 0; l < L; ++l) load_leaf<T, ALIGNED>(brow, in ? (leaf0 + l) * kLeaf : n, n, bv[u][l]);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (k + u < cnt) {
            A leaf[L];
#pragma unroll
            for (int l = 0; l < L; ++l) {
              A sl = A(0);
#pragma unroll
              for (int e = 0; e < kLeaf; ++e) sl = sl + a[l][e] * bv[u][l][e];
              leaf[l] = sl;
            }
#pragma unroll
            for (int w = 1; w < L; w <<= 1)
#pragma unroll
              for (int l = 0; l < L; l += 2 * w) leaf[l] = leaf[l] + leaf[l + w];
            A x = leaf[0];
#pragma unroll
            for (int w = 1; w < 64; w <<= 1) x = x + __shfl_xor(x, w, 64);
            if (lane == k + u) tv = x;
          }
        }
      }
      // pairwise merge of tile t into the stack: left operands are the earlier subtrees
      A v = tv;
      bool done = false;
#pragma unroll
      for (int l = 0; l <= kMaxTilesLog; ++l) {
        if (!done) {
          if ((t >> l) & 1) {
            v = stk[l] + v;
          } else {
            stk[l] = v;
            done = true;
          }
        }
      }
    }
    A res = A(0);
#pragma unroll
    for (int l = 0; l <= kMaxTilesLog; ++l)
      if ((1 << l) == tiles) res = stk[l];
    if (lane < cnt) out[jb + lane] = Num<T>::store(res);
  }
}

struct SddmmArgs {
  hipStream_t s;
  const void *rp, *col, *dC, *B;
  void* out;
  int64_t ldc, ldb, row_begin, nrows, n, nnz, k;
  void* ws;
  size_t ws_bytes;
  bool planned;  // ws already holds this launch's plan (ofx_sddmm_csr_plan): no planner launch
};

// Work layout only: every dv[j] is its own dot product, so how rows are cut into items never
// changes a bit.  The forward's default split (65536 / n, part of ITS numeric contract) made the
// narrow kernel's hub chunks 1-2k (N=64) and 2-4k (N=32) nonzeros long: one lane-group walks a
// chunk in chunk / U dependent rounds, and on a power-law graph those chains set the launch time
// (1M power-law, N=32: 1.67 ms, slower than N=64).  Items of at most kSddmmChunk nonzeros keep the
// chains short; the wide kernel (n > 2048, one wave per item) keeps the forward's cut.
constexpr int64_t kSddmmChunk = 256;
constexpr int64_t kMaxNarrowN = 256 * kLeaf;  // sddmm_aligned's narrow configurations

Schedule sddmm_schedule(int64_t n) {
  Schedule s = resolve_schedule(n, nullptr);
  if (n <= kMaxNarrowN) s.split = s.chunk = kSddmmChunk;
  return s;
}

#ifndef OFX_SD_U
#define OFX_SD_U 0
#endif
#ifndef OFX_SD_LG8
#define OFX_SD_LG8 8
#endif
#ifndef OFX_SD_LG16
#define OFX_SD_LG16 16
#endif
template <typename T, typename I, int LG, int L, bool ALIGNED>
int sddmm_cfg(const SddmmArgs& a) {
  constexpr int U = OFX_SD_U > 0 ? OFX_SD_U : (L >= 4 ? 2 : 4);
  constexpr int64_t GPB = (kBlock / 64) * (64 / LG);
  const Schedule sched = sddmm_schedule(a.n);
  const plan::WsLayout w = plan::ws_layout(a.nrows, a.nnz, 0, 0, sched);
  plan::WorkList wl{};
  if (w.total > 0) {
    OFX_REQUIRE(a.ws && a.ws_bytes >= w.total, OFX_EWORKSPACE,
                "sddmm_csr: workspace of %zu bytes < %zu required", a.ws_bytes, w.total);
    if (a.planned) {
      plan::worklist_of(w, static_cast<char*>(a.ws), &wl);
    } else {
      const int rc = plan::launch_plan<I>(a.s, static_cast<const I*>(a.rp), a.row_begin, a.nrows,
                                          a.nnz, sched, w, static_cast<char*>(a.ws), &wl);
      if (rc) return rc;
    }
  }
  const int64_t work = a.nrows + (w.total > 0 ? w.max_chunks : 0);
  const int64_t grid = (work + GPB - 1) / GPB;
  for (int64_t b0 = 0; b0 < grid; b0 += kLaunchBlocks) {  // < 2^31 threads per launch
    hipLaunchKernelGGL((sddmm_kernel<T, I, LG, L, U, ALIGNED>),
                       dim3((unsigned)std::min(kLaunchBlocks, grid - b0)), dim3(kBlock), 0, a.s,
                       static_cast<const I*>(a.rp), static_cast<const I*>(a.col),
                       static_cast<const T*>(a.dC), a.ldc, static_cast<const T*>(a.B), a.ldb, a.k,
                       static_cast<T*>(a.out), a.row_begin, a.nrows, a.n,
                       w.total > 0 ? sched.chunk : INT64_MAX, wl.counters, wl.items, wl.order, b0,
                       w.total > 0 ? device_error_words() : nullptr);
    OFX_HIP_CHECK(hipGetLastError());
  }
  return OFX_OK;
}

template <typename T, typename I, bool ALIGNED>
int sddmm_aligned(const SddmmArgs& a) {
  const int64_t leaves = (a.n + kLeaf - 1) / kLeaf;
  if (leaves <= 1) return sddmm_cfg<T, I, 1, 1, ALIGNED>(a);
  if (leaves <= 2) return sddmm_cfg<T, I, 2, 1, ALIGNED>(a);
  if (leaves <= 4) return sddmm_cfg<T, I, 4, 1, ALIGNED>(a);
  if (leaves <= 8) return sddmm_cfg<T, I, OFX_SD_LG8, 8 / OFX_SD_LG8, ALIGNED>(a);
  if (leaves <= 16) return sddmm_cfg<T, I, OFX_SD_LG16, 16 / OFX_SD_LG16, ALIGNED>(a);
  if (leaves <= 32) return sddmm_cfg<T, I, 32, 1, ALIGNED>(a);
  if (leaves <= 64) return sddmm_cfg<T, I, 64, 1, ALIGNED>(a);
  if (leaves <= 128) return sddmm_cfg<T, I, 64, 2, ALIGNED>(a);
  if (leaves <= 256) return sddmm_cfg<T, I, 64, 4, ALIGNED>(a);
  int64_t tiles = 1;
  while (tiles * kWideLeaves < leaves) tiles *= 2;
  OFX_REQUIRE(tiles <= (1 << kMaxTilesLog), OFX_EUNSUPPORTED,
              "sddmm_csr: n=%lld > %d is not supported", (long long)a.n,
              kWideLeaves * kLeaf << kMaxTilesLog);
  const Schedule sched = sddmm_schedule(a.n);
  const plan::WsLayout w = plan::ws_layout(a.nrows, a.nnz, 0, 0, sched);
  plan::WorkList wl{};
  if (w.total > 0) {
    OFX_REQUIRE(a.ws && a.ws_bytes >= w.total, OFX_EWORKSPACE,
                "sddmm_csr: workspace of %zu bytes < %zu required", a.ws_bytes, w.total);
    if (a.planned) {
      plan::worklist_of(w, static_cast<char*>(a.ws), &wl);
    } else {
      const int rc = plan::launch_plan<I>(a.s, static_cast<const I*>(a.rp), a.row_begin, a.nrows,
                                          a.nnz, sched, w, static_cast<char*>(a.ws), &wl);
      if (rc) return rc;
    }
  }
  const int64_t work = a.nrows + (w.total > 0 ? w.max_chunks : 0);
  const int64_t grid = (work + kBlock / 64 - 1) / (kBlock / 64);
  for (int64_t b0 = 0; b0 < grid; b0 += kLaunchBlocks) {  // < 2^31 threads per launch
    hipLaunchKernelGGL((sddmm_wide_kernel<T, I, ALIGNED>),
                       dim3((unsigned)std::min(kLaunchBlocks, grid - b0)), dim3(kBlock), 0, a.s,
                       static_cast<const I*>(a.rp), static_cast<const I*>(a.col),
                       static_cast<const T*>(a.dC), a.ldc, static_cast<const T*>(a.B), a.ldb, a.k,
                       static_cast<T*>(a.out), a.row_begin, a.nrows, a.n,
                       w.total > 0 ? sched.chunk : INT64_MAX, (int)tiles, wl.counters, wl.items,
                       wl.order, b0, w.total > 0 ? device_error_words() : nullptr);
    OFX_HIP_CHECK(hipGetLastError());
  }
  return OFX_OK;
}

template <typename T, typename I>
int sddmm_typed(const SddmmArgs& a) {
  const bool aligned = a.n % kLeaf == 0 && a.ldc % kLeaf == 0 && a.ldb % kLeaf == 0 &&
                       ((uintptr_t)a.dC % 16) == 0 && ((uintptr_t)a.B % 16) == 0 &&
                       ((size_t)a.ldc * sizeof(T)) % 16 == 0 && ((size_t)a.ldb * sizeof(T)) % 16 == 0;
  return aligned ? sddmm_aligned<T, I, true>(a) : sddmm_aligned<T, I, false>(a);
}

template <typename I>
int sddmm_idx(int val_dtype, const SddmmArgs& a) {
  switch (val_dtype) {
    case OFX_DT_FLOAT: return sddmm_typed<float, I>(a);
    case OFX_DT_DOUBLE: return sddmm_typed<double, I>(a);
    case OFX_DT_BFLOAT16: return sddmm_typed<bf16, I>(a);
    case OFX_DT_FLOAT16: return sddmm_typed<f16, I>(a);
    default: return fail(OFX_EUNSUPPORTED, "sddmm_csr: unsupported value dtype %d", val_dtype);
  }
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_csr_transpose_workspace_size(int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                                size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes && m >= 0 && k >= 0 && nnz >= 0, OFX_EINVAL, "csr_transpose: bad arguments");
    OFX_REQUIRE(nnz <= INT32_MAX, OFX_EINVAL, "csr_transpose: nnz > 2^31-1 is not supported");
    size_t cub = 0;
    if (idx_dtype == OFX_DT_INT32) return transpose_ws<int32_t>(nnz, k, bytes, &cub);
    if (idx_dtype == OFX_DT_INT64) return transpose_ws<int64_t>(nnz, k, bytes, &cub);
    return fail(OFX_EUNSUPPORTED, "csr_transpose: index dtype %d is not int32/int64", idx_dtype);
  });
}

extern "C" int ofx_csr_transpose(void* stream, int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                 const void* row_ptr, const void* col_idx, void* out_row_ptr,
                                 void* out_col_idx, void* out_perm, void* workspace,
                                 size_t workspace_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(m >= 0 && k >= 0 && nnz >= 0 && row_ptr && out_row_ptr &&
                    (nnz == 0 || (col_idx && out_col_idx && out_perm)),
                OFX_EINVAL, "csr_transpose: bad arguments");
    OFX_REQUIRE(nnz <= INT32_MAX, OFX_EINVAL, "csr_transpose: nnz > 2^31-1 is not supported");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (idx_dtype == OFX_DT_INT32)
      return transpose<int32_t>(s, m, k, nnz, (const int32_t*)row_ptr, (const int32_t*)col_idx,
                                (int32_t*)out_row_ptr, (int32_t*)out_col_idx, (int32_t*)out_perm,
                                workspace, workspace_bytes);
    if (idx_dtype == OFX_DT_INT64)
      return transpose<int64_t>(s, m, k, nnz, (const int64_t*)row_ptr, (const int64_t*)col_idx,
                                (int64_t*)out_row_ptr, (int64_t*)out_col_idx, (int64_t*)out_perm,
                                workspace, workspace_bytes);
    return fail(OFX_EUNSUPPORTED, "csr_transpose: index dtype %d is not int32/int64", idx_dtype);
  });
}

extern "C" int ofx_gather_values(void* stream, int idx_dtype, int val_dtype, int64_t nnz,
                                 const void* perm, const void* src, void* dst) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (nnz == 0) return OFX_OK;
    OFX_REQUIRE(perm && src && dst, OFX_EINVAL, "gather_values: NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned g = (unsigned)std::min<int64_t>((nnz + kBlock - 1) / kBlock, 65536);
    auto go = [&](auto* ip) -> int {
      using I = std::remove_const_t<std::remove_pointer_t<decltype(ip)>>;
      switch (dtype_size(val_dtype)) {
        case 2:
          hipLaunchKernelGGL((gather_values_kernel<uint16_t, I>), dim3(g), dim3(kBlock), 0, s,
                             (const I*)perm, (const uint16_t*)src, nnz, (uint16_t*)dst);
          break;
        case 4:
          hipLaunchKernelGGL((gather_values_kernel<uint32_t, I>), dim3(g), dim3(kBlock), 0, s,
                             (const I*)perm, (const uint32_t*)src, nnz, (uint32_t*)dst);
          break;
        case 8:
          hipLaunchKernelGGL((gather_values_kernel<uint64_t, I>), dim3(g), dim3(kBlock), 0, s,
                             (const I*)perm, (const uint64_t*)src, nnz, (uint64_t*)dst);
          break;
        default: return fail(OFX_EUNSUPPORTED, "gather_values: bad value dtype %d", val_dtype);
      }
      OFX_HIP_CHECK(hipGetLastError());
      return OFX_OK;
    };
    OFX_REQUIRE(is_value_dtype(val_dtype) || is_index_dtype(val_dtype), OFX_EUNSUPPORTED,
                "gather_values: bad value dtype %d", val_dtype);
    if (idx_dtype == OFX_DT_INT32) return go((const int32_t*)nullptr);
    if (idx_dtype == OFX_DT_INT64) return go((const int64_t*)nullptr);
    return fail(OFX_EUNSUPPORTED, "gather_values: bad index dtype %d", idx_dtype);
  });
}

extern "C" int ofx_sddmm_csr_workspace_size(int idx_dtype, int val_dtype, int64_t m, int64_t n,
                                            int64_t nnz, size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes && m >= 0 && n >= 0 && nnz >= 0, OFX_EINVAL, "sddmm_csr: bad arguments");
    OFX_REQUIRE(is_index_dtype(idx_dtype) && is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
                "sddmm_csr: unsupported dtypes (%d, %d)", idx_dtype, val_dtype);
    *bytes = plan::ws_layout(m, nnz, 0, 0, sddmm_schedule(n)).total;
    return OFX_OK;
  });
}

extern "C" int ofx_sddmm_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                             int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                             const void* a, int64_t lda, const void* b, int64_t ldb, void* out,
                             int64_t row_begin, int64_t row_end, void* workspace,
                             size_t workspace_bytes) {
  return ofx_sddmm_csr_ex(stream, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, a, lda, b,
                          ldb, out, row_begin, row_end, workspace, workspace_bytes, nullptr);
}

// ofx_sddmm_csr with options: only `planned` is read (the workspace holds the plan
// ofx_sddmm_csr_plan built for this row_ptr, row range and n; the launch skips the planner).
extern "C" int ofx_sddmm_csr_ex(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                                int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                                const void* a, int64_t lda, const void* b, int64_t ldb, void* out,
                                int64_t row_begin, int64_t row_end, void* workspace,
                                size_t workspace_bytes, const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_TAKE_DEVICE_ERROR("sddmm_csr");  // an earlier launch's loud failure (spmm_plan.h)
    OFX_READ_OPTIONS(opts, "sddmm_csr");  // NULL: every default (planned = 0)
    OFX_REQUIRE(is_index_dtype(idx_dtype) && is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
                "sddmm_csr: unsupported dtypes (%d, %d)", idx_dtype, val_dtype);
    OFX_REQUIRE(m >= 0 && k >= 0 && n >= 0 && nnz >= 0 && lda >= n && ldb >= n, OFX_EINVAL,
                "sddmm_csr: bad sizes");
    OFX_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= m, OFX_EINVAL,
                "sddmm_csr: row range [%lld, %lld) outside [0, %lld)", (long long)row_begin,
                (long long)row_end, (long long)m);
    if (row_end == row_begin || nnz == 0) return OFX_OK;
    OFX_REQUIRE(row_ptr && col_idx && out && (n == 0 || (a && b)), OFX_EINVAL,
                "sddmm_csr: NULL pointer");
    if (n == 0) return fail(OFX_EINVAL, "sddmm_csr: n == 0 (use a zero fill)");
    SddmmArgs args{static_cast<hipStream_t>(stream), row_ptr, col_idx, a, b, out, lda, ldb,
                   row_begin, row_end - row_begin, n, nnz, k, workspace, workspace_bytes,
                   opts->planned != 0};
    if (idx_dtype == OFX_DT_INT32) return sddmm_idx<int32_t>(val_dtype, args);
    return sddmm_idx<int64_t>(val_dtype, args);
  });
}

// The SDDMM's work-list plan alone, into `workspace` (ofx_sddmm_csr_workspace_size bytes), for
// later ofx_sddmm_csr_ex launches with planned = 1 over the same row_ptr, row range and n.
extern "C" int ofx_sddmm_csr_plan(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t n,
                                  int64_t nnz, const void* row_ptr, int64_t row_begin,
                                  int64_t row_end, void* workspace, size_t workspace_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_TAKE_DEVICE_ERROR("sddmm_csr_plan");
    OFX_REQUIRE(is_index_dtype(idx_dtype) && is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
                "sddmm_csr_plan: unsupported dtypes (%d, %d)", idx_dtype, val_dtype);
    OFX_REQUIRE(m >= 0 && n >= 0 && nnz >= 0 && 0 <= row_begin && row_begin <= row_end &&
                    row_end <= m, OFX_EINVAL, "sddmm_csr_plan: bad sizes or row range");
    const int64_t nrows = row_end - row_begin;
    if (nrows == 0 || nnz == 0 || n == 0) return OFX_OK;  // the launch plans nothing either
    const Schedule sched = sddmm_schedule(n);
    const plan::WsLayout w = plan::ws_layout(nrows, nnz, 0, 0, sched);
    if (w.total == 0) return OFX_OK;
    OFX_REQUIRE(row_ptr != nullptr, OFX_EINVAL, "sddmm_csr_plan: NULL row_ptr");
    OFX_REQUIRE(workspace != nullptr && workspace_bytes >= w.total, OFX_EWORKSPACE,
                "sddmm_csr_plan: workspace of %zu bytes < %zu required", workspace_bytes, w.total);
    plan::WorkList wl{};
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (idx_dtype == OFX_DT_INT32)
      return plan::launch_plan<int32_t>(s, static_cast<const int32_t*>(row_ptr), row_begin, nrows,
                                        nnz, sched, w, static_cast<char*>(workspace), &wl);
    return plan::launch_plan<int64_t>(s, static_cast<const int64_t*>(row_ptr), row_begin, nrows,
                                      nnz, sched, w, static_cast<char*>(workspace), &wl);
  });
}
