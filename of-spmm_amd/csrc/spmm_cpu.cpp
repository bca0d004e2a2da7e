// spmm_cpu.cpp — the DeviceType::kCPU kernel of op "spmm_csr" (SURVEY.md §8 row a2).
//
// Row-parallel over OpenMP in the idiom of CpuStream::ParallelFor
// (oneflow/core/ep/cpu/cpu_stream.h:104-145): rows are independent, each row is reduced by
// one thread in the contract order of spmm_common.h (gather -> multiply -> segment-sum,
// oneflow/user/kernels/gather_kernel_util.cpp:72-92 + unsorted_segment_sum_kernel_util.cpp:29-45),
// including the same hub-row chunking as the HIP kernel, so CPU and GPU produce identical bits.
// Thread count: OMP_NUM_THREADS like oneflow/core/job/env_global_objects_scope.cpp:90-99.
#pragma clang fp contract(off)

#include <omp.h>

#include <climits>
#include <vector>

#include "ofx_internal.h"
#include "spmm_common.h"

namespace ofx {
namespace {

// A column outside [0, k): the reference CPU gather zero-fills the gathered row of an index >= the
// table size (oneflow/user/kernels/gather_kernel_util.cpp:84-89), so the nonzero adds val * 0; a
// negative index fails its CHECK_GE (:80), reported here as OFX_EINVAL (`neg`).
template <typename T, typename I>
void row_sum(const I* col, const T* val, const T* B, int64_t ldb, int64_t k, int64_t n,
             int64_t j0, int64_t j1, typename Num<T>::acc* acc, bool* neg) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  for (int64_t c = 0; c < n; ++c) acc[c] = A(0);
  for (int64_t j = j0; j < j1; ++j) {
    const A v = Num<T>::load(val[j]);
    const int64_t cj = (int64_t)col[j];
    if (cj >= 0 && cj < k) {
      const T* brow = B + cj * ldb;
      for (int64_t c = 0; c < n; ++c) acc[c] = acc[c] + Num<T>::mul(v, Num<T>::load(brow[c]));
    } else {  // the zero-filled gathered row
      if (cj < 0) *neg = true;
      for (int64_t c = 0; c < n; ++c) acc[c] = acc[c] + Num<T>::mul(v, A(0));
    }
  }
}

template <typename T, typename I>
int cpu_spmm(int nthreads, int64_t k, int64_t n, const I* rp, const I* col, const T* val,
             const T* B, int64_t ldb, T* C, int64_t ldc, int64_t row_begin, int64_t row_end,
             const Schedule& s, const T* bias, int act) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  const int64_t rows = row_end - row_begin;
  bool any_neg = false;
#pragma omp parallel num_threads(nthreads) reduction(|| : any_neg)
  {
    std::vector<A> acc(n), part(n);
    bool neg = false;
#pragma omp for schedule(dynamic, 64)
    for (int64_t g = 0; g < rows; ++g) {
      const int64_t r = row_begin + g;
      const int64_t j0 = (int64_t)rp[r], j1 = (int64_t)rp[r + 1];
      const int64_t len = j1 - j0;
      if (len <= s.split) {
        row_sum<T, I>(col, val, B, ldb, k, n, j0, j1, acc.data(), &neg);
      } else {
        const int64_t nc = num_chunks(len, s.chunk);
        for (int64_t c = 0; c < n; ++c) acc[c] = A(0);
        for (int64_t q = 0; q < nc; ++q) {
          const int64_t a = j0 + q * s.chunk;
          const int64_t e = (q == nc - 1) ? j1 : a + s.chunk;
          row_sum<T, I>(col, val, B, ldb, k, n, a, e, part.data(), &neg);
          for (int64_t c = 0; c < n; ++c) acc[c] = acc[c] + part[c];
        }
      }
      T* out = C + g * ldc;
      for (int64_t c = 0; c < n; ++c) out[c] = epilogue<T>(acc[c], bias, c, act);
    }
    any_neg = any_neg || neg;
  }
  OFX_REQUIRE(!any_neg, OFX_EINVAL,
              "spmm_csr_cpu: negative column index (gather_kernel_util.cpp:80 CHECK_GE(idx, 0))");
  return OFX_OK;
}

template <typename I>
int cpu_dispatch(int nthreads, int val_dtype, int64_t k, int64_t n, const void* rp, const void* col,
                 const void* val, const void* b, int64_t ldb, void* c, int64_t ldc,
                 int64_t row_begin, int64_t row_end, const Schedule& s, const void* bias,
                 int act) {
  const I* r = static_cast<const I*>(rp);
  const I* ci = static_cast<const I*>(col);
  switch (val_dtype) {
    case OFX_DT_FLOAT:
      return cpu_spmm<float, I>(nthreads, k, n, r, ci, (const float*)val, (const float*)b, ldb,
                                (float*)c, ldc, row_begin, row_end, s, (const float*)bias, act);
    case OFX_DT_DOUBLE:
      return cpu_spmm<double, I>(nthreads, k, n, r, ci, (const double*)val, (const double*)b, ldb,
                                 (double*)c, ldc, row_begin, row_end, s, (const double*)bias, act);
    case OFX_DT_BFLOAT16:
      return cpu_spmm<bf16, I>(nthreads, k, n, r, ci, (const bf16*)val, (const bf16*)b, ldb,
                               (bf16*)c, ldc, row_begin, row_end, s, (const bf16*)bias, act);
    case OFX_DT_FLOAT16:
      return cpu_spmm<f16, I>(nthreads, k, n, r, ci, (const f16*)val, (const f16*)b, ldb, (f16*)c,
                              ldc, row_begin, row_end, s, (const f16*)bias, act);
    default: return fail(OFX_EUNSUPPORTED, "spmm_csr_cpu: unsupported value dtype %d", val_dtype);
  }
}

}  // namespace
}  // namespace ofx

using namespace ofx;

namespace ofx {
namespace {
int spmm_cpu_entry(int num_threads, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                   int64_t nnz, const void* row_ptr, const void* col_idx, const void* values,
                   const void* b, int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                   int64_t row_end, const void* bias, int act, const ofx_spmm_options* opts) {
  OFX_READ_OPTIONS(opts, "spmm_csr_cpu");
  OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED,
              "spmm_csr_cpu: index dtype %d is not int32/int64", idx_dtype);
  OFX_REQUIRE(is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
              "spmm_csr_cpu: unsupported value dtype %d", val_dtype);
  OFX_REQUIRE(m >= 0 && k >= 0 && n >= 0 && nnz >= 0, OFX_EINVAL, "spmm_csr_cpu: negative size");
  OFX_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= m, OFX_EINVAL,
              "spmm_csr_cpu: row range [%lld, %lld) outside [0, %lld)", (long long)row_begin,
              (long long)row_end, (long long)m);
  OFX_REQUIRE(ldb >= n && ldc >= n, OFX_EINVAL, "spmm_csr_cpu: ldb/ldc < n");
  OFX_REQUIRE(act == OFX_ACT_NONE || act == OFX_ACT_RELU, OFX_EINVAL,
              "spmm_csr_cpu: unknown activation %d", act);
  if (row_end == row_begin || n == 0) return OFX_OK;
  OFX_REQUIRE(row_ptr && c && (nnz == 0 || (col_idx && values && b)), OFX_EINVAL,
              "spmm_csr_cpu: NULL pointer");
  const int nt = num_threads > 0 ? num_threads : omp_get_max_threads();
  const Schedule s = resolve_schedule(n, opts);
  if (idx_dtype == OFX_DT_INT32)
    return cpu_dispatch<int32_t>(nt, val_dtype, k, n, row_ptr, col_idx, values, b, ldb, c, ldc,
                                 row_begin, row_end, s, bias, act);
  return cpu_dispatch<int64_t>(nt, val_dtype, k, n, row_ptr, col_idx, values, b, ldb, c, ldc,
                               row_begin, row_end, s, bias, act);
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_spmm_csr_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m,
                                int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                const void* col_idx, const void* values, const void* b,
                                int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                                int64_t row_end, const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return spmm_cpu_entry(num_threads, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, values,
                          b, ldb, c, ldc, row_begin, row_end, nullptr, OFX_ACT_NONE, opts);
  });
}

extern "C" int ofx_spmm_csr_fused_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m,
                                      int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                      const void* col_idx, const void* values, const void* b,
                                      int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                                      int64_t row_end, const void* bias, int activation,
                                      const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return spmm_cpu_entry(num_threads, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, values,
                          b, ldb, c, ldc, row_begin, row_end, bias, activation, opts);
  });
}

// ---- BalancedSplitter (oneflow/core/common/balanced_splitter.cpp:20-40) -------------------
extern "C" int ofx_balanced_range(int64_t total, int64_t parts, int64_t idx, int64_t* begin,
                                  int64_t* end) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(total >= 0 && parts > 0 && idx >= 0 && idx < parts && begin && end, OFX_EINVAL,
                "balanced_range: bad arguments (total=%lld parts=%lld idx=%lld)", (long long)total,
                (long long)parts, (long long)idx);
    const int64_t base = total / parts, extra = total % parts;
    // The first `extra` parts hold base+1 elements.
    const int64_t lo = idx < extra ? idx * (base + 1) : extra * (base + 1) + (idx - extra) * base;
    *begin = lo;
    *end = lo + base + (idx < extra ? 1 : 0);
    return OFX_OK;
  });
}

extern "C" int ofx_csr_row_slice_host(int idx_dtype, const void* row_ptr, int64_t row_begin,
                                      int64_t row_end, void* out_row_ptr, int64_t* nnz_begin,
                                      int64_t* nnz_end) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "csr_row_slice_host: bad dtype");
    OFX_REQUIRE(row_ptr && 0 <= row_begin && row_begin <= row_end, OFX_EINVAL,
                "csr_row_slice_host: bad arguments");
    auto run = [&](auto* rp, auto* out) {
      const int64_t base = (int64_t)rp[row_begin];
      if (out)
        for (int64_t i = 0; i <= row_end - row_begin; ++i)
          out[i] = (std::remove_pointer_t<decltype(out)>)((int64_t)rp[row_begin + i] - base);
      if (nnz_begin) *nnz_begin = base;
      if (nnz_end) *nnz_end = (int64_t)rp[row_end];
    };
    if (idx_dtype == OFX_DT_INT32)
      run(static_cast<const int32_t*>(row_ptr), static_cast<int32_t*>(out_row_ptr));
    else
      run(static_cast<const int64_t*>(row_ptr), static_cast<int64_t*>(out_row_ptr));
    return OFX_OK;
  });
}

// ---- backward building blocks on the host (DeviceType::kCPU; same bits as the HIP kernels) ---
namespace ofx {
namespace {

template <typename I>
void cpu_transpose(int64_t m, int64_t k, int64_t nnz, const I* rp, const I* col, I* out_rp,
                   I* out_col, I* out_perm) {
  // key k for a column outside [0, k): after row_ptr_T[k], never read (csrc/spmm_backward.hip
  // transpose_keys_kernel)
  auto key = [&](int64_t j) {
    const int64_t c = (int64_t)col[j];
    return (uint64_t)c < (uint64_t)k ? c : k;
  };
  std::vector<int64_t> cnt(k + 2, 0);
  for (int64_t j = 0; j < nnz; ++j) ++cnt[key(j) + 1];
  for (int64_t c = 0; c <= k; ++c) cnt[c + 1] += cnt[c];
  for (int64_t c = 0; c <= k; ++c) out_rp[c] = (I)cnt[c];
  for (int64_t r = 0; r < m; ++r)  // rows ascending -> stable within each column
    for (int64_t j = (int64_t)rp[r]; j < (int64_t)rp[r + 1]; ++j) {
      const int64_t pos = cnt[key(j)]++;
      out_col[pos] = (I)r;
      out_perm[pos] = (I)j;
    }
}

template <typename T, typename I>
void cpu_sddmm(int nthreads, int64_t k, int64_t n, const I* rp, const I* col, const T* a,
               int64_t lda, const T* b, int64_t ldb, T* out, int64_t row_begin, int64_t row_end) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  const int64_t leaves = (n + 7) / 8;
  int64_t padded = 1;
  while (padded < leaves) padded *= 2;
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<A> leaf(padded);
    const std::vector<T> zero(n, Num<T>::store(A(0)));  // the zero-filled row of a column outside [0, k)
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
      const T* arow = a + (r - row_begin) * lda;
      for (int64_t j = (int64_t)rp[r]; j < (int64_t)rp[r + 1]; ++j) {
        const int64_t cj = (int64_t)col[j];
        const T* brow = (uint64_t)cj < (uint64_t)k ? b + cj * ldb : zero.data();
        for (int64_t l = 0; l < padded; ++l) {
          A s = A(0);
          for (int64_t e = 8 * l; e < 8 * l + 8 && e < n; ++e)
            s = s + Num<T>::load(arow[e]) * Num<T>::load(brow[e]);
          leaf[l] = s;
        }
        for (int64_t w = 1; w < padded; w *= 2)
          for (int64_t l = 0; l < padded; l += 2 * w) leaf[l] = leaf[l] + leaf[l + w];
        out[j] = Num<T>::store(leaf[0]);
      }
    }
  }
}

}  // namespace
}  // namespace ofx

extern "C" int ofx_gather_values_host(int idx_dtype, int val_dtype, int64_t nnz, const void* perm,
                                      const void* src, void* dst) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "gather_values: bad index dtype %d",
                idx_dtype);
    const int vs = dtype_size(val_dtype);
    OFX_REQUIRE(vs == 2 || vs == 4 || vs == 8, OFX_EUNSUPPORTED, "gather_values: bad value dtype %d",
                val_dtype);
    OFX_REQUIRE(nnz >= 0 && (nnz == 0 || (perm && src && dst)), OFX_EINVAL,
                "gather_values: NULL argument");
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    for (int64_t t = 0; t < nnz; ++t) {
      const int64_t j = idx_dtype == OFX_DT_INT32 ? (int64_t) static_cast<const int32_t*>(perm)[t]
                                                  : static_cast<const int64_t*>(perm)[t];
      OFX_REQUIRE(j >= 0 && j < nnz, OFX_EINVAL, "gather_values: perm[%lld] = %lld outside [0, %lld)",
                  (long long)t, (long long)j, (long long)nnz);
      memcpy(d + (size_t)t * vs, s + (size_t)j * vs, (size_t)vs);
    }
    return OFX_OK;
  });
}

namespace ofx {
namespace {
// A negative column of nonzeros [j0, j1): the CPU gather's CHECK_GE(idx, 0)
// (gather_kernel_util.cpp:80), which the kCPU forward reports as OFX_EINVAL; the gradient ops
// of the same CPU operator report it the same way.
int negative_column(int idx_dtype, const void* col_idx, int64_t j0, int64_t j1) {
  bool neg = false;
  if (idx_dtype == OFX_DT_INT32) {
    const int32_t* c = static_cast<const int32_t*>(col_idx);
#pragma omp parallel for reduction(|| : neg) schedule(static)
    for (int64_t j = j0; j < j1; ++j) neg = neg || c[j] < 0;
  } else {
    const int64_t* c = static_cast<const int64_t*>(col_idx);
#pragma omp parallel for reduction(|| : neg) schedule(static)
    for (int64_t j = j0; j < j1; ++j) neg = neg || c[j] < 0;
  }
  return neg ? 1 : 0;
}
int64_t row_ptr_at(int idx_dtype, const void* row_ptr, int64_t r) {
  return idx_dtype == OFX_DT_INT32 ? (int64_t) static_cast<const int32_t*>(row_ptr)[r]
                                   : (int64_t) static_cast<const int64_t*>(row_ptr)[r];
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_csr_transpose_cpu(int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                     const void* row_ptr, const void* col_idx, void* out_row_ptr,
                                     void* out_col_idx, void* out_perm) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(m >= 0 && k >= 0 && nnz >= 0 && row_ptr && out_row_ptr &&
                    (nnz == 0 || (col_idx && out_col_idx && out_perm)),
                OFX_EINVAL, "csr_transpose_cpu: bad arguments");
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "csr_transpose_cpu: bad index dtype %d",
                idx_dtype);
    OFX_REQUIRE(nnz == 0 || !negative_column(idx_dtype, col_idx, 0, nnz), OFX_EINVAL,
                "csr_transpose_cpu: negative column index (gather_kernel_util.cpp:80 CHECK_GE(idx, 0))");
    if (idx_dtype == OFX_DT_INT32)
      cpu_transpose<int32_t>(m, k, nnz, (const int32_t*)row_ptr, (const int32_t*)col_idx,
                             (int32_t*)out_row_ptr, (int32_t*)out_col_idx, (int32_t*)out_perm);
    else if (idx_dtype == OFX_DT_INT64)
      cpu_transpose<int64_t>(m, k, nnz, (const int64_t*)row_ptr, (const int64_t*)col_idx,
                             (int64_t*)out_row_ptr, (int64_t*)out_col_idx, (int64_t*)out_perm);
    else
      return fail(OFX_EUNSUPPORTED, "csr_transpose_cpu: bad index dtype %d", idx_dtype);
    return OFX_OK;
  });
}

extern "C" int ofx_sddmm_csr_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m,
                                 int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                 const void* col_idx, const void* a, int64_t lda, const void* b,
                                 int64_t ldb, void* out, int64_t row_begin, int64_t row_end) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype) && is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
                "sddmm_csr_cpu: unsupported dtypes (%d, %d)", idx_dtype, val_dtype);
    OFX_REQUIRE(m >= 0 && k >= 0 && n > 0 && nnz >= 0 && lda >= n && ldb >= n && 0 <= row_begin &&
                    row_begin <= row_end && row_end <= m,
                OFX_EINVAL, "sddmm_csr_cpu: bad sizes");
    if (row_end == row_begin || nnz == 0) return OFX_OK;
    OFX_REQUIRE(!negative_column(idx_dtype, col_idx, row_ptr_at(idx_dtype, row_ptr, row_begin),
                                 row_ptr_at(idx_dtype, row_ptr, row_end)),
                OFX_EINVAL,
                "sddmm_csr_cpu: negative column index (gather_kernel_util.cpp:80 CHECK_GE(idx, 0))");
    const int nt = num_threads > 0 ? num_threads : omp_get_max_threads();
    auto run = [&](auto* ip) {
      using I = std::remove_const_t<std::remove_pointer_t<decltype(ip)>>;
      const I* rp = (const I*)row_ptr;
      const I* ci = (const I*)col_idx;
      switch (val_dtype) {
        case OFX_DT_FLOAT:
          cpu_sddmm<float, I>(nt, k, n, rp, ci, (const float*)a, lda, (const float*)b, ldb, (float*)out, row_begin, row_end);
          break;
        case OFX_DT_DOUBLE:
          cpu_sddmm<double, I>(nt, k, n, rp, ci, (const double*)a, lda, (const double*)b, ldb, (double*)out, row_begin, row_end);
          break;
        case OFX_DT_BFLOAT16:
          cpu_sddmm<bf16, I>(nt, k, n, rp, ci, (const bf16*)a, lda, (const bf16*)b, ldb, (bf16*)out, row_begin, row_end);
          break;
        default:
          cpu_sddmm<f16, I>(nt, k, n, rp, ci, (const f16*)a, lda, (const f16*)b, ldb, (f16*)out, row_begin, row_end);
          break;
      }
    };
    if (idx_dtype == OFX_DT_INT32) run((const int32_t*)nullptr);
    else run((const int64_t*)nullptr);
    return OFX_OK;
  });
}

// ---- COO -> CSR on the host (same output as csr_build.hip) ------------------------------------
#include <algorithm>
#include <numeric>

namespace ofx {
namespace {
template <typename T, typename I>
int64_t cpu_coo_to_csr(int64_t m, int64_t k, int64_t nnz, const I* row, const I* col, const T* val,
                       int merge, I* out_rp, I* out_col, T* out_val) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  std::vector<int64_t> perm(nnz);
  std::iota(perm.begin(), perm.end(), 0);
  auto key = [&](int64_t i) { return (uint64_t)row[i] * (uint64_t)k + (uint64_t)col[i]; };
  std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return key(a) < key(b); });
  int64_t o = 0;
  std::vector<int64_t> cnt(m + 1, 0);
  for (int64_t i = 0; i < nnz;) {
    int64_t e = i + 1;
    if (merge)
      while (e < nnz && key(perm[e]) == key(perm[i])) ++e;
    out_col[o] = col[perm[i]];
    if (val) {
      A acc = A(0);
      for (int64_t q = i; q < e; ++q) acc = acc + Num<T>::load(val[perm[q]]);
      out_val[o] = Num<T>::store(acc);
    }
    ++cnt[(int64_t)row[perm[i]] + 1];
    ++o;
    i = e;
  }
  for (int64_t r = 0; r < m; ++r) cnt[r + 1] += cnt[r];
  for (int64_t r = 0; r <= m; ++r) out_rp[r] = (I)cnt[r];
  return o;
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_coo_to_csr_cpu(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t nnz,
                                  const void* row, const void* col, const void* values,
                                  int merge_duplicates, void* out_row_ptr, void* out_col_idx,
                                  void* out_values, int64_t* out_nnz) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(m >= 0 && k >= 0 && nnz >= 0 && out_row_ptr && out_nnz &&
                    (nnz == 0 || (row && col && out_col_idx)),
                OFX_EINVAL, "coo_to_csr_cpu: bad arguments");
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "coo_to_csr_cpu: bad index dtype");
    OFX_REQUIRE((values == nullptr) == (out_values == nullptr), OFX_EINVAL,
                "coo_to_csr_cpu: values and out_values must both be given or both be NULL");
    auto run = [&](auto* ip) -> int {
      using I = std::remove_const_t<std::remove_pointer_t<decltype(ip)>>;
      const I* r = (const I*)row;
      const I* c = (const I*)col;
      for (int64_t i = 0; i < nnz; ++i)
        OFX_REQUIRE(r[i] >= 0 && r[i] < m && c[i] >= 0 && c[i] < k, OFX_EINVAL,
                    "coo_to_csr_cpu: entry %lld (%lld, %lld) outside %lld x %lld", (long long)i,
                    (long long)r[i], (long long)c[i], (long long)m, (long long)k);
      const int vdt = values ? val_dtype : OFX_DT_FLOAT;
      switch (vdt) {
        case OFX_DT_FLOAT:
          *out_nnz = cpu_coo_to_csr<float, I>(m, k, nnz, r, c, (const float*)values, merge_duplicates,
                                              (I*)out_row_ptr, (I*)out_col_idx, (float*)out_values);
          break;
        case OFX_DT_DOUBLE:
          *out_nnz = cpu_coo_to_csr<double, I>(m, k, nnz, r, c, (const double*)values, merge_duplicates,
                                               (I*)out_row_ptr, (I*)out_col_idx, (double*)out_values);
          break;
        case OFX_DT_BFLOAT16:
          *out_nnz = cpu_coo_to_csr<bf16, I>(m, k, nnz, r, c, (const bf16*)values, merge_duplicates,
                                             (I*)out_row_ptr, (I*)out_col_idx, (bf16*)out_values);
          break;
        case OFX_DT_FLOAT16:
          *out_nnz = cpu_coo_to_csr<f16, I>(m, k, nnz, r, c, (const f16*)values, merge_duplicates,
                                            (I*)out_row_ptr, (I*)out_col_idx, (f16*)out_values);
          break;
        default: return fail(OFX_EUNSUPPORTED, "coo_to_csr_cpu: bad value dtype %d", vdt);
      }
      return OFX_OK;
    };
    if (idx_dtype == OFX_DT_INT32) return run((const int32_t*)nullptr);
    return run((const int64_t*)nullptr);
  });
}

// ---- fused-epilogue backward on the host (csrc/epilogue_grad.hip states the order) -----------
namespace {

constexpr int64_t kGradRows = 2048;  // same chunking as the HIP kernel
constexpr int kGradLanes = 8;

template <typename T>
int relu_bias_grad_cpu(int num_threads, int64_t m, int64_t n, const T* y, int64_t ldy,
                       const T* dy, int64_t lddy, T* dx, int64_t lddx, T* d_bias, int relu) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  const int64_t nch = (m + kGradRows - 1) / kGradRows;
  std::vector<A> part(d_bias ? (size_t)nch * (size_t)n : 0);
  if (num_threads > 0) omp_set_num_threads(num_threads);
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < nch; ++c) {
    const int64_t r1 = (c + 1) * kGradRows < m ? (c + 1) * kGradRows : m;
    for (int64_t j = 0; j < n; ++j) {
      A acc = A(0);
      for (int64_t r = c * kGradRows; r < r1; ++r) {
        const A g = (relu && !(Num<T>::load(y[r * ldy + j]) > A(0))) ? A(0)
                                                                       : Num<T>::load(dy[r * lddy + j]);
        if (dx) dx[r * lddx + j] = Num<T>::store(g);
        acc = acc + g;
      }
      if (d_bias) part[(size_t)c * n + j] = acc;
    }
  }
  if (d_bias) {
    for (int64_t j = 0; j < n; ++j) {
      A lane[kGradLanes];
      for (int l = 0; l < kGradLanes; ++l) {
        A acc = A(0);
        for (int64_t c = l; c < nch; c += kGradLanes) acc = acc + part[(size_t)c * n + j];
        lane[l] = acc;
      }
      for (int s = kGradLanes / 2; s >= 1; s >>= 1)
        for (int l = 0; l < s; ++l) lane[l] = lane[l] + lane[l + s];
      d_bias[j] = Num<T>::store(lane[0]);
    }
  }
  return OFX_OK;
}

}  // namespace

extern "C" int ofx_relu_bias_grad_cpu(int num_threads, int val_dtype, int64_t m, int64_t n,
                                      const void* y, int64_t ldy, const void* dy, int64_t lddy,
                                      void* dx, int64_t lddx, void* d_bias, int relu) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_value_dtype(val_dtype), OFX_EUNSUPPORTED, "relu_bias_grad: bad dtype %d",
                val_dtype);
    OFX_REQUIRE(m >= 0 && n >= 0, OFX_EINVAL, "relu_bias_grad: negative size");
    if (n == 0) return OFX_OK;
    OFX_REQUIRE(m == 0 || (dy && (!relu || y) && lddy >= n && (!relu || ldy >= n)), OFX_EINVAL,
                "relu_bias_grad: NULL input or leading dimension < n");
    OFX_REQUIRE(dx == nullptr || lddx >= n, OFX_EINVAL, "relu_bias_grad: lddx < n");
  #define OFX_RBG(T)                                                                               \
    return relu_bias_grad_cpu<T>(num_threads, m, n, static_cast<const T*>(y), ldy,                 \
                                 static_cast<const T*>(dy), lddy, static_cast<T*>(dx), lddx,       \
                                 static_cast<T*>(d_bias), relu)
    switch (val_dtype) {
      case OFX_DT_FLOAT: OFX_RBG(float);
      case OFX_DT_DOUBLE: OFX_RBG(double);
      case OFX_DT_BFLOAT16: OFX_RBG(bf16);
      default: OFX_RBG(f16);
    }
  #undef OFX_RBG
  });
}
