// spmm_csr.hip — the C-ABI of the CSR x dense SpMM forward (op "spmm_csr") and its small helper
// kernels (CSR validation, row slices, synthetic dense inputs).  The forward kernels themselves
// (plan / main / small form / reduce) are in spmm_csr_impl.h, compiled once per
// (value, index) type pair in spmm_inst_*.hip and dispatched from here through launch_typed.
//
// Reference semantics (OneFlow has no SpMM): the composition
//   gather rows B[col[j]]      oneflow/user/kernels/gather_kernel_util.cpp:72-92
//   multiply by val[j]
//   unsorted_segment_sum       oneflow/user/kernels/unsorted_segment_sum_kernel_util.cpp:29-45
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <type_traits>

#include "ofx_internal.h"
#include "spmm_common.h"
#include "spmm_plan.h"
#include "spmm_launch.h"
#include "dbg_bounds.h"

namespace ofx {
namespace {

using plan::ws_layout;

// ---- validation / slicing / synthetic dense ------------------------------------------------
template <typename I>
__global__ void csr_validate_kernel(const I* __restrict__ rp, const I* __restrict__ col,
                                    int64_t m, int64_t k, int64_t nnz, unsigned int* flag) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = t0; i <= m; i += stride) {
    const int64_t v = (int64_t)rp[i];
    bool bad = (i == 0 && v != 0) || (i == m && v != nnz) || v < 0 || v > nnz;
    if (!bad && i < m) bad = (int64_t)rp[i + 1] < v;
    if (bad) atomicMax(flag, 1u);
  }
  for (int64_t j = t0; j < nnz; j += stride) {
    const int64_t c = (int64_t)col[j];
    if (c < 0 || c >= k) atomicMax(flag, 2u);
  }
}

template <typename I>
__global__ void csr_row_slice_kernel(const I* __restrict__ rp, int64_t row_begin, int64_t rows,
                                     I* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= rows) out[i] = (I)((int64_t)rp[row_begin + i] - (int64_t)rp[row_begin]);
}

template <typename T>
__global__ void synth_dense_kernel(int64_t r_begin, int64_t rows, int64_t n, int64_t ld,
                                   uint64_t seed, int exact, T* __restrict__ out) {
  const int64_t total = rows * n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t rr = i / n, cc = i - rr * n;
    const uint64_t h = hash2(seed, (uint64_t)((r_begin + rr) * n + cc));
    const float f = exact ? exact_dense(h) : u_pm1(h);
    out[rr * ld + cc] = Num<T>::store((typename Num<T>::acc)f);
  }
}

template <typename I>
int launch_idx(int val_dtype, const Launch& L) {
  switch (val_dtype) {
    case OFX_DT_FLOAT: return launch_typed<float, I>(L);
    case OFX_DT_DOUBLE: return launch_typed<double, I>(L);
    case OFX_DT_BFLOAT16: return launch_typed<bf16, I>(L);
    case OFX_DT_FLOAT16: return launch_typed<f16, I>(L);
    default: return fail(OFX_EUNSUPPORTED, "spmm_csr: unsupported value dtype %d", val_dtype);
  }
}

size_t acc_bytes_of(int val_dtype) { return val_dtype == OFX_DT_DOUBLE ? 8 : 4; }

int check_common(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n, int64_t nnz) {
  OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED,
              "spmm_csr: index dtype %d is not int32/int64", idx_dtype);
  OFX_REQUIRE(is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
              "spmm_csr: value dtype %d is not float/double/float16/bfloat16", val_dtype);
  OFX_REQUIRE(m >= 0 && k >= 0 && n >= 0 && nnz >= 0, OFX_EINVAL,
              "spmm_csr: negative size (m=%lld k=%lld n=%lld nnz=%lld)", (long long)m,
              (long long)k, (long long)n, (long long)nnz);
  OFX_REQUIRE(idx_dtype == OFX_DT_INT64 || (nnz <= INT32_MAX && k <= INT32_MAX), OFX_EINVAL,
              "spmm_csr: int32 indices cannot address nnz=%lld / k=%lld", (long long)nnz,
              (long long)k);
  return OFX_OK;
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int64_t ofx_spmm_default_split(int64_t n) { return default_split(n); }

extern "C" int ofx_spmm_csr_workspace_size(int idx_dtype, int val_dtype, int64_t m, int64_t k,
                                           int64_t n, int64_t nnz, const ofx_spmm_options* opts,
                                           size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes != nullptr, OFX_EINVAL, "spmm_csr_workspace_size: bytes is NULL");
    OFX_READ_OPTIONS(opts, "spmm_csr_workspace_size");
    int rc = check_common(idx_dtype, val_dtype, m, k, n, nnz);
    if (rc) return rc;
    const Schedule s = launch_schedule(m, nnz, n, resolve_schedule(n, opts));
    *bytes = use_small_form(m, nnz, n, s) ? 0 : ws_layout(m, nnz, n, acc_bytes_of(val_dtype), s).total;
    return OFX_OK;
  });
}

namespace ofx {
namespace {
int spmm_entry(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
               int64_t nnz, const void* row_ptr, const void* col_idx, const void* values,
               const void* values_perm, const void* b, int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
               int64_t row_end, const void* bias, int act, void* workspace,
               size_t workspace_bytes, const ofx_spmm_options* opts) {
  OFX_TAKE_DEVICE_ERROR("spmm_csr");  // an earlier launch's loud failure (spmm_plan.h)
  OFX_READ_OPTIONS(opts, "spmm_csr");
  int rc = check_common(idx_dtype, val_dtype, m, k, n, nnz);
  if (rc) return rc;
  OFX_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= m, OFX_EINVAL,
              "spmm_csr: row range [%lld, %lld) outside [0, %lld)", (long long)row_begin,
              (long long)row_end, (long long)m);
  OFX_REQUIRE(ldb >= n && ldc >= n, OFX_EINVAL, "spmm_csr: ldb=%lld / ldc=%lld < n=%lld",
              (long long)ldb, (long long)ldc, (long long)n);
  OFX_REQUIRE(act == OFX_ACT_NONE || act == OFX_ACT_RELU, OFX_EINVAL,
              "spmm_csr: unknown activation %d", act);
  const int64_t nrows = row_end - row_begin;
  if (nrows == 0 || n == 0) return OFX_OK;  // nothing to write
  OFX_REQUIRE(row_ptr && c, OFX_EINVAL, "spmm_csr: NULL row_ptr or output");
  OFX_REQUIRE(nnz == 0 || (col_idx && values && b), OFX_EINVAL,
              "spmm_csr: NULL col_idx/values/b with nnz=%lld", (long long)nnz);
  const int64_t nnz_est = launch_nnz(m, nrows, nnz, opts);
  Launch L{static_cast<hipStream_t>(stream), row_ptr, col_idx, values, b, c, ldb, ldc,
           row_begin, nrows, n, nnz, launch_schedule(nrows, nnz_est, n, resolve_schedule(n, opts)),
           workspace, workspace_bytes,
           bias, act, k, values_perm, nnz_est};
  if (idx_dtype == OFX_DT_INT32) return launch_idx<int32_t>(val_dtype, L);
  return launch_idx<int64_t>(val_dtype, L);
}
}  // namespace
}  // namespace ofx

extern "C" int ofx_spmm_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                            int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                            const void* values, const void* b, int64_t ldb, void* c, int64_t ldc,
                            int64_t row_begin, int64_t row_end, void* workspace,
                            size_t workspace_bytes, const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return spmm_entry(stream, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, values, nullptr,
                      b, ldb, c, ldc, row_begin, row_end, nullptr, OFX_ACT_NONE, workspace,
                      workspace_bytes, opts);
  });
}

// The configuration the launch of ofx_spmm_csr with these arguments would take (form, lane layout,
// loads in flight, flags), written to `buf` as "form=<small|mid|narrow|prefetch|bandwidth> ...";
// nothing is launched and no pointer is dereferenced (b and c only enter the alignment checks of
// the width dispatch).  The tests assert each form rule of spmm_launch.h on both sides of its
// threshold with it.
extern "C" int ofx_spmm_csr_describe(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                                     int64_t nnz, const void* b, int64_t ldb, const void* c,
                                     int64_t ldc, int64_t row_begin, int64_t row_end,
                                     const ofx_spmm_options* opts, char* buf, size_t buf_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(buf != nullptr && buf_bytes > 0, OFX_EINVAL, "spmm_csr_describe: no buffer");
    buf[0] = 0;
    OFX_READ_OPTIONS(opts, "spmm_csr_describe");
    int rc = check_common(idx_dtype, val_dtype, m, k, n, nnz);
    if (rc) return rc;
    OFX_REQUIRE(0 <= row_begin && row_begin < row_end && row_end <= m && n > 0, OFX_EINVAL,
                "spmm_csr_describe: empty launch (rows [%lld, %lld), n=%lld)", (long long)row_begin,
                (long long)row_end, (long long)n);
    OFX_REQUIRE(ldb >= n && ldc >= n, OFX_EINVAL, "spmm_csr_describe: ldb / ldc < n");
    const int64_t nrows = row_end - row_begin;
    const int64_t nnz_est = launch_nnz(m, nrows, nnz, opts);
    Launch L{nullptr, nullptr, nullptr, nullptr, b, const_cast<void*>(c), ldb, ldc, row_begin, nrows,
             n, nnz, launch_schedule(nrows, nnz_est, n, resolve_schedule(n, opts)), nullptr, 0,
             nullptr, OFX_ACT_NONE, k, nullptr, nnz_est, buf, buf_bytes};
    if (idx_dtype == OFX_DT_INT32) return launch_idx<int32_t>(val_dtype, L);
    return launch_idx<int64_t>(val_dtype, L);
  });
}

extern "C" int ofx_spmm_csr_gathered(void* stream, int idx_dtype, int val_dtype, int64_t m,
                                     int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                     const void* col_idx, const void* values,
                                     const void* values_perm, const void* b, int64_t ldb, void* c,
                                     int64_t ldc, int64_t row_begin, int64_t row_end,
                                     void* workspace, size_t workspace_bytes,
                                     const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(nnz == 0 || values_perm != nullptr, OFX_EINVAL,
                "spmm_csr_gathered: NULL values_perm with nnz=%lld", (long long)nnz);
    return spmm_entry(stream, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, values,
                      values_perm, b, ldb, c, ldc, row_begin, row_end, nullptr, OFX_ACT_NONE,
                      workspace, workspace_bytes, opts);
  });
}

extern "C" int ofx_spmm_csr_plan(void* stream, int idx_dtype, int val_dtype, int64_t m,
                                 int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                 int64_t row_begin, int64_t row_end, void* workspace,
                                 size_t workspace_bytes, const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_TAKE_DEVICE_ERROR("spmm_csr_plan");
    OFX_READ_OPTIONS(opts, "spmm_csr_plan");
    int rc = check_common(idx_dtype, val_dtype, m, k, n, nnz);
    if (rc) return rc;
    OFX_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= m, OFX_EINVAL,
                "spmm_csr_plan: row range [%lld, %lld) outside [0, %lld)", (long long)row_begin,
                (long long)row_end, (long long)m);
    const int64_t nrows = row_end - row_begin;
    if (nrows == 0 || n == 0) return OFX_OK;  // the launch writes nothing either
    const int64_t nnz_est = launch_nnz(m, nrows, nnz, opts);  // as the launch estimates it
    const Schedule s = launch_schedule(nrows, nnz_est, n, resolve_schedule(n, opts));
    if (use_small_form(nrows, nnz_est, n, s)) return OFX_OK;  // the small form needs no plan
    const plan::WsLayout w = plan::ws_layout(nrows, nnz, n, acc_bytes_of(val_dtype), s);
    if (w.total == 0) return OFX_OK;  // identity work list: nothing to plan
    OFX_REQUIRE(row_ptr != nullptr, OFX_EINVAL, "spmm_csr_plan: NULL row_ptr");
    OFX_REQUIRE(workspace != nullptr && workspace_bytes >= w.total, OFX_EWORKSPACE,
                "spmm_csr_plan: workspace of %zu bytes is smaller than the %zu bytes required",
                workspace_bytes, w.total);
    hipStream_t st = static_cast<hipStream_t>(stream);
  #ifdef OFX_DEBUG_BOUNDS
    {  // the planner's allocations (dbg_bounds.h): row_ptr and the workspace
      dbg::HostBounds hb;
      hb.add(row_ptr, (uint64_t)((row_end + 1) * (idx_dtype == OFX_DT_INT32 ? 4 : 8)));
      hb.add(workspace, workspace_bytes);
      OFX_REQUIRE(hb.publish(st, 3ull << 48) == 0, OFX_EDEVICE, "spmm_csr_plan: debug bounds");
    }
  #endif
    plan::WorkList wl{};
    char* ws = static_cast<char*>(workspace);
    if (idx_dtype == OFX_DT_INT32)
      return plan::launch_plan<int32_t>(st, static_cast<const int32_t*>(row_ptr), row_begin, nrows,
                                        nnz_est, s, w, ws, &wl);
    return plan::launch_plan<int64_t>(st, static_cast<const int64_t*>(row_ptr), row_begin, nrows,
                                      nnz_est, s, w, ws, &wl);
  });
}

extern "C" int ofx_spmm_csr_fused(void* stream, int idx_dtype, int val_dtype, int64_t m,
                                  int64_t k, int64_t n, int64_t nnz, const void* row_ptr,
                                  const void* col_idx, const void* values, const void* b,
                                  int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                                  int64_t row_end, const void* bias, int activation,
                                  void* workspace, size_t workspace_bytes,
                                  const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return spmm_entry(stream, idx_dtype, val_dtype, m, k, n, nnz, row_ptr, col_idx, values, nullptr,
                      b, ldb, c, ldc, row_begin, row_end, bias, activation, workspace,
                      workspace_bytes, opts);
  });
}

extern "C" int ofx_csr_validate(void* stream, int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                const void* row_ptr, const void* col_idx, void* flag_dev) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "csr_validate: bad index dtype %d",
                idx_dtype);
    OFX_REQUIRE(row_ptr && flag_dev && (nnz == 0 || col_idx), OFX_EINVAL,
                "csr_validate: NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    OFX_HIP_CHECK(hipMemsetAsync(flag_dev, 0, sizeof(unsigned int), s));
    int64_t work = std::max<int64_t>(m + 1, nnz);
    int64_t grid = std::min<int64_t>((work + 255) / 256, 4096);
    if (grid < 1) grid = 1;
    if (idx_dtype == OFX_DT_INT32)
      hipLaunchKernelGGL(csr_validate_kernel<int32_t>, dim3((unsigned)grid), dim3(256), 0, s,
                         static_cast<const int32_t*>(row_ptr), static_cast<const int32_t*>(col_idx),
                         m, k, nnz, static_cast<unsigned int*>(flag_dev));
    else
      hipLaunchKernelGGL(csr_validate_kernel<int64_t>, dim3((unsigned)grid), dim3(256), 0, s,
                         static_cast<const int64_t*>(row_ptr), static_cast<const int64_t*>(col_idx),
                         m, k, nnz, static_cast<unsigned int*>(flag_dev));
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}

extern "C" int ofx_csr_row_slice(void* stream, int idx_dtype, const void* row_ptr,
                                 int64_t row_begin, int64_t row_end, void* out_row_ptr) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "csr_row_slice: bad index dtype %d",
                idx_dtype);
    OFX_REQUIRE(0 <= row_begin && row_begin <= row_end, OFX_EINVAL,
                "csr_row_slice: bad row range [%lld, %lld)", (long long)row_begin,
                (long long)row_end);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t rows = row_end - row_begin;
    const int64_t grid = (rows + 1 + 255) / 256;
    if (idx_dtype == OFX_DT_INT32)
      hipLaunchKernelGGL(csr_row_slice_kernel<int32_t>, dim3((unsigned)grid), dim3(256), 0, s,
                         static_cast<const int32_t*>(row_ptr), row_begin, rows,
                         static_cast<int32_t*>(out_row_ptr));
    else
      hipLaunchKernelGGL(csr_row_slice_kernel<int64_t>, dim3((unsigned)grid), dim3(256), 0, s,
                         static_cast<const int64_t*>(row_ptr), row_begin, rows,
                         static_cast<int64_t*>(out_row_ptr));
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}

extern "C" int ofx_synth_dense(void* stream, int val_dtype, int64_t r_begin, int64_t r_end,
                               int64_t n, int64_t ld, uint64_t seed, int exact, void* out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(r_begin <= r_end && ld >= n && n >= 0, OFX_EINVAL, "synth_dense: bad shape");
    const int64_t rows = r_end - r_begin;
    if (rows == 0 || n == 0) return OFX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t total = rows * n;
    const int64_t grid = std::min<int64_t>((total + 255) / 256, 65536);
    switch (val_dtype) {
      case OFX_DT_FLOAT:
        hipLaunchKernelGGL(synth_dense_kernel<float>, dim3((unsigned)grid), dim3(256), 0, s, r_begin,
                           rows, n, ld, seed, exact, static_cast<float*>(out));
        break;
      case OFX_DT_DOUBLE:
        hipLaunchKernelGGL(synth_dense_kernel<double>, dim3((unsigned)grid), dim3(256), 0, s,
                           r_begin, rows, n, ld, seed, exact, static_cast<double*>(out));
        break;
      case OFX_DT_BFLOAT16:
        hipLaunchKernelGGL(synth_dense_kernel<bf16>, dim3((unsigned)grid), dim3(256), 0, s, r_begin,
                           rows, n, ld, seed, exact, static_cast<bf16*>(out));
        break;
      case OFX_DT_FLOAT16:
        hipLaunchKernelGGL(synth_dense_kernel<f16>, dim3((unsigned)grid), dim3(256), 0, s, r_begin,
                           rows, n, ld, seed, exact, static_cast<f16*>(out));
        break;
      default: return fail(OFX_EUNSUPPORTED, "synth_dense: unsupported dtype %d", val_dtype);
    }
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}

// ---- OFX_DEBUG_BOUNDS builds (dbg_bounds.h) ----------------------------------------------------
#ifdef OFX_DEBUG_BOUNDS
namespace ofx {
// the first violation of any launch: kHitWords device words, zeroed once
unsigned long long* dbg_hit_words() {
  static unsigned long long* words = nullptr;
  if (words == nullptr) {
    void* p = nullptr;
    if (hipMalloc(&p, dbg::kHitWords * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, dbg::kHitWords * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    words = static_cast<unsigned long long*>(p);
  }
  return words;
}
}  // namespace ofx
#endif

extern "C" int ofx_debug_bounds_read(uint64_t* out, int reset) {
  return ::ofx::guarded(__func__, [&]() -> int {
  #ifdef OFX_DEBUG_BOUNDS
    OFX_REQUIRE(out != nullptr, OFX_EINVAL, "debug_bounds_read: out is NULL");
    unsigned long long* w = dbg_hit_words();
    OFX_REQUIRE(w != nullptr, OFX_EDEVICE, "debug_bounds_read: no hit buffer");
    OFX_HIP_CHECK(hipDeviceSynchronize());
    OFX_HIP_CHECK(hipMemcpy(out, w, dbg::kHitWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) OFX_HIP_CHECK(hipMemset(w, 0, dbg::kHitWords * sizeof(uint64_t)));
    return OFX_OK;
  #else
    (void)out, (void)reset;
    return fail(OFX_EUNSUPPORTED, "debug_bounds_read: a release build (build with OFX_DEBUG_BOUNDS)");
  #endif
  });
}
