// epilogue_grad.hip — backward of the fused epilogue of fused_spmm_csr:
//
//   dx[i, j]  = relu ? (y[i, j] > 0 ? dy[i, j] : 0) : dy[i, j]          relu_grad from the output,
//               oneflow/core/autograd/gradient_funcs/activation.cpp:195-205 (ReluGrad(dy, y))
//   d_bias[j] = sum_i dx[i, j]                                          bias_add grad,
//               oneflow/core/autograd/gradient_funcs/bias_add.cpp:62 (reduce_sum over axis 0)
//
// in one pass over y and dy.  The column sum has a fixed order (OneFlow's reduce_sum leaves it
// to the device reduction; this one is stated so the CPU kernel and the oracle give the same
// bits): rows in chunks of kRows, each chunk summed sequentially from +0 in the accumulation type
// (fp32 for fp32/fp16/bf16, fp64 for fp64); the chunk partials of column j summed in kLanes
// interleaved lanes (lane l takes chunks l, l + kLanes, ... ascending), then the lanes pairwise
// ((l0 + l4) + (l2 + l6)) + ((l1 + l5) + (l3 + l7)); one rounding to T at the end.
//   Kernel 1 (HBM-bound, 2 reads + 1 write per element): a block per (chunk, 256 columns).
//   Kernel 2 (partials only, nchunks x n accumulators): 32 columns x 8 lanes per block.
#include <hip/hip_runtime.h>

#include "ofx_internal.h"
#include "spmm_common.h"

namespace ofx {
namespace {

constexpr int kBlock = 256;
constexpr int64_t kRows = 2048;  // rows per chunk (part of the order contract)
constexpr int kLanes = 8;        // chunk lanes of the final sum (part of the order contract)
constexpr int kCols2 = kBlock / kLanes;

template <typename T>
__global__ void __launch_bounds__(kBlock)
    relu_bias_grad_rows_kernel(int64_t m, int64_t n, const T* __restrict__ y, int64_t ldy,
                               const T* __restrict__ dy, int64_t lddy, T* __restrict__ dx,
                               int64_t lddx, int relu, typename Num<T>::acc* __restrict__ part) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  constexpr int kPre = 16;  // rows in flight per thread (the adds stay in row order)
  const int64_t j = (int64_t)blockIdx.y * kBlock + threadIdx.x;
  if (j >= n) return;
  const int64_t r0 = (int64_t)blockIdx.x * kRows;
  const int64_t r1 = r0 + kRows < m ? r0 + kRows : m;
  A acc = A(0);
  int64_t r = r0;
  for (; r + kPre <= r1; r += kPre) {
    T g[kPre], o[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      g[u] = dy[(r + u) * lddy + j];
      if (relu) o[u] = y[(r + u) * ldy + j];
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const A gv = (relu && !(Num<T>::load(o[u]) > A(0))) ? A(0) : Num<T>::load(g[u]);
      if (dx) dx[(r + u) * lddx + j] = Num<T>::store(gv);
      acc = acc + gv;
    }
  }
  for (; r < r1; ++r) {
    const A gv = (relu && !(Num<T>::load(y[r * ldy + j]) > A(0))) ? A(0) : Num<T>::load(dy[r * lddy + j]);
    if (dx) dx[r * lddx + j] = Num<T>::store(gv);
    acc = acc + gv;
  }
  if (part) part[(int64_t)blockIdx.x * n + j] = acc;
}

template <typename T>
__global__ void __launch_bounds__(kBlock)
    relu_bias_grad_cols_kernel(int64_t nchunks, int64_t n,
                               const typename Num<T>::acc* __restrict__ part, T* __restrict__ d_bias) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  constexpr int kPre = 16;
  __shared__ A sh[kLanes][kCols2];
  const int x = threadIdx.x % kCols2, lane = threadIdx.x / kCols2;
  const int64_t j = (int64_t)blockIdx.x * kCols2 + x;
  A acc = A(0);
  if (j < n) {
    int64_t c = lane;
    for (; c + (int64_t)(kPre - 1) * kLanes < nchunks; c += (int64_t)kPre * kLanes) {
      A v[kPre];
#pragma unroll
      for (int u = 0; u < kPre; ++u) v[u] = part[(c + (int64_t)u * kLanes) * n + j];
#pragma unroll
      for (int u = 0; u < kPre; ++u) acc = acc + v[u];
    }
    for (; c < nchunks; c += kLanes) acc = acc + part[c * n + j];
  }
  sh[lane][x] = acc;
  __syncthreads();
#pragma unroll
  for (int s = kLanes / 2; s >= 1; s >>= 1) {
    if (lane < s) sh[lane][x] = sh[lane][x] + sh[lane + s][x];
    __syncthreads();
  }
  if (lane == 0 && j < n) d_bias[j] = Num<T>::store(sh[0][x]);
}

int64_t nchunks_of(int64_t m) { return (m + kRows - 1) / kRows; }

template <typename T>
int launch(hipStream_t s, int64_t m, int64_t n, const void* y, int64_t ldy, const void* dy,
           int64_t lddy, void* dx, int64_t lddx, void* d_bias, int relu, void* ws) {
  using A = typename Num<T>::acc;
  const int64_t nch = nchunks_of(m);
  A* part = d_bias ? static_cast<A*>(ws) : nullptr;
  if (m > 0) {
    const dim3 grid((unsigned)nch, (unsigned)((n + kBlock - 1) / kBlock));
    hipLaunchKernelGGL((relu_bias_grad_rows_kernel<T>), grid, dim3(kBlock), 0, s, m, n,
                       static_cast<const T*>(y), ldy, static_cast<const T*>(dy), lddy,
                       static_cast<T*>(dx), lddx, relu, part);
    OFX_HIP_CHECK(hipGetLastError());
  }
  if (d_bias) {
    hipLaunchKernelGGL((relu_bias_grad_cols_kernel<T>), dim3((unsigned)((n + kCols2 - 1) / kCols2)),
                       dim3(kBlock), 0, s, nch, n, part, static_cast<T*>(d_bias));
    OFX_HIP_CHECK(hipGetLastError());
  }
  return OFX_OK;
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_relu_bias_grad_workspace_size(int val_dtype, int64_t m, int64_t n,
                                                 size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes != nullptr, OFX_EINVAL, "relu_bias_grad_workspace_size: bytes is NULL");
    OFX_REQUIRE(is_value_dtype(val_dtype), OFX_EUNSUPPORTED, "relu_bias_grad: bad dtype %d",
                val_dtype);
    OFX_REQUIRE(m >= 0 && n >= 0, OFX_EINVAL, "relu_bias_grad: negative size");
    *bytes = (size_t)nchunks_of(m) * (size_t)n * (val_dtype == OFX_DT_DOUBLE ? 8 : 4);
    return OFX_OK;
  });
}

extern "C" int ofx_relu_bias_grad(void* stream, int val_dtype, int64_t m, int64_t n, const void* y,
                                  int64_t ldy, const void* dy, int64_t lddy, void* dx,
                                  int64_t lddx, void* d_bias, int relu, void* workspace,
                                  size_t workspace_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(is_value_dtype(val_dtype), OFX_EUNSUPPORTED, "relu_bias_grad: bad dtype %d",
                val_dtype);
    OFX_REQUIRE(m >= 0 && n >= 0, OFX_EINVAL, "relu_bias_grad: negative size");
    if (n == 0) return OFX_OK;
    OFX_REQUIRE(m == 0 || (dy && (!relu || y) && lddy >= n && (!relu || ldy >= n)), OFX_EINVAL,
                "relu_bias_grad: NULL input or leading dimension < n");
    OFX_REQUIRE(dx == nullptr || lddx >= n, OFX_EINVAL, "relu_bias_grad: lddx < n");
    size_t need = 0;
    ofx_relu_bias_grad_workspace_size(val_dtype, m, n, &need);
    OFX_REQUIRE(d_bias == nullptr || (workspace && workspace_bytes >= need) || need == 0,
                OFX_EWORKSPACE, "relu_bias_grad: workspace of %zu bytes < %zu", workspace_bytes, need);
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (val_dtype) {
      case OFX_DT_FLOAT: return launch<float>(s, m, n, y, ldy, dy, lddy, dx, lddx, d_bias, relu, workspace);
      case OFX_DT_DOUBLE: return launch<double>(s, m, n, y, ldy, dy, lddy, dx, lddx, d_bias, relu, workspace);
      case OFX_DT_BFLOAT16: return launch<bf16>(s, m, n, y, ldy, dy, lddy, dx, lddx, d_bias, relu, workspace);
      default: return launch<f16>(s, m, n, y, ldy, dy, lddy, dx, lddx, d_bias, relu, workspace);
    }
  });
}
