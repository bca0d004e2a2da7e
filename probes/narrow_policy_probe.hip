// narrow_policy_probe.hip — probe (not product code): the products-shaped gather at N=16 fp32
// (64-B B rows, half an L2 line) with every cache-policy combination of gfx950's buffer loads
// (aux bits: 1 = sc0, 2 = nt, 16 = sc1).  The question is whether a scope bit turns the 128-B
// line fill of a 64-B row into a 64-B request (DESIGN.md §3 "Narrow rows": 1.75x over-fetch).
// The mapping is the product's N=16 one (16 lanes x 4 B per row, 16 rows in flight per lane);
// every 16-lane group takes a contiguous run of CH nonzeros.  Built by narrow_policy_probe.py.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int LPR = 16, U = 16, CH = 256;

template <int AUX>
__global__ __launch_bounds__(256) void narrow_kernel(const int32_t* __restrict__ col,
                                                     const float* __restrict__ b, int64_t nnz,
                                                     int64_t b_bytes, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, gl = lane & (LPR - 1), gbase = lane & ~(LPR - 1);
  const int64_t group = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int64_t j0 = group * CH;
  if (j0 >= nnz) return;
  const int64_t j1 = j0 + CH < nnz ? j0 + CH : nnz;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(b), (short)0, (int)(b_bytes > 0x7fffffff ? 0x7fffffff : b_bytes), 0x00020000);
  float acc = 0.f;
  for (int64_t jb = j0; jb < j1; jb += LPR) {
    const int cnt = (int)(j1 - jb < LPR ? j1 - jb : LPR);
    const int32_t mine = gl < cnt ? __builtin_nontemporal_load(col + jb + gl) : 0;
    float bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t c = __shfl(mine, gbase + (u & (LPR - 1)));
      const uint32_t off = (uint32_t)c * 64u + (uint32_t)gl * 4u;
      bv[u] = u < cnt ? __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, AUX) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += bv[u];
  }
  out[group * LPR + gl] = acc;
}

template <int AUX>
int run(const int32_t* col, const float* b, int64_t nnz, int64_t b_bytes, float* out, hipStream_t s) {
  const int64_t groups = (nnz + CH - 1) / CH;
  const int64_t blocks = (groups * LPR + 255) / 256;
  hipLaunchKernelGGL((narrow_kernel<AUX>), dim3((unsigned)blocks), dim3(256), 0, s, col, b, nnz,
                     b_bytes, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

// aux: the cache-policy bits of the B-row loads (0, 1, 2, 3, 16, 17, 18, 19).
extern "C" int narrow_launch(int aux, const int32_t* col, const float* b, int64_t nnz,
                             int64_t b_bytes, float* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (aux) {
    case 0: return run<0>(col, b, nnz, b_bytes, out, s);
    case 1: return run<1>(col, b, nnz, b_bytes, out, s);
    case 2: return run<2>(col, b, nnz, b_bytes, out, s);
    case 3: return run<3>(col, b, nnz, b_bytes, out, s);
    case 16: return run<16>(col, b, nnz, b_bytes, out, s);
    case 17: return run<17>(col, b, nnz, b_bytes, out, s);
    case 18: return run<18>(col, b, nnz, b_bytes, out, s);
    case 19: return run<19>(col, b, nnz, b_bytes, out, s);
    default: return 2;
  }
}
