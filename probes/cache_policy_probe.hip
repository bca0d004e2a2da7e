// cache_policy_probe.hip — probe (not product code): does steering B-row loads by column hotness
// through the gfx950 cache-policy bits keep the hot B rows resident in L2 / the Infinity Cache?
//
// The products-shaped gather of spmm_main_kernel (N=128 fp32: a 512-B B row per nonzero, 32 lanes
// x 16 B, eight rows in flight per lane) without rows or hub splitting: every half-wave takes a
// contiguous run of CH nonzeros, so the memory stream is the SpMM's (col stream + B-row gathers in
// nonzero order) with no load imbalance.  The column index carries a tag in bit 31 (set = cold),
// made on the host from the in-degree ranking; hot rows load with cache policy A_HOT, cold ones
// with A_COLD (buffer-load aux bits on gfx950: 1 = sc0, 2 = nt, 16 = sc1).  Each half-wave writes
// its sum so nothing is dead code.  Built by probes/cache_policy_probe.py.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int LPR = 32, U = 8, CH = 512;

template <int A_HOT, int A_COLD, bool BITMAP>
__global__ __launch_bounds__(256) void probe_kernel(const int32_t* __restrict__ col,
                                                    const uint32_t* __restrict__ hot_bits,
                                                    const float* __restrict__ b, int64_t nnz,
                                                    int64_t b_bytes, f4* __restrict__ out) {
  const int lane = threadIdx.x & 63, gl = lane & (LPR - 1), gbase = lane & ~(LPR - 1);
  const int64_t group = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int64_t j0 = group * CH;
  if (j0 >= nnz) return;
  const int64_t j1 = j0 + CH < nnz ? j0 + CH : nnz;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(b), (short)0, (int)(b_bytes > 0x7fffffff ? 0x7fffffff : b_bytes), 0x00020000);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t jb = j0; jb < j1; jb += LPR) {
    const int cnt = (int)(j1 - jb < LPR ? j1 - jb : LPR);
    int32_t mine = gl < cnt ? __builtin_nontemporal_load(col + jb + gl) : 0;
    if (BITMAP) {  // realistic form: untagged col, hotness from a per-column bitmap (L2-resident)
      const uint32_t w = hot_bits[(uint32_t)mine >> 5];
      mine = ((w >> (mine & 31)) & 1u) ? mine : (int32_t)((uint32_t)mine | 0x80000000u);
    }
    for (int k = 0; k < cnt; k += U) {
      f4 bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t c = __shfl(mine, gbase + ((k + u) & (LPR - 1)));
        const uint32_t off = ((uint32_t)c & 0x7fffffffu) * 512u + (uint32_t)gl * 16u;
        if (k + u < cnt) {
          if (c < 0)
            bv[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, A_COLD));
          else
            bv[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, A_HOT));
        } else {
          bv[u] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += bv[u];
    }
  }
  out[group * LPR + gl] = acc;
}

template <int A_HOT, int A_COLD, bool BITMAP>
int run(const int32_t* col, const uint32_t* bits, const float* b, int64_t nnz, int64_t b_bytes,
        void* out, hipStream_t s) {
  const int64_t groups = (nnz + CH - 1) / CH;
  const int64_t blocks = (groups * LPR + 255) / 256;
  hipLaunchKernelGGL((probe_kernel<A_HOT, A_COLD, BITMAP>), dim3((unsigned)blocks), dim3(256), 0, s,
                     col, bits, b, nnz, b_bytes, static_cast<f4*>(out));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

// mode: index into the policy table below; returns nonzero on a bad mode or launch error.
extern "C" int probe_launch(int mode, const int32_t* col, const uint32_t* hot_bits, const float* b,
                            int64_t nnz, int64_t b_bytes, void* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (mode) {
    case 0: return run<0, 0, false>(col, hot_bits, b, nnz, b_bytes, out, s);    // all default
    case 1: return run<2, 2, false>(col, hot_bits, b, nnz, b_bytes, out, s);    // all nt
    case 2: return run<0, 2, false>(col, hot_bits, b, nnz, b_bytes, out, s);    // cold nt
    case 3: return run<0, 16, false>(col, hot_bits, b, nnz, b_bytes, out, s);   // cold sc1
    case 4: return run<0, 18, false>(col, hot_bits, b, nnz, b_bytes, out, s);   // cold nt|sc1
    case 5: return run<0, 1, false>(col, hot_bits, b, nnz, b_bytes, out, s);    // cold sc0
    case 6: return run<0, 3, false>(col, hot_bits, b, nnz, b_bytes, out, s);    // cold sc0|nt
    case 7: return run<0, 17, false>(col, hot_bits, b, nnz, b_bytes, out, s);   // cold sc0|sc1
    case 8: return run<0, 19, false>(col, hot_bits, b, nnz, b_bytes, out, s);   // cold all bits
    case 9: return run<0, 2, true>(col, hot_bits, b, nnz, b_bytes, out, s);     // bitmap, cold nt
    case 10: return run<16, 2, false>(col, hot_bits, b, nnz, b_bytes, out, s);  // hot sc1, cold nt
    default: return 2;
  }
}

// ---- the per-launch hint pass: sampled in-degree -> count histogram -> top-T bitmap -------------
// Every SB-th run of 256 consecutive nonzeros is counted (u32 counters, saturating near 255 by a
// plain read before the atomic, so hub columns stop adding); a block-local LDS histogram of the
// clamped counts is merged into 256 global bins; every block of the bitmap pass derives the same
// threshold t* (the smallest count whose suffix of columns fits in T, at least 1) from the bins.
namespace {
constexpr int kHB = 256;

__global__ __launch_bounds__(kHB) void hint_count_kernel(const int32_t* __restrict__ col,
                                                         int64_t nnz, int64_t sb,
                                                         uint32_t* __restrict__ cnt) {
  const int64_t run = (int64_t)blockIdx.x * sb;  // run index (256 nonzeros per run)
  const int64_t j = run * kHB + threadIdx.x;
  if (j >= nnz) return;
  const int32_t c = __builtin_nontemporal_load(col + j);
  if (__builtin_nontemporal_load(cnt + c) < 250u) atomicAdd(cnt + c, 1u);
}

__global__ __launch_bounds__(kHB) void hint_hist_kernel(const uint32_t* __restrict__ cnt,
                                                        int64_t k, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  for (int64_t c = (int64_t)blockIdx.x * kHB + threadIdx.x; c < k; c += (int64_t)gridDim.x * kHB) {
    const uint32_t v = cnt[c];
    atomicAdd(&h[v > 255u ? 255u : v], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(hist + threadIdx.x, h[threadIdx.x]);
}

__global__ __launch_bounds__(kHB) void hint_bits_kernel(const uint32_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ hist, int64_t k,
                                                        int64_t target, uint32_t* __restrict__ bits) {
  __shared__ uint32_t tstar;
  if (threadIdx.x == 0) {  // suffix sums over 256 bins: cheap, identical in every block
    int64_t acc = 0;
    uint32_t t = 256;
    for (int b = 255; b >= 1; --b) {
      acc += hist[b];
      if (acc > target) break;
      t = (uint32_t)b;
    }
    tstar = t;
  }
  __syncthreads();
  const uint32_t t = tstar;
  const int64_t w = (int64_t)blockIdx.x * kHB + threadIdx.x;  // one bitmap word per thread
  if (w * 32 >= k) return;
  uint32_t word = 0;
  for (int i = 0; i < 32; ++i) {
    const int64_t c = w * 32 + i;
    if (c < k && cnt[c] >= t) word |= 1u << i;
  }
  bits[w] = word;
}
}  // namespace

// ws: (k + 256) u32 scratch (counters + histogram), zeroed here; bits: (k + 31) / 32 words.
extern "C" int probe_hints(const int32_t* col, int64_t nnz, int64_t k, int64_t target, int64_t sb,
                           uint32_t* ws, uint32_t* bits, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(ws, 0, (size_t)(k + 256) * 4, s) != hipSuccess) return 1;
  const int64_t runs = (nnz + kHB - 1) / kHB;
  const int64_t grid1 = (runs + sb - 1) / sb;
  hipLaunchKernelGGL(hint_count_kernel, dim3((unsigned)grid1), dim3(kHB), 0, s, col, nnz, sb, ws);
  hipLaunchKernelGGL(hint_hist_kernel, dim3(1024), dim3(kHB), 0, s, ws, k, ws + k);
  const int64_t words = (k + 31) / 32;
  hipLaunchKernelGGL(hint_bits_kernel, dim3((unsigned)((words + kHB - 1) / kHB)), dim3(kHB), 0, s,
                     ws, ws + k, k, target, bits);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
