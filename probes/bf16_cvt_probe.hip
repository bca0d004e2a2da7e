// Probe: gfx950's hardware f32 -> bf16 conversion (v_cvt_pk_bf16_f32, emitted for an fptrunc to
// __bf16) against the software round-to-nearest-even of csrc/spmm_common.h (round_bf16), over
// every one of the 2^32 f32 bit patterns.  Prints the mismatch count by class (NaN / other) and
// the first mismatches.  Not product code.
// build: hipcc --offload-arch=gfx950 -O3 -fno-gpu-flush-denormals-to-zero probes/bf16_cvt_probe.hip -o bf16_cvt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ uint32_t sw_round(uint32_t u) {
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u & 0xffff0000u) | 0x400000u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
}

__global__ void probe(unsigned long long* counts, uint32_t* first, uint32_t base) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t u = base + (uint32_t)i;
  float f;
  memcpy(&f, &u, 4);
  const __bf16 h = (__bf16)f;
  uint16_t hb;
  memcpy(&hb, &h, 2);
  const uint32_t hw = (uint32_t)hb << 16;
  const uint32_t sw = sw_round(u);
  if (hw != sw) {
    const bool nan = (u & 0x7fffffffu) > 0x7f800000u;
    const unsigned long long k = atomicAdd(&counts[nan ? 1 : 0], 1ull);
    if (k < 4) {
      first[(nan ? 8 : 0) + 2 * k] = u;
      first[(nan ? 8 : 0) + 2 * k + 1] = hw;
    }
  }
}

int main() {
  unsigned long long* counts;
  uint32_t* first;
  hipMalloc(&counts, 16);
  hipMalloc(&first, 64);
  hipMemset(counts, 0, 16);
  hipMemset(first, 0, 64);
  const uint64_t per = 1ull << 28;
  for (uint64_t b = 0; b < (1ull << 32); b += per)
    hipLaunchKernelGGL(probe, dim3((unsigned)(per / 256)), dim3(256), 0, 0, counts, first, (uint32_t)b);
  hipDeviceSynchronize();
  unsigned long long hc[2];
  uint32_t hf[16];
  hipMemcpy(hc, counts, 16, hipMemcpyDeviceToHost);
  hipMemcpy(hf, first, 64, hipMemcpyDeviceToHost);
  printf("{\"mismatch_non_nan\": %llu, \"mismatch_nan\": %llu, \"first_non_nan\": [", hc[0], hc[1]);
  for (int k = 0; k < 4; ++k) printf("%s[\"0x%08x\", \"0x%08x\"]", k ? ", " : "", hf[2 * k], hf[2 * k + 1]);
  printf("], \"first_nan\": [");
  for (int k = 0; k < 4; ++k) printf("%s[\"0x%08x\", \"0x%08x\"]", k ? ", " : "", hf[8 + 2 * k], hf[8 + 2 * k + 1]);
  printf("]}\n");
  return 0;
}
