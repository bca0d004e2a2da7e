// Micro-probe for DESIGN.md §9 item 6 (small graphs bound by their longest row): one long CSR row
// at N=16, fp32, traversed by
//   (a) a 16-lane group, one column per lane, 32 B-row loads in flight (the shipped small form);
//   (b) a full wave: quarter q loads the B rows of nonzeros 4u+q, the products are formed in
//       parallel and added in nonzero order through cross-lane moves (same bits as (a)).
// Not product code: a standalone timing of the two traversals on one wave.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off probes/long_row_probe.hip -o long_row_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int N = 16;

__global__ void row16(const int* col, const float* val, int len, const float* B, float* C) {
  const int lane = threadIdx.x;
  if (lane >= N) return;
  float acc = 0.f;
  constexpr int U = 32;
  for (int j = 0; j < len; j += U) {
    float b[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int jj = j + u < len ? j + u : len - 1;
      v[u] = val[jj];
      b[u] = B[(size_t)col[jj] * N + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (j + u < len) acc = acc + v[u] * b[u];
  }
  C[lane] = acc;
}

__global__ void row64(const int* col, const float* val, int len, const float* B, float* C) {
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  float acc = 0.f;
  constexpr int U = 32;  // loads in flight per lane: 4 * U nonzeros per batch
  for (int j = 0; j < len; j += 4 * U) {
    float p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int jj = j + 4 * u + q;
      const int js = jj < len ? jj : len - 1;
      const float b = B[(size_t)col[js] * N + c];
      p[u] = val[js] * b;  // the contract's rounded product
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = __shfl(p[u], r * 16 + c);
        if (j + 4 * u + r < len) acc = acc + x;
      }
    }
  }
  if (q == 0) C[c] = acc;
}

int main(int argc, char** argv) {
  const int len = argc > 1 ? atoi(argv[1]) : 5065, K = 20000;
  std::vector<int> col(len);
  std::vector<float> val(len), B((size_t)K * N);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); };
  for (int i = 0; i < len; ++i) { col[i] = rnd() % K; val[i] = (int)(rnd() % 2001 - 1000) / 1024.f; }
  for (auto& x : B) x = (int)(rnd() % 2001 - 1000) / 512.f;
  int* dc; float *dv, *dB, *C1, *C2;
  CK(hipMalloc(&dc, len * 4)); CK(hipMalloc(&dv, len * 4)); CK(hipMalloc(&dB, B.size() * 4));
  CK(hipMalloc(&C1, N * 4)); CK(hipMalloc(&C2, N * 4));
  CK(hipMemcpy(dc, col.data(), len * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, val.data(), len * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float t[2];
  for (int k = 0; k < 2; ++k) {
    auto go = [&]() { if (k == 0) row16<<<1, 64>>>(dc, dv, len, dB, C1); else row64<<<1, 64>>>(dc, dv, len, dB, C2); };
    go(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 200; ++r) go();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t[k], e0, e1));
  }
  float h1[N], h2[N], ref[N];
  CK(hipMemcpy(h1, C1, N * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(h2, C2, N * 4, hipMemcpyDeviceToHost));
  for (int c = 0; c < N; ++c) {
    float a = 0.f;
    for (int i = 0; i < len; ++i) { volatile float p = val[i] * B[(size_t)col[i] * N + c]; a = a + p; }
    ref[c] = a;
  }
  const bool eq1 = !memcmp(h1, ref, sizeof ref), eq2 = !memcmp(h2, ref, sizeof ref);
  printf("{\"len\": %d, \"row16_us\": %.2f, \"row64_us\": %.2f, \"row16_bitexact\": %s, \"row64_bitexact\": %s}\n",
         len, t[0] / 200 * 1e3, t[1] / 200 * 1e3, eq1 ? "true" : "false", eq2 ? "true" : "false");
  return (eq1 && eq2) ? 0 : 1;
}
