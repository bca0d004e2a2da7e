// Probe: are 8-B and 16-B buffer loads and global stores at 2-B-aligned addresses exact on gfx950
// (the shifted 16-bit window for odd bf16 / f16 widths would issue them)?  Every lane loads the 4
// (8) 16-bit elements starting at element e (any e, so every 2-B alignment) of a buffer of known
// values with raw_buffer_load_b64 (b128) and stores them with one 8-B (16-B) store at element e
// of an output; the host compares.  Also times a window load stream at 2-B offsets against the
// same stream 8-B aligned.  Not product code.
// build: hipcc --offload-arch=gfx950 -O3 probes/unaligned_probe.hip -o unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int BYTES>
__global__ void copy_windows(const uint16_t* in, int n_in, uint16_t* out, int shift) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = lane * (BYTES / 2) + shift;  // element index of this lane's window
  if (e + BYTES / 2 > n_in) return;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(in), 0,
                                                              n_in * 2, 0x00020000);
  if constexpr (BYTES == 8) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)e * 2, 0, 0);
    *reinterpret_cast<u32x2*>(out + e) = v;  // 2-B aligned 8-B store
  } else {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)e * 2, 0, 0);
    *reinterpret_cast<u32x4*>(out + e) = v;
  }
}

// a gather stream: every lane loads `iters` windows at rows (pseudo-random) of a table of rows of
// `ld` elements, window at element `col` of the row; sums them so nothing is dead
__global__ void gather_windows(const uint16_t* in, int rows, int ld, int col, int iters,
                               uint32_t* sink) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(in), 0,
                                                              rows * ld * 2, 0x00020000);
  uint32_t acc = 0, h = blockIdx.x * 977u + threadIdx.x * 131u;
  for (int i = 0; i < iters; ++i) {
    h = h * 1664525u + 1013904223u;
    const uint32_t row = (h >> 8) % (uint32_t)rows;
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (row * ld + col) * 2, 0, 0);
    acc += v.x ^ v.y;
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int n = 1 << 20;
  std::vector<uint16_t> h(n);
  for (int i = 0; i < n; ++i) h[i] = (uint16_t)(i * 2654435761u >> 7);
  uint16_t *din, *dout;
  hipMalloc(&din, n * 2);
  hipMalloc(&dout, n * 2 + 64);
  hipMemcpy(din, h.data(), n * 2, hipMemcpyHostToDevice);
  int bad_total = 0;
  for (int bytes : {8, 16})
    for (int shift = 0; shift < 8; ++shift) {
      hipMemset(dout, 0xff, n * 2 + 64);
      const int lanes = n / (bytes / 2);
      if (bytes == 8)
        copy_windows<8><<<(lanes + 255) / 256, 256>>>(din, n, dout, shift);
      else
        copy_windows<16><<<(lanes + 255) / 256, 256>>>(din, n, dout, shift);
      std::vector<uint16_t> o(n);
      hipMemcpy(o.data(), dout, n * 2, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int i = shift; i + bytes / 2 <= n && i < n - bytes; ++i) bad += o[i] != h[i];
      printf("window %2d B at element offset %d (address %% 8 = %d): %d mismatches\n", bytes, shift,
             (shift * 2) % 8, bad);
      bad_total += bad;
    }
  // gather rate: 2-B misaligned windows vs aligned ones (the same rows, ld = 48 / 47 elements)
  uint32_t* sink;
  hipMalloc(&sink, 4 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int rows = 400000;
  uint16_t* table;
  hipMalloc(&table, (size_t)rows * 48 * 2 + 64);
  for (int ld : {48, 47})
    for (int col : {0, 1, 4, 43}) {
      if (col + 4 > ld) continue;
      gather_windows<<<4096, 256>>>(table, rows, ld, col, 64, sink);
      hipEventRecord(a);
      for (int rep = 0; rep < 10; ++rep) gather_windows<<<4096, 256>>>(table, rows, ld, col, 64, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double loads = 4096.0 * 256 * 64 * 10;
      printf("gather ld=%d col=%d (window address %% 8 = %d): %.3f ms, %.2f G windows/s\n", ld, col,
             (col * 2) % 8, ms, loads / (ms * 1e-3) / 1e9);
    }
  printf("%s\n", bad_total ? "UNALIGNED WINDOWS WRONG" : "unaligned windows exact");
  return bad_total ? 1 : 0;
}
