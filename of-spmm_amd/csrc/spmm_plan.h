// spmm_plan.h — the work-list planner shared by the SpMM forward kernel (spmm_csr.hip) and the
// SDDMM kernel (spmm_backward.hip).  Device code; included by HIP translation units only.
#ifndef OFX_SPMM_PLAN_H_
#define OFX_SPMM_PLAN_H_

#include <hip/hip_runtime.h>

#include <climits>

#include "ofx_internal.h"
#include "spmm_common.h"
#include "dbg_bounds.h"

namespace ofx {
namespace plan {
namespace {  // internal linkage: every HIP translation unit gets its own copy

constexpr int kBlock = 256;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- work planning (three small launches, no contended atomics) ----------------------------
// Every row gets a class: hub (len > split: cut into chunks -> partials + spmm_reduce) or one of
// kBins degree bins (kBins = 2: bin 0 = heavy, len > heavy; bin 1 = the rest; with more bins the
// thresholds step by 4x).  The main kernel walks ONE work list: the hub chunks first, then the
// non-hub rows bin by bin (a stable counting sort by degree), so the longest work starts first
// and the grid ends on short rows.  Two bins measured best on MI355X: the light rows keep index
// order (sequential row_ptr reads and C writes); more bins cost products-scale 1.2% in random
// row_ptr/C traffic.  Rows are taken kPlanRows per block.
//   plan_count  per-block totals of (hubs, hub chunks, rows per bin)
//   plan_scan   one block: exclusive offsets across blocks; counters[0] = hub chunks,
//               counters[1] = hubs, counters[2 + b] = start of bin b in `order`
//   plan_write  hubs[3i..3i+2] = {local row, first chunk slot, chunks},
//               items[2s..2s+1] = {local row, chunk} for s < counters[0],
//               order[...] = local row, bins in order, ascending rows inside a bin.
// The layout is a pure function of row_ptr (deterministic); the partial of chunk s is part[s].
constexpr int kPlanRowsPerThread = 4;
constexpr int64_t kPlanRows = (int64_t)kBlock * kPlanRowsPerThread;
constexpr int kBins = 2;
constexpr int kPlanVals = 2 + kBins;  // hubs, chunks, bins...
constexpr int64_t kOwnItems = 8;      // hubs with more chunks get their items written wave-wide

template <typename I>
__device__ __forceinline__ int plan_row(const I* __restrict__ rp, int64_t row_begin, int64_t nrows,
                                        int64_t g, int64_t split, int64_t chunk, int64_t heavy,
                                        int64_t& nc) {
  nc = 0;
  if (g >= nrows) return -2;  // no row
  const int64_t len = (int64_t)OFX_LDP(rp + (row_begin + g + 1)) -
                      (int64_t)OFX_LDP(rp + (row_begin + g));
  if (len > split) {
    nc = num_chunks(len, chunk);
    return -1;  // hub
  }
  if (heavy == INT64_MAX) return kBins - 1;  // binning off: one bin, identity order
  int64_t t = heavy;
  for (int b = 0; b < kBins - 1; ++b, t >>= 2)
    if (len > t) return b;
  return kBins - 1;
}

// Block-wide exclusive scan of kPlanVals int64 values (256 threads); returns the block totals.
// Each wave scans with cross-lane moves (no barrier), the four wave totals meet in LDS: two
// barriers instead of the sixteen of a shared-memory Hillis-Steele scan.
__device__ __forceinline__ void block_scan_vals(int64_t (&v)[kPlanVals], int64_t (&tot)[kPlanVals]) {
  constexpr int kWaves = kBlock / 64;
  __shared__ int64_t wsum[kPlanVals][kWaves];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t inc[kPlanVals];
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) inc[i] = v[i];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) {
      const int64_t y = (int64_t)__shfl_up((long long)inc[i], off);
      if (lane >= off) inc[i] += y;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) wsum[i][wv] = inc[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) {
    int64_t pre = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const int64_t x = wsum[i][w];
      all += x;
      if (w < wv) pre += x;
    }
    tot[i] = all;
    v[i] = pre + inc[i] - v[i];  // exclusive
  }
  __syncthreads();
}

template <typename I>
__device__ __forceinline__ void plan_thread(const I* __restrict__ rp, int64_t row_begin,
                                            int64_t nrows, int64_t base, int64_t split,
                                            int64_t chunk, int64_t heavy,
                                            int (&cls)[kPlanRowsPerThread],
                                            int64_t (&nc)[kPlanRowsPerThread],
                                            int64_t (&v)[kPlanVals]) {
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) v[i] = 0;
#pragma unroll
  for (int q = 0; q < kPlanRowsPerThread; ++q) {
    cls[q] = plan_row(rp, row_begin, nrows, base + q, split, chunk, heavy, nc[q]);
    if (cls[q] == -1) {
      v[0] += 1;
      v[1] += nc[q];
    } else if (cls[q] >= 0) {
#pragma unroll
      for (int b = 0; b < kBins; ++b) v[2 + b] += (cls[q] == b);
    }
  }
}

template <typename I>
__global__ void __launch_bounds__(kBlock)
    spmm_plan_count_kernel(const I* __restrict__ rp, int64_t row_begin, int64_t nrows,
                           int64_t split, int64_t chunk, int64_t heavy,
                           int64_t* __restrict__ block_tot) {
  int cls[kPlanRowsPerThread];
  int64_t nc[kPlanRowsPerThread], v[kPlanVals], tot[kPlanVals];
  const int64_t base = (int64_t)blockIdx.x * kPlanRows + (int64_t)threadIdx.x * kPlanRowsPerThread;
  plan_thread(rp, row_begin, nrows, base, split, chunk, heavy, cls, nc, v);
  block_scan_vals(v, tot);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i)
      OFX_STP(block_tot + (kPlanVals * blockIdx.x + i), tot[i]);
  }
}

// One block: each thread owns a run of `per` consecutive plan blocks, sums it, one block-wide
// scan of the 256 run totals gives the run offsets, then each thread rewrites its run as
// exclusive offsets.  (A Hillis-Steele block scan per tile of 256 plan blocks took 21 us at
// products scale: ten tiles x eight barrier steps.)
__global__ void __launch_bounds__(kBlock)
    spmm_plan_scan_kernel(int64_t* __restrict__ block_tot, int64_t nblocks,
                          unsigned long long* __restrict__ counters) {
  const int64_t per = (nblocks + kBlock - 1) / kBlock;
  const int64_t b0 = (int64_t)threadIdx.x * per;
  const int64_t b1 = b0 + per < nblocks ? b0 + per : nblocks;
  int64_t v[kPlanVals], tot[kPlanVals];
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) v[i] = 0;
#pragma unroll 8
  for (int64_t b = b0; b < b1; ++b) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) v[i] += OFX_LDP(block_tot + (kPlanVals * b + i));
  }
  block_scan_vals(v, tot);  // v: exclusive offset of this thread's run
#pragma unroll 8
  for (int64_t b = b0; b < b1; ++b) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) {
      const int64_t x = OFX_LDP(block_tot + (kPlanVals * b + i));
      OFX_STP(block_tot + (kPlanVals * b + i), v[i]);
      v[i] += x;
    }
  }
  if (threadIdx.x == 0) {
    OFX_STP(counters + 0, (unsigned long long)tot[1]);
    OFX_STP(counters + 1, (unsigned long long)tot[0]);
    int64_t start = 0;
    for (int b = 0; b < kBins; ++b) {
      OFX_STP(counters + (2 + b), (unsigned long long)start);
      start += tot[2 + b];
    }
  }
}

// Writes one tile's hubs / chunk items / binned order, given this thread's exclusive offsets `v`
// inside the tile, the tile's offsets `off` across tiles and the bins' start positions.
__device__ __forceinline__ void plan_write_rows(const int (&cls)[kPlanRowsPerThread],
                                                const int64_t (&nc)[kPlanRowsPerThread],
                                                const int64_t (&v)[kPlanVals], const int64_t* off,
                                                const unsigned long long* bin_start, int64_t base,
                                                int64_t* __restrict__ hubs,
                                                int64_t* __restrict__ items,
                                                int64_t* __restrict__ order) {
  int64_t hi = off[0] + v[0];
  int64_t slot = off[1] + v[1];
  int64_t pos[kBins];
#pragma unroll
  for (int b = 0; b < kBins; ++b) pos[b] = (int64_t)bin_start[b] + off[2 + b] + v[2 + b];
  int64_t first[kPlanRowsPerThread];
#pragma unroll
  for (int q = 0; q < kPlanRowsPerThread; ++q) {
    const int64_t g = base + q;
    first[q] = slot;
    if (cls[q] == -1) {
      OFX_STP(hubs + (3 * hi + 0), g);
      OFX_STP(hubs + (3 * hi + 1), slot);
      OFX_STP(hubs + (3 * hi + 2), nc[q]);
      if (nc[q] <= kOwnItems) {
        for (int64_t c = 0; c < nc[q]; ++c) {
          OFX_STP(items + (2 * (slot + c) + 0), g);
          OFX_STP(items + (2 * (slot + c) + 1), c);
        }
      }
      ++hi;
      slot += nc[q];
    } else if (cls[q] >= 0) {
#pragma unroll
      for (int b = 0; b < kBins; ++b)
        if (cls[q] == b) OFX_STP(order + (pos[b]++), g);
    }
  }
  // Hubs with many chunks: the whole wave writes their (row, chunk) items, 64 lanes strided
  // (one thread looping over a 900-chunk hub held the Reddit-shaped plan at 38 us).
#pragma unroll
  for (int q = 0; q < kPlanRowsPerThread; ++q) {
    unsigned long long big = __ballot(cls[q] == -1 && nc[q] > kOwnItems);
    while (big) {
      const int src = __ffsll((long long)big) - 1;
      big &= big - 1;
      const int64_t g = (int64_t)__shfl((long long)(base + q), src);
      const int64_t s0 = (int64_t)__shfl((long long)first[q], src);
      const int64_t ncs = (int64_t)__shfl((long long)nc[q], src);
      for (int64_t c = threadIdx.x & 63; c < ncs; c += 64) {
        OFX_STP(items + (2 * (s0 + c) + 0), g);
        OFX_STP(items + (2 * (s0 + c) + 1), c);
      }
    }
  }
}

template <typename I>
__global__ void __launch_bounds__(kBlock)
    spmm_plan_write_kernel(const I* __restrict__ rp, int64_t row_begin, int64_t nrows,
                           int64_t split, int64_t chunk, int64_t heavy,
                           const int64_t* __restrict__ block_off,
                           const unsigned long long* __restrict__ counters,
                           int64_t* __restrict__ hubs, int64_t* __restrict__ items,
                           int64_t* __restrict__ order) {
  int cls[kPlanRowsPerThread];
  int64_t nc[kPlanRowsPerThread], v[kPlanVals], tot[kPlanVals];
  const int64_t base = (int64_t)blockIdx.x * kPlanRows + (int64_t)threadIdx.x * kPlanRowsPerThread;
  plan_thread(rp, row_begin, nrows, base, split, chunk, heavy, cls, nc, v);
  block_scan_vals(v, tot);
  plan_write_rows(cls, nc, v, block_off + kPlanVals * blockIdx.x, counters + 2, base, hubs, items,
                  order);
}

// plan_scan folded into plan_write for launches of at most kFusedPlanBlocks plan blocks (<= 256K
// rows): every write block sums the per-block totals itself (its exclusive offset and the grand
// totals, O(blocks) reads per block), so the planner is two launches instead of three.  Block 0
// publishes the counters.  Same layout as the three-launch form.
constexpr int64_t kFusedPlanBlocks = 256;

template <typename I>
__global__ void __launch_bounds__(kBlock)
    spmm_plan_write_fused_kernel(const I* __restrict__ rp, int64_t row_begin, int64_t nrows,
                                 int64_t split, int64_t chunk, int64_t heavy,
                                 const int64_t* __restrict__ block_tot, int64_t nblocks,
                                 unsigned long long* __restrict__ counters,
                                 int64_t* __restrict__ hubs, int64_t* __restrict__ items,
                                 int64_t* __restrict__ order) {
  __shared__ unsigned long long s_off[kPlanVals], s_tot[kPlanVals], s_bin[kBins];
  // the per-block totals and this block's row_ptr entries are loaded together (one memory
  // round trip, not two)
  int cls[kPlanRowsPerThread];
  int64_t nc[kPlanRowsPerThread], v[kPlanVals], tot[kPlanVals], off[kPlanVals];
  const int64_t base = (int64_t)blockIdx.x * kPlanRows + (int64_t)threadIdx.x * kPlanRowsPerThread;
  int64_t po[kPlanVals] = {}, pt[kPlanVals] = {};
  for (int64_t b = threadIdx.x; b < nblocks; b += kBlock) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) {
      const int64_t x = OFX_LDP(block_tot + (kPlanVals * b + i));
      pt[i] += x;
      if (b < (int64_t)blockIdx.x) po[i] += x;
    }
  }
  plan_thread(rp, row_begin, nrows, base, split, chunk, heavy, cls, nc, v);
  // wave sums of the partial offsets / totals, then one slot per wave (integer sums: any order
  // gives the same value)
  __shared__ int64_t w_off[kPlanVals][kBlock / 64], w_tot[kPlanVals][kBlock / 64];
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      po[i] += (int64_t)__shfl_xor((long long)po[i], m);
      pt[i] += (int64_t)__shfl_xor((long long)pt[i], m);
    }
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) {
      w_off[i][threadIdx.x >> 6] = po[i];
      w_tot[i][threadIdx.x >> 6] = pt[i];
    }
  }
  block_scan_vals(v, tot);  // its barriers also publish the wave slots above
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < kPlanVals; ++i) {
      int64_t a = 0, b = 0;
      for (int w = 0; w < kBlock / 64; ++w) {
        a += w_off[i][w];
        b += w_tot[i][w];
      }
      s_off[i] = (unsigned long long)a;
      s_tot[i] = (unsigned long long)b;
    }
    unsigned long long start = 0;
    for (int b = 0; b < kBins; ++b) {
      s_bin[b] = start;
      start += s_tot[2 + b];
    }
    if (blockIdx.x == 0) {
      OFX_STP(counters + 0, s_tot[1]);
      OFX_STP(counters + 1, s_tot[0]);
      for (int b = 0; b < kBins; ++b) OFX_STP(counters + (2 + b), s_bin[b]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) off[i] = (int64_t)s_off[i];
  plan_write_rows(cls, nc, v, off, s_bin, base, hubs, items, order);
}

struct WsLayout {
  size_t counters, block_tot, hubs, items, order, part, total;
  int64_t max_hubs, max_chunks, plan_blocks;
};

// The plan (and so a workspace) is used when some row can be a hub or fall outside the lightest
// bin; otherwise the work list is the identity and no workspace is needed.
constexpr int64_t kMinBinRows = 16384;  // below this the grid is one wave of blocks: no tail

WsLayout ws_layout(int64_t nrows, int64_t nnz, int64_t n, size_t acc_bytes, const Schedule& s) {
  WsLayout w{};
  const bool bin = s.heavy != INT64_MAX && (nrows >= kMinBinRows || s.force_bin);
  const bool hub = s.split != INT64_MAX && nnz > s.split;
  if (!bin && !hub) return w;  // identity work list: no plan, no workspace
  w.max_hubs = s.split == INT64_MAX ? 0 : nnz / (s.split + 1) + 1;
  w.max_chunks = s.split == INT64_MAX ? 0 : nnz / s.chunk + 1;
  w.plan_blocks = (nrows + kPlanRows - 1) / kPlanRows;
  size_t off = 0;
  w.counters = off;
  off = align_up(off + (2 + kBins) * sizeof(unsigned long long), 256);
  w.block_tot = off;
  off = align_up(off + (size_t)w.plan_blocks * kPlanVals * sizeof(int64_t), 256);
  w.hubs = off;
  off = align_up(off + (size_t)w.max_hubs * 3 * sizeof(int64_t), 256);
  w.items = off;
  off = align_up(off + (size_t)w.max_chunks * 2 * sizeof(int64_t), 256);
  w.order = off;
  off = align_up(off + (size_t)nrows * sizeof(int64_t), 256);
  w.part = off;
  off = align_up(off + (size_t)w.max_chunks * (size_t)n * acc_bytes, 256);
  w.total = off;
  return w;
}

struct WorkList {
  unsigned long long* counters;
  int64_t* hubs;
  int64_t* items;
  int64_t* order;
  void* part;
};

// The work list's pointers inside workspace `ws` laid out as `w` (a plan built earlier).
inline void worklist_of(const WsLayout& w, char* ws, WorkList* wl) {
  wl->counters = reinterpret_cast<unsigned long long*>(ws + w.counters);
  wl->hubs = reinterpret_cast<int64_t*>(ws + w.hubs);
  wl->items = reinterpret_cast<int64_t*>(ws + w.items);
  wl->order = reinterpret_cast<int64_t*>(ws + w.order);
  wl->part = ws + w.part;
}

// Launches plan_count / plan_scan / plan_write on `stream` into workspace `ws` laid out as `w`.
template <typename I>
int launch_plan(hipStream_t stream, const I* rp, int64_t row_begin, int64_t nrows, int64_t nnz,
                const Schedule& sched, const WsLayout& w, char* ws, WorkList* wl) {
  // Heavy-bin threshold: rows above ~5x the mean degree go first (measured: products and the
  // 1M power-law config both peak at 4-6x the mean).  Order only, never numerics.
  const int64_t heavy = sched.heavy == 0 ? auto_heavy(nrows, nnz) : sched.heavy;
  worklist_of(w, ws, wl);
  auto* block_tot = reinterpret_cast<int64_t*>(ws + w.block_tot);
  const unsigned pgrid = (unsigned)w.plan_blocks;
  hipLaunchKernelGGL((spmm_plan_count_kernel<I>), dim3(pgrid), dim3(kBlock), 0, stream, rp,
                     row_begin, nrows, sched.split, sched.chunk, heavy, block_tot);
  OFX_HIP_CHECK(hipGetLastError());
  if (w.plan_blocks <= kFusedPlanBlocks) {
    hipLaunchKernelGGL((spmm_plan_write_fused_kernel<I>), dim3(pgrid), dim3(kBlock), 0, stream, rp,
                       row_begin, nrows, sched.split, sched.chunk, heavy, block_tot,
                       w.plan_blocks, wl->counters, wl->hubs, wl->items, wl->order);
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  }
  hipLaunchKernelGGL(spmm_plan_scan_kernel, dim3(1), dim3(kBlock), 0, stream, block_tot,
                     w.plan_blocks, wl->counters);
  OFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((spmm_plan_write_kernel<I>), dim3(pgrid), dim3(kBlock), 0, stream, rp,
                     row_begin, nrows, sched.split, sched.chunk, heavy, block_tot, wl->counters,
                     wl->hubs, wl->items, wl->order);
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

}  // namespace
}  // namespace plan
}  // namespace ofx

#endif  // OFX_SPMM_PLAN_H_
