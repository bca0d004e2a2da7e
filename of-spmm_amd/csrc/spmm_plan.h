// spmm_plan.h — the work-list planner shared by the SpMM forward kernel (spmm_csr.hip) and the
// SDDMM kernel (spmm_backward.hip).  Device code; included by HIP translation units only.
#ifndef OFX_SPMM_PLAN_H_
#define OFX_SPMM_PLAN_H_

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <climits>

#include "ofx_internal.h"
#include "spmm_common.h"
#include "dbg_bounds.h"

namespace ofx {

// Agent-coherent accesses: relaxed agent-scope atomics (global_load / global_store ... sc1), seen
// across the XCDs' L2s without an L2 write-back or invalidate.  An agent-scope fence is both
// (buffer_wbl2 sc1 + buffer_inv sc1: the whole XCD's L2 written back and its lines dropped, for
// every other wave on it too); the ordering these accesses need comes from s_waitcnt instead.
// tests/test_isa_ordering.py pins this order in the ISA of every hand-off (the planner's status
// words, the in-kernel hub reduce): sc1 payload stores, s_waitcnt vmcnt(0), then the signal; sc1
// loads issued after the consumed signal.  OFX_AB_UNORDERED_HANDOFF (A/B builds only: `make
// asm-ab-handoff`) removes both halves, to show that the test rejects such a build.
template <typename A>
__device__ __forceinline__ A coh_load(const A* p) {
  if (!OFX_DOK(p, sizeof(A))) return A(0);  // OFX_DEBUG_BOUNDS builds only
#ifdef OFX_AB_UNORDERED_HANDOFF
  return *(volatile const A*)p;
#else
  return __hip_atomic_load(const_cast<A*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
template <typename A>
__device__ __forceinline__ void coh_store(A* p, A v) {
  if (!OFX_DOK(p, sizeof(A))) return;
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// This wave's stores have reached their coherence point (gfx9: stores count in vmcnt).
#ifdef OFX_AB_UNORDERED_HANDOFF
__device__ __forceinline__ void wait_stores() { asm volatile("" ::: "memory"); }
#else
__device__ __forceinline__ void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#endif

namespace plan {
namespace {  // internal linkage: every HIP translation unit gets its own copy

constexpr int kBlock = 256;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- work planning (one launch, decoupled look-back) ------------------------------------------
// Every row gets a class: hub (len > split: cut into chunks -> partials + their reduce) or one of
// kBins degree bins (kBins = 2: bin 0 = heavy, len > heavy; bin 1 = light, the rest).  The main
// kernel walks ONE work list: the hub chunks first, then the heavy rows, then the light rows, so
// the longest work starts first and the grid ends on short rows.  Two bins measured best on
// MI355X: the light rows keep index order (sequential row_ptr reads and C writes); more bins cost
// products-scale 1.2% in random row_ptr/C traffic.  Rows are taken 256 * plan_rpt per
// block.  The plan writes
//   hubs[3i..3i+2] = {local row, first chunk slot, chunks}          (i < counters[1])
//   items[2s..2s+1] = {local row, chunk}                            (s < counters[0])
//   order[0 .. nlight) = the light rows, ascending
//   order[nrows - 1 - h] = heavy row h, h < counters[3] (heavy rows fill the array from its end)
//   arrive[first slot of each hub] = 0                              (the in-kernel hub reduce)
// and counters = {hub chunks, hubs, 0, heavy rows, epoch, host tag, ok / fail / poison tags}.  Item q
// of the non-hub rows is order_row(order, nrows, nheavy, q).  The layout is a pure function of
// row_ptr (deterministic); the partial of chunk s is part[s].
//
// One launch (spmm_plan_kernel): every block counts its rows' classes, then finds the offsets of
// its hubs / chunks / heavy rows / light rows among all earlier blocks by decoupled look-back
// (each block publishes its totals, then its inclusive prefix, in a status word tagged with the
// launch's tag: the workspace is never zeroed, and a word from an earlier launch or leftover
// memory carries another tag), and writes its part of the list.
//
// The launch's tag (a host-chosen epoch is frozen into a captured hipGraph, so every
// replay would take the previous replay's status words as its own) mixes a device-side epoch word
// (counters[kEpoch]: read by every block at entry, advanced by the last block once its look-back
// is done, by which time every block has read it) with the host's per-call tag: replays of one
// capture get distinct tags, and so do calls from different processes on one buffer.  The last
// block also records the plan as valid (counters[kOk] = the tag, with the host tag beside it);
// a block whose look-back gives up records the tag as failed (counters[kFail]), refuses the tag a
// replay of the same capture would take next (counters[kPoison]: a block of this launch that had
// not started yet may publish under it), and sets the library's device-error word.  Every
// consumer of the work list (spmm_main, spmm_reduce, SDDMM) checks plan_valid() at entry; for a
// failed, stale or never-built plan the first consumer (spmm_main, SDDMM) fills its whole output
// with one canonical quiet NaN (poison_value, VERDICT r5 item 3: no stale or uninitialised value
// reads as a result) and the rest write nothing; the host reports the error word at its next
// entry (ofx_device_error_check).
//
// Because heavy rows fill the order array from its end and light rows from its start, no block
// needs a grand total.  A block
// waits only on lower-numbered blocks, which are dispatched first (each XCD dispatches its blocks
// in order), so the chain always progresses.  This replaced count + scan + write launches
// (products 11.3 + 9.6 + 14.6 us, arxiv-shaped 4.8 + 5.8 us).
// Rows per planner thread: 4 up to kPlanRptRows rows, 16 above.  Fewer plan blocks shorten the
// look-back (products: 2,392 blocks of 1,024 rows -> 598 of 4,096); more rows per block lengthen
// each block's count-and-write, which a launch of few blocks feels (graph replay, same box,
// profiles/r04i_ab.jsonl, rows per thread 4 / 8 / 16: products 8477 / 8440 / 8413 us, 1M
// power-law N=16 359 / 353 / 352; 20k rows 29.1 / 30.6 / 33.4, 60k x 1.5M 42.7 / 44.3 / 47.5).
constexpr int64_t kPlanRptRows = int64_t(1) << 18;
inline int plan_rpt(int64_t nrows) { return nrows <= kPlanRptRows ? 4 : 16; }
constexpr int kBins = 2;
constexpr int kPlanVals = 2 + kBins;  // hubs, chunks, bins...
constexpr int64_t kOwnItems = 8;      // hubs with more chunks get their items written wave-wide
constexpr int kLookWords = 16;        // per plan block: status, totals[4], inclusive prefix[4]
constexpr int kLookWin = 4;           // windows of 64 predecessors polled per look-back step
constexpr unsigned long long kAgg = 1, kInc = 2;  // status = tag << 2 | state
// counters[]: the list's sizes, then the validity words (above)
constexpr int kEpoch = 4, kHostTag = 5, kOk = 6, kFail = 7, kPoison = 8, kCounterWords = 9;
// Polls of one status word before the look-back gives up (seconds; a wait in a correct launch is
// microseconds): a planner bug or a stalled predecessor then fails the plan loudly (plan_valid,
// the device-error word) instead of hanging the GPU.  Tests lower it (ofx_debug_set); 0 makes
// every block but the first give up without polling.
constexpr int kSpinLimit = 1 << 22;

// The tag of a plan launch from the device epoch word and the host's per-call tag: 62 bits, odd
// (never 0, the "no valid plan" value of counters[kOk]).
__host__ __device__ __forceinline__ unsigned long long plan_tag(unsigned long long epoch,
                                                               unsigned long long host_tag) {
  return (splitmix64(epoch * 0x9e3779b97f4a7c15ull + splitmix64(host_tag)) >> 2) | 1ull;
}

// Whether `counters` describe a plan that completed (every block wrote its part of the list) and
// has not been superseded by a failed or half-built one.  Uniform across the grid.
__device__ __forceinline__ bool plan_valid(const unsigned long long* __restrict__ counters) {
  const unsigned long long e = OFX_LDP(counters + kEpoch), h = OFX_LDP(counters + kHostTag);
  const unsigned long long ok = OFX_LDP(counters + kOk), fl = OFX_LDP(counters + kFail);
  const unsigned long long poison = OFX_LDP(counters + kPoison);
  return ok != 0 && ok == plan_tag(e - 1, h) && fl != ok && poison != ok;
}

// The library's device-error words (host-mapped, ofx_device_error_check reads them): a plain
// system-scope vector store, never an atomic read-modify-write on host memory.
constexpr int kErrPlanFailed = 0, kErrPlanInvalid = 1;
__device__ __forceinline__ void raise_device_error(unsigned* err, int which) {
  if (err != nullptr)
    __hip_atomic_store(err + which, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

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

// Non-hub work item q (heavy rows first, then light rows) of a plan with `nheavy` heavy rows.
__device__ __forceinline__ int64_t order_row(const int64_t* __restrict__ order, int64_t nrows,
                                             int64_t nheavy, int64_t q) {
  return q < nheavy ? OFX_LDP(order + (nrows - 1 - q)) : OFX_LDP(order + (q - nheavy));
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

template <int RPT, typename I>
__device__ __forceinline__ void plan_thread(const I* __restrict__ rp, int64_t row_begin,
                                            int64_t nrows, int64_t base, int64_t split,
                                            int64_t chunk, int64_t heavy,
                                            int (&cls)[RPT], int64_t (&nc)[RPT],
                                            int64_t (&v)[kPlanVals]) {
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) v[i] = 0;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
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

// Writes one block's hubs / chunk items / heavy and light rows, given this thread's exclusive
// offsets `v` inside the block and the block's offsets `off` among all earlier blocks.
template <int RPT>
__device__ __forceinline__ void plan_write_rows(const int (&cls)[RPT], const int64_t (&nc)[RPT],
                                                const int64_t (&v)[kPlanVals], const int64_t* off,
                                                int64_t base, int64_t nrows,
                                                int64_t* __restrict__ hubs,
                                                int64_t* __restrict__ items,
                                                int64_t* __restrict__ order,
                                                unsigned* __restrict__ arrive) {
  int64_t hi = off[0] + v[0];
  int64_t slot = off[1] + v[1];
  int64_t heavy_pos = off[2] + v[2];  // heavy row h goes to order[nrows - 1 - h]
  int64_t light_pos = off[3] + v[3];
  int64_t first[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int64_t g = base + q;
    first[q] = slot;
    if (cls[q] == -1) {
      OFX_STP(hubs + (3 * hi + 0), g);
      OFX_STP(hubs + (3 * hi + 1), slot);
      OFX_STP(hubs + (3 * hi + 2), nc[q]);
      // the hub's arrival count for the in-kernel reduce (indexed by its first chunk slot): zero
      // here, and the last chunk to arrive resets it, so a plan built once stays valid
      if (arrive != nullptr) OFX_STP(arrive + slot, 0u);
      if (nc[q] <= kOwnItems) {
        for (int64_t c = 0; c < nc[q]; ++c) {
          OFX_STP(items + (2 * (slot + c) + 0), g);
          OFX_STP(items + (2 * (slot + c) + 1), c);
        }
      }
      ++hi;
      slot += nc[q];
    } else if (cls[q] == 0 && kBins > 1) {
      OFX_STP(order + (nrows - 1 - heavy_pos++), g);
    } else if (cls[q] >= 0) {
      OFX_STP(order + (light_pos++), g);
    }
  }
  // Hubs with many chunks: the whole wave writes their (row, chunk) items, 64 lanes strided
  // (one thread looping over a 900-chunk hub held the Reddit-shaped plan at 38 us).
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
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

// Status word of plan block b.  The look-back crosses XCDs: every look word is written and read
// agent-coherent (coh_store / coh_load), and a status is published only once this wave's payload
// stores are complete (wait_stores).  Acquire / release atomics here cost an L2 write-back and
// invalidate per access: products' 2,392-block plan took 262 us with them (profiles/r04g_*).
__device__ __forceinline__ unsigned long long look_status(unsigned long long* look, int64_t b) {
  return coh_load(look + b * kLookWords);
}
__device__ __forceinline__ void look_publish(unsigned long long* look, int64_t b,
                                             unsigned long long status) {
  wait_stores();
  coh_store(look + b * kLookWords, status);
}

template <int RPT, typename I>
__global__ void __launch_bounds__(kBlock)
    spmm_plan_kernel(const I* __restrict__ rp, int64_t row_begin, int64_t nrows, int64_t split,
                     int64_t chunk, int64_t heavy, unsigned long long* __restrict__ look,
                     unsigned long long host_tag, int64_t nblocks,
                     unsigned long long* __restrict__ counters, int64_t* __restrict__ hubs,
                     int64_t* __restrict__ items, int64_t* __restrict__ order,
                     unsigned* __restrict__ arrive, int spin_limit, unsigned* err) {
  __shared__ int64_t s_off[kPlanVals];
  __shared__ int s_fail;
  int cls[RPT];
  int64_t nc[RPT], v[kPlanVals], tot[kPlanVals];
  const int64_t b = blockIdx.x;
  const int64_t base = (b * kBlock + (int64_t)threadIdx.x) * RPT;
  // this launch's tag (see the top of the file): wave 0 reads the epoch word before it publishes
  // anything (here, in flight with the row loads below), and the last block advances it only
  // after every block has published
  const unsigned long long dev_epoch = threadIdx.x < 64 ? coh_load(counters + kEpoch) : 0ull;
  plan_thread<RPT>(rp, row_begin, nrows, base, split, chunk, heavy, cls, nc, v);
  block_scan_vals(v, tot);
  if (threadIdx.x < 64) {
    const unsigned long long epoch = plan_tag(dev_epoch, host_tag);
    // Wave 0 publishes this block's totals (block 0: its inclusive prefix at once), then looks
    // back over up to kLookWin windows of 64 predecessors per step, one predecessor per lane and
    // window, every window's status polled in the same round trip: the nearest predecessor
    // holding its inclusive prefix ends the walk, the aggregates of those after it are added.
    // One lane per step (the round-4 first cut) made the chain ~nblocks / 2 memory round trips
    // long: products' 2,392 plan blocks took ~0.7 ms (profiles/r04e_ab.jsonl); 64 lanes cut it
    // 64-fold.  Round 5: one window per step still cost a block b >= 64 two round trips per window
    // (the poll, then the payload) while the inclusive prefixes of its nearest window were not
    // yet out; kLookWin windows at once make that one poll and one payload round trip for every
    // block of a launch of <= 256 plan blocks (every mid-size launch).
    const int lane = threadIdx.x;
    unsigned long long* my = look + b * kLookWords;
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < kPlanVals; ++i) {
        coh_store(my + 1 + i, (unsigned long long)tot[i]);
        if (b == 0) coh_store(my + 1 + kPlanVals + i, (unsigned long long)tot[i]);
      }
      look_publish(look, b, epoch << 2 | (b == 0 ? kInc : kAgg));
    }
    int64_t pre[kPlanVals] = {};
    bool failed = spin_limit == 0 && b > 0;  // test knob: give up without polling
    for (int64_t end = failed ? 0 : b; end > 0; end -= 64 * kLookWin) {
      // window w, lane l: predecessor end - 1 - 64 w - l (window 0, lane 0: the nearest)
      int64_t p[kLookWin];
      unsigned long long st[kLookWin];
#pragma unroll
      for (int w = 0; w < kLookWin; ++w) {
        p[w] = end - 1 - 64 * w - lane;
        st[w] = 0;  // no tag: polled below (lanes past block 0 are never read)
      }
      // every window's status in one round trip; bounded: a predecessor that never publishes
      // cannot hang the launch
      for (int spins = 0;;) {
        bool waiting = false;
#pragma unroll
        for (int w = 0; w < kLookWin; ++w)
          if (p[w] >= 0 && (st[w] >> 2) != epoch) st[w] = look_status(look, p[w]);
#pragma unroll
        for (int w = 0; w < kLookWin; ++w) waiting |= p[w] >= 0 && (st[w] >> 2) != epoch;
        if (!waiting || ++spins >= spin_limit) break;
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("" ::: "memory");  // the payload loads below issue after the statuses returned
      bool missing = false;
#pragma unroll
      for (int w = 0; w < kLookWin; ++w) missing |= p[w] >= 0 && (st[w] >> 2) != epoch;
      if (__ballot(missing)) {
        failed = true;  // no prefix: this block writes nothing and publishes no prefix
        break;
      }
      // the nearest inclusive predecessor: the first window holding one, its lowest lane
      int stop_w = kLookWin, stop = 64;
#pragma unroll
      for (int w = kLookWin - 1; w >= 0; --w) {
        const unsigned long long incs = __ballot(p[w] >= 0 && (st[w] & 3) == kInc);
        if (incs) {
          stop_w = w;
          stop = __ffsll((long long)incs) - 1;
        }
      }
      int64_t x[kPlanVals] = {};
#pragma unroll
      for (int w = 0; w < kLookWin; ++w) {
        const bool take = p[w] >= 0 && (w < stop_w || (w == stop_w && lane <= stop));
        const unsigned long long* pw = look + (p[w] >= 0 ? p[w] : 0) * kLookWords;
        const bool inc = w == stop_w && lane == stop;
#pragma unroll
        for (int i = 0; i < kPlanVals; ++i)
          x[i] += take ? (int64_t)coh_load(pw + (inc ? 1 + kPlanVals + i : 1 + i)) : 0;
      }
#pragma unroll
      for (int w = 1; w < 64; w <<= 1)
#pragma unroll
        for (int i = 0; i < kPlanVals; ++i) x[i] += (int64_t)__shfl_xor((long long)x[i], w, 64);
#pragma unroll
      for (int i = 0; i < kPlanVals; ++i) pre[i] += x[i];
      if (stop_w < kLookWin) break;
    }
    if (lane == 0) {
      s_fail = failed ? 1 : 0;
      if (b > 0 && !failed) {
#pragma unroll
        for (int i = 0; i < kPlanVals; ++i)
          coh_store(my + 1 + kPlanVals + i, (unsigned long long)(pre[i] + tot[i]));
        look_publish(look, b, epoch << 2 | kInc);
      }
#pragma unroll
      for (int i = 0; i < kPlanVals; ++i) s_off[i] = pre[i];
    }
    if (lane == 0 && failed) {
      // Loud failure: the consumers see counters[kFail] == the tag and poison their output, and the
      // host reports the error word at its next entry.  A predecessor that had not published may
      // not even have started; it can read the advanced epoch word and publish under the NEXT
      // launch's tag (a replay of the same capture), so that tag is refused too (kPoison).
      coh_store(counters + kFail, epoch);
      coh_store(counters + kPoison, plan_tag(dev_epoch + 1, host_tag));
      raise_device_error(err, kErrPlanFailed);
    }
    if (lane == 0 && b == nblocks - 1) {  // the last block knows the grand totals
      if (!failed) {
        OFX_STP(counters + 0, (unsigned long long)(pre[1] + tot[1]));
        OFX_STP(counters + 1, (unsigned long long)(pre[0] + tot[0]));
        OFX_STP(counters + 2, 0ull);
        OFX_STP(counters + 3, (unsigned long long)(pre[2] + tot[2]));
        OFX_STP(counters + kHostTag, host_tag);
      }
      OFX_STP(counters + kOk, failed ? 0ull : epoch);
      // a successful look-back means every block has published, so every block has read the
      // epoch word: the next launch on this workspace gets the next tag
      OFX_STP(counters + kEpoch, dev_epoch + 1);
    }
  }
  __syncthreads();
  if (s_fail) return;  // uniform across the block
  int64_t off[kPlanVals];
#pragma unroll
  for (int i = 0; i < kPlanVals; ++i) off[i] = s_off[i];
  plan_write_rows(cls, nc, v, off, base, nrows, hubs, items, order, arrive);
}

struct WsLayout {
  size_t counters, look, hubs, items, order, arrive, part, total;
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
  const int64_t rows_per_block = (int64_t)kBlock * plan_rpt(nrows);
  w.plan_blocks = (nrows + rows_per_block - 1) / rows_per_block;
  // The look region is sized for the smallest rows-per-thread (the most blocks), not this
  // launch's: the size is then monotone in nrows, so the workspace query over the matrix's m
  // bounds every row range of it (m = 2^18 + 1 planned 65 blocks, rows [1, m) 256).
  const int64_t look_blocks = (nrows + (int64_t)kBlock * 4 - 1) / ((int64_t)kBlock * 4);
  size_t off = 0;
  w.counters = off;
  off = align_up(off + kCounterWords * sizeof(unsigned long long), 256);
  w.look = off;
  off = align_up(off + (size_t)look_blocks * kLookWords * sizeof(unsigned long long), 256);
  w.hubs = off;
  off = align_up(off + (size_t)w.max_hubs * 3 * sizeof(int64_t), 256);
  w.items = off;
  off = align_up(off + (size_t)w.max_chunks * 2 * sizeof(int64_t), 256);
  w.order = off;
  off = align_up(off + (size_t)nrows * sizeof(int64_t), 256);
  w.arrive = off;  // per chunk slot (only hubs' first slots are used): the in-kernel reduce
  off = align_up(off + (size_t)w.max_chunks * sizeof(unsigned), 256);
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
  unsigned* arrive;
  void* part;
};

// The work list's pointers inside workspace `ws` laid out as `w` (a plan built earlier).
inline void worklist_of(const WsLayout& w, char* ws, WorkList* wl) {
  wl->counters = reinterpret_cast<unsigned long long*>(ws + w.counters);
  wl->hubs = reinterpret_cast<int64_t*>(ws + w.hubs);
  wl->items = reinterpret_cast<int64_t*>(ws + w.items);
  wl->order = reinterpret_cast<int64_t*>(ws + w.order);
  wl->arrive = reinterpret_cast<unsigned*>(ws + w.arrive);
  wl->part = ws + w.part;
}

// The host's per-call part of a plan's tag (a per-process random start and a counter; the device
// epoch word makes the tag launch-unique within one capture, see the top of the file).  A status
// word left by another launch (or uninitialised memory) matches a tag with probability 2^-62.
inline unsigned long long next_host_tag() {
  static std::atomic<unsigned long long> counter{
      splitmix64((unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count() ^
                 (unsigned long long)(uintptr_t)&counter)};
  return (splitmix64(counter.fetch_add(1)) >> 2) | 1ull;
}

// Launches the planner on `stream` into workspace `ws` laid out as `w`: one kernel.
template <typename I>
int launch_plan(hipStream_t stream, const I* rp, int64_t row_begin, int64_t nrows, int64_t nnz,
                const Schedule& sched, const WsLayout& w, char* ws, WorkList* wl) {
  // Heavy-bin threshold: rows above ~5x the mean degree go first (measured: products and the
  // 1M power-law config both peak at 4-6x the mean).  Order only, never numerics.
  const int64_t heavy = sched.heavy == 0 ? auto_heavy(nrows, nnz) : sched.heavy;
  worklist_of(w, ws, wl);
  auto* look = reinterpret_cast<unsigned long long*>(ws + w.look);
  OFX_REQUIRE(w.plan_blocks < (int64_t)UINT32_MAX, OFX_EINVAL, "spmm_csr: too many rows to plan");
  const unsigned long long host_tag = next_host_tag();
  const int spin = debug_knob(OFX_DEBUG_PLAN_SPIN_LIMIT, kSpinLimit);
  unsigned* err = device_error_words();
  if (plan_rpt(nrows) == 4)
    hipLaunchKernelGGL((spmm_plan_kernel<4, I>), dim3((unsigned)w.plan_blocks), dim3(kBlock), 0,
                       stream, rp, row_begin, nrows, sched.split, sched.chunk, heavy, look, host_tag,
                       w.plan_blocks, wl->counters, wl->hubs, wl->items, wl->order, wl->arrive,
                       spin, err);
  else
    hipLaunchKernelGGL((spmm_plan_kernel<16, I>), dim3((unsigned)w.plan_blocks), dim3(kBlock), 0,
                       stream, rp, row_begin, nrows, sched.split, sched.chunk, heavy, look, host_tag,
                       w.plan_blocks, wl->counters, wl->hubs, wl->items, wl->order, wl->arrive,
                       spin, err);
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

}  // namespace
}  // namespace plan
}  // namespace ofx

#endif  // OFX_SPMM_PLAN_H_
