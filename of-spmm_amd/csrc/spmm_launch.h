// spmm_launch.h — host-side launch descriptor of the SpMM forward and the size rules that the
// workspace query, the planner entry and the launch share (spmm_csr.hip); the kernels and their
// launch templates are in spmm_csr_impl.h, instantiated per (value, index) type in spmm_inst_*.hip.
#ifndef OFX_SPMM_LAUNCH_H_
#define OFX_SPMM_LAUNCH_H_

#include <hip/hip_runtime.h>

#include "spmm_common.h"

namespace ofx {

struct Launch {
  hipStream_t stream;
  const void *rp, *col, *val, *b;
  void* c;
  int64_t ldb, ldc, row_begin, nrows, n, nnz;
  Schedule sched;
  void* ws;
  size_t ws_bytes;
  const void* bias;  // fused epilogue (T[n] or NULL) and OFX_ACT_*
  int act;
  int64_t b_rows;  // k: rows of B (cache-footprint choice of load hints)
  const void* vperm;  // NULL, or I[nnz]: nonzero j's value is val[vperm[j]] (A^T of a gradient)
  int64_t nnz_est;    // this launch's nonzeros, estimated (launch_nnz): the form choice and the
                      // automatic heavy threshold; `nnz` (the matrix's) bounds the workspace
  char* describe = nullptr;  // ofx_spmm_csr_describe: write the configuration here, launch nothing
  size_t describe_bytes = 0;
};

// Nonzeros of a launch over `nrows` of the matrix's `m` rows: nnz * nrows / m.  row_ptr lives on
// the device, so the exact count is not known to the host; a row range of these graphs (rows
// randomly permuted; BalancedSplitter ranges measured within 3% of the mean nnz) holds about its
// share.  The form heuristics use it so that a rank's slice of an S(0) split is treated as the
// launch it is (with the matrix's nnz an 11M-nonzero graph on 8 ranks took the
// single-GPU crossovers at 1.4M local nonzeros).  The workspace bounds keep the matrix's nnz.
// A caller that knows the range's count passes it (options.range_nnz, ADVICE r3: an S(0) slice
// of a degree-sorted or clustered graph can hold far more or fewer than its share).
inline int64_t launch_nnz(int64_t m, int64_t nrows, int64_t nnz, const ofx_spmm_options* o) {
  if (m <= 0 || nrows >= m) return nnz;
  if (o != nullptr && o->range_nnz > 0) return o->range_nnz < nnz ? o->range_nnz : nnz;
  return (int64_t)((__int128)nnz * nrows / m);
}

// Which form a launch takes is a fixed function of (rows, estimated nnz, n, variant), so the
// workspace query, the plan-once entry and the launch agree.  The thresholds are counts, set from
// the round-3 forms sweep over power-law graphs of 89k-124M nonzeros at N = 16-128 (every form
// forced on every graph, same box; profiles/r03b_probe_forms.jsonl, DESIGN.md §3 "Forms"), and a
// GPU test runs each rule on both sides of its threshold.
//
// Small form (spmm_small_kernel): one launch when the launch has at most kSmallRows rows, at most
// kSmallFormNnz nonzeros and at most kSmallFormElems products (nnz * n).  A block adds its long
// rows one after another, so the form pays for a long row with a serial chain; the nonzero cap
// keeps the power-law maximum degree small (PubMed-shaped, 89k nonzeros: 18.7 / 22.6 / 27.8 us at
// N = 16 / 32 / 64 against 24-31 us planned; 20k rows with 400k nonzeros and a 5,065-nonzero row:
// 54 us against 38 us in the mid form).
constexpr int64_t kSmallRows = 32768;
constexpr int64_t kSmallFormNnz = int64_t(1) << 17;
constexpr int64_t kSmallFormElems = int64_t(1) << 23;
constexpr int kSmallLight = 2;  // rows of more than kSmallLight * U nonzeros take the whole block
constexpr int kForceSmallVariant = 30000;  // tuning: the small form at any size (probes only)

inline bool use_small_form(int64_t nrows, int64_t nnz, int64_t n, const Schedule& s) {
  if (s.variant == kForceSmallVariant) return true;
  return s.variant == 0 && nrows <= kSmallRows && nnz <= kSmallFormNnz &&
         nnz <= kSmallFormElems / (n > 0 ? n : 1);
}

// Mid form (spmm_main_kernel with block items): launches of at most kSmallRows rows above the small
// form and at most kMidFormElems products.  Every hub chunk and every row above the heavy threshold
// (the plan's bin 0, at least kBlockItemMin nonzeros) is taken by a whole block (block_accumulate,
// the small form's engine); the other rows keep one lane-group each.  Bits are unchanged: only who
// adds changes.  Few rows means few lane-groups, so a long row summed by one group would hold the
// launch (20k rows, 400k nonzeros: 38-51 us here against 53-91 us with wave items and 88-147 us
// in the bandwidth configuration).  With more rows the block items' LDS (33-41 KB per block, on
// every block of the launch) costs more than it saves (arxiv-shaped, 169k rows: 112 us at N = 16
// against 78 us in the prefetching form).
constexpr int64_t kMidFormElems = int64_t(1) << 28;
constexpr int64_t kBlockItemMin = 64;
constexpr int kForceMidVariant = 30001;       // tuning: mid form at any size, big-launch rows
constexpr int kForceMidSmallVariant = 30002;  // tuning: mid form, small-launch rows (U=32, PF)

inline bool use_mid_form(int64_t nrows, int64_t nnz, int64_t n, const Schedule& s) {
  if (s.variant == kForceMidVariant || s.variant == kForceMidSmallVariant) return true;
  return s.variant == 0 && nrows <= kSmallRows && !use_small_form(nrows, nnz, n, s) &&
         nnz <= kMidFormElems / (n > 0 ? n : 1);
}

// Prefetching form (planned, U = 32 / 16 loads in flight per lane with the next (col, val) batch
// loaded during the current one; above N = 16 hub chunks and heavy rows take a whole wave):
// launches of more rows than the mid form and at most kPrefetchNnz nonzeros.  Such a launch is
// too short for its traffic to hide the chains of its longest items, so more loads in flight per
// chain win; past it, the bandwidth configuration's occupancy wins.  Measured crossover between
// 2M nonzeros (prefetching 73 / 93 / 118 / 160 us at N = 16 / 32 / 64 / 128 against 109 / 172 /
// 165 / 195 us) and 5M (149 / 209 / 274 / 391 us against 118 / 188 / 217 / 353 us).
constexpr int64_t kPrefetchNnz = int64_t(3) << 20;

inline bool use_prefetch_form(int64_t nrows, int64_t nnz, int64_t n, const Schedule& s) {
  return s.variant == 0 && !use_small_form(nrows, nnz, n, s) && !use_mid_form(nrows, nnz, n, s) &&
         nnz <= kPrefetchNnz;
}

constexpr int kForceBigVariant = 30003;   // tuning: the planned big form, bandwidth configuration
constexpr int kForceWaveVariant = 30004;  // tuning: the prefetching form with wave items
constexpr int kForcePrefetchVariant = 30005;  // tuning: the prefetching form without wave items
// tests: the bandwidth configuration with global B loads (the B >= 4 GiB path, whose out-of-range
// columns read g_zero_row) at any size
constexpr int kForceGlobalVariant = 30006;

// Tuning variants that force a form (small / mid / big / wave) but keep the automatic
// configuration.
inline bool is_form_variant(int v) {
  return v == kForceSmallVariant || v == kForceMidVariant || v == kForceMidSmallVariant ||
         v == kForceBigVariant || v == kForceWaveVariant || v == kForcePrefetchVariant ||
         v == kForceGlobalVariant;
}

// The schedule a launch of `nrows` rows runs with: the mid form always plans (binned work list)
// and raises the automatic heavy threshold to kBlockItemMin.  The workspace query, the planner
// entry (ofx_spmm_csr_plan) and the launch all go through this, so a plan built once matches.
inline Schedule launch_schedule(int64_t nrows, int64_t nnz, int64_t n, Schedule s) {
  if (!use_mid_form(nrows, nnz, n, s)) return s;
  s.force_bin = 1;
  if (s.heavy == 0) {
    const int64_t h = auto_heavy(nrows, nnz);
    s.heavy = h > kBlockItemMin ? h : kBlockItemMin;
  }
  return s;
}

// Every (value, index) type pair: spmm_inst_<T>_<I>.hip (explicit instantiations).
template <typename T, typename I>
int launch_typed(const Launch& L);
// The tuning table (variant = 10000 + id): spmm_csr_tuned.hip.
template <typename T, typename I>
int launch_tuned(const Launch& L, int id);

}  // namespace ofx

#endif  // OFX_SPMM_LAUNCH_H_
