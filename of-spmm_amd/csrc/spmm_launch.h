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
};

// Nonzeros of a launch over `nrows` of the matrix's `m` rows: nnz * nrows / m.  row_ptr lives on
// the device, so the exact count is not known to the host; a row range of these graphs (rows
// randomly permuted; BalancedSplitter ranges measured within 3% of the mean nnz) holds about its
// share.  The form heuristics use it so that a rank's slice of an S(0) split is treated as the
// launch it is (with the matrix's nnz an 11M-nonzero graph on 8 ranks took the
// single-GPU crossovers at 1.4M local nonzeros).  The workspace bounds keep the matrix's nnz.
inline int64_t launch_nnz(int64_t m, int64_t nrows, int64_t nnz) {
  if (m <= 0 || nrows >= m) return nnz;
  return (int64_t)((__int128)nnz * nrows / m);
}

// Small form (spmm_small_kernel): one launch when the launch has at most kSmallRows rows and at
// most kSmallFormElems products (nnz * n).  Its longest row then costs at most that many products
// of one block's in-order adds, against the planned form's three planning launches + reduce.
// A fixed function of (rows, nnz, n, variant): the workspace query and the launch agree.
constexpr int64_t kSmallRows = 32768;
constexpr int64_t kSmallFormElems = int64_t(1) << 20;
constexpr int kSmallLight = 2;  // rows of more than kSmallLight * U nonzeros take the whole block
constexpr int kForceSmallVariant = 30000;  // tuning: the small form at any size (probes only)

inline bool use_small_form(int64_t nrows, int64_t nnz, int64_t n, const Schedule& s) {
  if (s.variant == kForceSmallVariant) return true;
  return s.variant == 0 && nrows <= kSmallRows && nnz <= kSmallFormElems / (n > 0 ? n : 1);
}

// Mid form (spmm_main_kernel with block items): launches above the small form and at most
// kMidFormElems products.  Such a launch is short enough that its longest item sets its time:
// a hub chunk or a long row summed by one lane-group is a chain of len / U dependent load rounds
// (arxiv-shaped at N=16: a 7k-nonzero row held the launch at 600 us, profiles/r02j_probe_mid.json).
// In the mid form every hub chunk and every row above the heavy threshold (the plan's bin 0,
// at least kBlockItemMin nonzeros) is taken by a whole block (block_accumulate, the small form's
// engine); the other rows keep one lane-group each.  Bits are unchanged: only who adds changes.
constexpr int64_t kMidFormElems = int64_t(1) << 28;
constexpr int64_t kBlockItemMin = 64;
constexpr int kForceMidVariant = 30001;       // tuning: mid form at any size, big-launch rows
constexpr int kForceMidSmallVariant = 30002;  // tuning: mid form, small-launch rows (U=32, PF)

inline bool use_mid_form(int64_t nrows, int64_t nnz, int64_t n, const Schedule& s) {
  if (s.variant == kForceMidVariant || s.variant == kForceMidSmallVariant) return true;
  return s.variant == 0 && !use_small_form(nrows, nnz, n, s) &&
         nnz <= kMidFormElems / (n > 0 ? n : 1);
}

constexpr int kForceBigVariant = 30003;   // tuning: the planned big form, bandwidth configuration
constexpr int kForceWaveVariant = 30004;  // tuning: the planned form with wave items (U=32, PF)

// Tuning variants that force a form (small / mid / big / wave) but keep the automatic
// configuration.
inline bool is_form_variant(int v) {
  return v == kForceSmallVariant || v == kForceMidVariant || v == kForceMidSmallVariant ||
         v == kForceBigVariant || v == kForceWaveVariant;
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
