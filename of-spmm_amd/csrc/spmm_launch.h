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
};

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

// Every (value, index) type pair: spmm_inst_<T>_<I>.hip (explicit instantiations).
template <typename T, typename I>
int launch_typed(const Launch& L);
// The tuning table (variant = 10000 + id): spmm_csr_tuned.hip.
template <typename T, typename I>
int launch_tuned(const Launch& L, int id);

}  // namespace ofx

#endif  // OFX_SPMM_LAUNCH_H_
