#ifndef OFX_SPMM_CSR_IMPL_H_
#define OFX_SPMM_CSR_IMPL_H_
// spmm_csr_impl.h — the SpMM forward kernels for CDNA4 (gfx950) and their launch templates;
// included by the per-type instantiation units (spmm_inst_*.hip) and the tuning table
// (spmm_csr_tuned.hip) only, so the heavy template code compiles in parallel.
//
//
// Reference semantics (OneFlow has no SpMM): the composition
//   gather rows B[col[j]]      oneflow/user/kernels/gather_kernel_util.cpp:72-92
//   multiply by val[j]
//   unsorted_segment_sum       oneflow/user/kernels/unsorted_segment_sum_kernel_util.cpp:29-45
// without materialising the nnz x N intermediate and without the CUDA path's atomics
// (unsorted_segment_sum_kernel_util.cu:67), which are non-deterministic.  Width dispatch and
// 64-bit addressing follow the intent of gather_kernel_util.cu:29-107.
//
// Layout on the device: row_ptr I[m+1], col_idx I[nnz], values T[nnz],
// B T[k][ldb] row-major, C T[rows][ldc] row-major.
//
// Kernels:
//   spmm_plan_*  count / scan / write: classify rows (hub = longer than the split threshold,
//                else one of 4 degree bins), lay out the work list: hub chunks first, then the
//                other rows heaviest bin first (stable counting sort; deterministic layout).
//   spmm_main    the dominant launch.  One lane-group (LPR lanes) per work item; each lane owns
//                VEC consecutive columns (16-B loads of B rows); col/val are loaded cooperatively
//                (LPR < 64: coalesced, broadcast by ds_bpermute) or as wave-uniform scalar loads
//                (LPR == 64); U B-row loads are in flight per lane before the in-order
//                multiply-adds.  Hub chunks -> fp32/fp64 partial rows; rows -> C directly.
//                Small launches: hub chunks and heavy rows take a whole wave each, its groups
//                interleaving the nonzeros and adding the products in order (accumulate_wave).
//   spmm_reduce  per hub row: sums its chunk partials in chunk order -> C row.
// Every output element is produced by exactly one lane in a fixed order: results are
// bitwise deterministic and equal to the CPU kernel / oracle with the same schedule.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <type_traits>

#include "ofx_internal.h"
#include "spmm_common.h"
#include "spmm_plan.h"
#include "spmm_launch.h"
#include "dbg_bounds.h"

namespace ofx {
namespace {


using plan::WorkList;
using plan::WsLayout;
using plan::launch_plan;
using plan::ws_layout;

constexpr int kBlock = 256;        // 4 waves
constexpr int64_t kMaxReduceBlocks = 16384;

template <typename T, int VEC>
struct alignas(sizeof(T) * VEC) Pack {
  T v[VEC];
};

// Compile-time kernel configuration: VEC elements per lane, LPR lanes per row-group, U B-row
// loads in flight per lane, WPB waves per block, NT = non-temporal hints on the once-touched
// streams (col_idx, values, C) so they do not displace B rows from L2 / Infinity Cache.
// PF: the next batch's (col, val) pairs are loaded before this batch's B rows, so a long row
// pays one memory round trip per batch instead of two (the small-problem configurations).
// BNT: the B-row loads themselves carry the non-temporal hint (tuning variants only).
// WH: small launches: hub chunks and heavy rows take a whole wave each (the wave's 64/LPR groups
// interleave the nonzeros of one item), the light rows one group each (accumulate_wave).
// BI: the mid form: hub chunks and heavy rows take a whole block each (block_accumulate).
// BUF: B rows through raw buffer loads with the hardware range check (B < 4 GiB, BRows); the
// global-load form (BUF = false) serves larger B in the bandwidth configurations only.
// HL (with WH): the wave items run in HL-lane groups of one element per lane with HU loads in
// flight (WaveMap), not in the light rows' VEC x LPR groups.  Narrow rows then take 4-lane groups
// of 16-B loads (16 light rows per wave at few registers) while a hub chunk still gets a whole
// wave with few cross-lane moves per product: the kernel's register count (the larger of the two
// paths) stays at the light path's.
// SH (bandwidth configurations, fp32): n need not be a multiple of VEC; the lane holding a row's
// last columns takes the VEC-wide window ending at column n - 1 (16-B accesses at 4-B alignment).
// LR: the hubs' chunk partials are added by the last chunk to finish, inside spmm_main (hub_tail),
// instead of by the spmm_reduce launch (the mid-size forms, where a launch is a tenth of the call).
// HV (with HL): elements per lane of the wave items' HL-lane groups (1: one element per lane), so
// that 16-bit rows of 33-64 columns take one pass of 32 lanes; with SH the last window is shifted
// there as in the light rows.
#ifndef OFX_AB_NO_LR
constexpr bool kLR = true;  // the mid-size forms (prefetching, mid, narrow <= kPrefetchNnz): LR
#else
constexpr bool kLR = false;  // A/B builds only (probes/ab_build.sh): the spmm_reduce launch
#endif
template <int VEC_, int LPR_, int U_ = 8, int WPB_ = 4, bool NT_ = false, bool PF_ = false,
          bool BNT_ = false, bool WH_ = false, bool BI_ = false, bool BUF_ = true, int HL_ = 0,
          int HU_ = 16, bool SH_ = false, bool LR_ = false, int HV_ = 1, bool XL_ = false>
struct Cfg {
  static constexpr int VEC = VEC_, LPR = LPR_, U = U_, WPB = WPB_;
  static constexpr bool NT = NT_, PF = PF_, BNT = BNT_, WH = WH_, BI = BI_, BUF = BUF_, SH = SH_;
  static constexpr bool LR = LR_;
  static constexpr int HL = HL_, HU = HU_, HV = HV_;
  // XL (with WH and HL): the wave items' products go through LDS instead of cross-lane moves
  // (accumulate_wave_xl): one group adds them all in nonzero order, so a wave can hold many
  // narrow groups -- many nonzeros per round of B-row loads -- without G x the moves
  static constexpr bool XL = XL_;
  // loads in flight per lane of the wave-item form: G * UW * VEC cross-lane moves per batch are
  // unrolled, so UW keeps that at <= 256 (4..32)
  static constexpr int G = LPR < 64 ? 64 / LPR : 1;
  static constexpr int UW_RAW = 256 / (G * VEC);
  static constexpr int UW = UW_RAW > 32 ? 32 : (UW_RAW < 4 ? 4 : UW_RAW);
};

// The lane mapping of the wave items (accumulate_wave): the light rows' one, or HL lanes of HV
// elements each (HL > 0).
template <typename K>
struct WaveMap {
  static constexpr int VEC = K::HL > 0 ? K::HV : K::VEC;
  static constexpr int LPR = K::HL > 0 ? K::HL : K::LPR;
  static constexpr int UW = K::HL > 0 ? K::HU : K::UW;
  static constexpr bool BNT = K::BNT, BUF = K::BUF;
  // XL: LDS floats per wave for one batch of products (G * UW nonzeros x LPR * VEC columns)
  static constexpr int XL_FLOATS = (64 / LPR) * UW * LPR * VEC;
};

template <typename X>
struct RawOf {
  using type = X;
};
template <>
struct RawOf<bf16> {
  using type = uint16_t;
};
template <>
struct RawOf<f16> {
  using type = uint16_t;
};

template <bool NT, typename X>
__device__ __forceinline__ X ld_stream(const X* p, int line = __builtin_LINE()) {
#ifdef OFX_DEBUG_BOUNDS
  if (!dok(p, sizeof(X), line)) return X{};
#else
  (void)line;
#endif
  if constexpr (NT) {
    using R = typename RawOf<X>::type;
    const R r = __builtin_nontemporal_load(reinterpret_cast<const R*>(p));
    return __builtin_bit_cast(X, r);
  } else {
    return *p;
  }
}

template <int BYTES>
struct RawVec;
template <>
struct RawVec<16> {
  typedef uint32_t type __attribute__((ext_vector_type(4)));
};
template <>
struct RawVec<8> {
  typedef uint32_t type __attribute__((ext_vector_type(2)));
};
template <>
struct RawVec<4> {
  typedef uint32_t type;
};
template <>
struct RawVec<2> {
  typedef uint16_t type;
};

// One B-row slice of a lane (a Pack of VEC elements), optionally with the non-temporal hint.
template <bool BNT, typename P>
__device__ __forceinline__ P ld_brow(const void* p) {
  if constexpr (BNT && (sizeof(P) == 16 || sizeof(P) == 8 || sizeof(P) == 4 || sizeof(P) == 2)) {
    using R = typename RawVec<sizeof(P)>::type;
    return __builtin_bit_cast(P, __builtin_nontemporal_load(reinterpret_cast<const R*>(p)));
  } else {
    return *reinterpret_cast<const P*>(p);
  }
}

__device__ __forceinline__ int32_t shfl(int32_t v, int src) { return __shfl(v, src); }
__device__ __forceinline__ int64_t shfl(int64_t v, int src) {
  return (int64_t)__shfl((long long)v, src);
}
__device__ __forceinline__ float shfl(float v, int src) { return __shfl(v, src); }
__device__ __forceinline__ double shfl(double v, int src) { return __shfl(v, src); }
// Lane `src` (wave-uniform) of v, as a scalar.
__device__ __forceinline__ int32_t readlane(int32_t v, int src) {
  return __builtin_amdgcn_readlane(v, src);
}
__device__ __forceinline__ int64_t readlane(int64_t v, int src) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float readlane(float v, int src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}
__device__ __forceinline__ double readlane(double v, int src) {
  return __builtin_bit_cast(double, readlane(__builtin_bit_cast(int64_t, v), src));
}

// The zero row of out-of-range columns.  The reference gather zero-fills the gathered row of an
// index outside the table (CPU: idx >= size, oneflow/user/kernels/gather_kernel_util.cpp:84-89;
// CUDA: any index outside [0, size), gather_kernel_util.cu:36), so such a nonzero adds val * 0
// (+-0, or NaN for a non-finite value): the bits of loading zeros.  A lane whose column is out of
// range loads a VEC slot of this zero-initialised buffer instead of a B row, so nothing outside B
// is read and no per-element select is needed (one 64-bit address select per nonzero).
constexpr int64_t kZeroRowBytes = 16384;
__device__ __attribute__((aligned(256))) uint32_t g_zero_row[kZeroRowBytes / 4];

// B-row loads of one lane in one column pass (columns [c0, c0 + W); cc = the lane's first column,
// c0 for a lane past n), with the reference gather's zero fill of a column outside [0, k).
//   BUF (B < 4 GiB: every configuration but the papers-scale one): raw buffer loads through one
//   descriptor over B's k rows.  The byte offset of column c is min(c, k) * ldb_bytes + the lane's
//   column bytes; row k lies past the descriptor's range, and the hardware returns zeros for it.
//   So an out-of-range column costs nothing beyond one clamp (v_min_u32 for int32 indices), and
//   the address is 32-bit arithmetic instead of a 64-bit multiply-add per load.
//   !BUF: global loads; an out-of-range column loads this lane's slot of g_zero_row instead (a
//   64-bit select per load).
template <typename T, bool BUF>
struct BRows {
  const T* base;  // !BUF: B + cc
  const T* zero;  // !BUF: this lane's slot of g_zero_row
  int64_t ldb, k;
  __amdgpu_buffer_rsrc_t rsrc;  // BUF: B[0 .. k) rows
  uint32_t ldb_bytes, cc_bytes, k32;
  template <typename I>
  __device__ __forceinline__ uint32_t clamp_row(I c) const {
#ifdef OFX_AB_NO_ZERO_FILL  // A/B builds only (probes/ab_build.sh): no bound
    return (uint32_t)c;
#else
    if constexpr (sizeof(I) == 4) return __builtin_elementwise_min((uint32_t)c, k32);
    else return (uint64_t)c < (uint64_t)k ? (uint32_t)c : k32;
#endif
  }
  __device__ __forceinline__ const T* row(int64_t c) const {
    return (uint64_t)c < (uint64_t)k ? base + c * ldb : zero;
  }
  template <bool NTB, typename P, typename I>
  __device__ __forceinline__ P load(I c) const {
    if constexpr (BUF) {
      const uint32_t off = clamp_row(c) * ldb_bytes + cc_bytes;
      constexpr int aux = NTB ? 2 : 0;  // nt
      if constexpr (sizeof(P) == 16) {
        return __builtin_bit_cast(P, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, aux));
      } else if constexpr (sizeof(P) == 8) {
        return __builtin_bit_cast(P, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, aux));
      } else if constexpr (sizeof(P) == 4) {
        return __builtin_bit_cast(P, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, aux));
      } else if constexpr (sizeof(P) == 32) {
        // two 16-B halves (8-element fp32 lanes); row k (past the range) reads zeros for both
        typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
        const auto lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, aux);
        const auto hi = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16u, 0, aux);
        const u32x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(P, v);
      } else {
        static_assert(sizeof(P) == 2, "B-row slice of 2, 4, 8, 16 or 32 bytes");
        return __builtin_bit_cast(P, __builtin_amdgcn_raw_buffer_load_b16(rsrc, off, 0, aux));
      }
    } else {
      const T* q = row((int64_t)c);
      if (!OFX_DOK(q, sizeof(P))) return P{};  // OFX_DEBUG_BOUNDS builds only
      return ld_brow<NTB, P>(q);
    }
  }
};
template <typename T, bool BUF>
__device__ __forceinline__ BRows<T, BUF> brows(const T* B, int64_t c0, int64_t cc, bool active,
                                               int64_t ldb, int64_t k) {
  BRows<T, BUF> r;
  const int64_t lc = active ? cc : c0;
  r.base = B + lc;
  r.zero = reinterpret_cast<const T*>(g_zero_row) + (lc - c0);
  r.ldb = ldb;
  r.k = k;
  if constexpr (BUF) {
    // the launch guarantees (k + 1) * ldb * sizeof(T) < 2^32; all descriptor inputs are kernel
    // arguments (wave-uniform), so no waterfall loop is emitted around the loads
    r.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(B), 0,
                                               (int)(uint32_t)(k * ldb * (int64_t)sizeof(T)),
                                               0x00020000);
    r.ldb_bytes = (uint32_t)(ldb * (int64_t)sizeof(T));
    r.cc_bytes = (uint32_t)(lc * (int64_t)sizeof(T));
    r.k32 = (uint32_t)k;
  }
  return r;
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// acc[e] += val[j] * B[col[j], cc + e] for j in [j0, j1), in ascending j, mul then add.
// Bc = B + cc.  All lanes of a group call this with the same j0/j1.
template <typename T, typename I, typename K>
__device__ __forceinline__ void accumulate(const I* __restrict__ col, const T* __restrict__ val,
                                           const I* __restrict__ vperm,
                                           const BRows<T, K::BUF>& br, int64_t j0, int64_t j1,
                                           int gl, int gbase, bool active,
                                           typename Num<T>::acc (&acc)[K::VEC]) {
#pragma clang fp contract(off)
  constexpr int VEC = K::VEC, LPR = K::LPR, kUnroll = K::U;
  using A = typename Num<T>::acc;
  using P = Pack<T, VEC>;
  if constexpr (LPR == 64) {
#if !defined(OFX_AB_LPR64_SCALAR)
    // j0/j1 are wave-uniform.  Batches of 64 nonzeros: the (col, val) pairs are loaded coalesced,
    // one per lane, the next batch's during this one; each nonzero's pair reaches the wave as
    // scalars through v_readlane (no LDS), and U B rows are in flight per lane, issued branch-free
    // where B is one buffer (slots past the row end load row k: zeros from the range check, no
    // memory access).  The scalar-cache form this replaces (s_load of each col / val) paid two
    // dependent round trips per U nonzeros (OFX_AB_LPR64_SCALAR keeps it for A/B builds).
    auto load_batch = [&](int64_t jb, I& c, A& v) {
      const int n_ = (int)((j1 - jb) < 64 ? (j1 - jb) : 64);
      c = 0;
      v = A(0);
      if (gl < n_) {
        c = ld_stream<K::NT>(col + jb + gl);
        const int64_t jv = vperm ? (int64_t)ld_stream<K::NT>(vperm + jb + gl) : jb + gl;
        v = Num<T>::load(ld_stream<K::NT>(val + jv));
      }
    };
    I nxc;
    A nxv;
    if (j0 < j1) load_batch(j0, nxc, nxv);
    for (int64_t jb = j0; jb < j1; jb += 64) {
      const int cnt = (int)((j1 - jb) < 64 ? (j1 - jb) : 64);
      const I myc = nxc;
      const A myv = nxv;
      if (jb + 64 < j1) load_batch(jb + 64, nxc, nxv);  // in flight during this batch
      for (int k = 0; k < cnt; k += kUnroll) {
        P bv[kUnroll];
        A vv[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const int s = k + u;  // wave-uniform, < 64
          const I cu = readlane(myc, s);
          vv[u] = readlane(myv, s);
          if constexpr (K::BUF) {
            bv[u] = br.template load<K::BNT, P>(s < cnt && active ? cu : (I)br.k32);
          } else {
            if (s < cnt && active) bv[u] = br.template load<K::BNT, P>(cu);
          }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          if (k + u < cnt && active) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + Num<T>::mul(vv[u], Num<T>::load(bv[u].v[e]));
          }
        }
      }
    }
#else
    // j0/j1 are wave-uniform: col/val come through the scalar cache.
    for (int64_t j = j0; j < j1; j += kUnroll) {
      const int cnt = (int)((j1 - j) < kUnroll ? (j1 - j) : kUnroll);
      P bv[kUnroll];
      A vv[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (u < cnt) {
          const int64_t cu = (int64_t)ld_stream<K::NT>(col + j + u);
          const int64_t jv = vperm ? (int64_t)ld_stream<K::NT>(vperm + j + u) : j + u;
          vv[u] = Num<T>::load(ld_stream<K::NT>(val + jv));
          if (active) bv[u] = br.template load<K::BNT, P>(cu);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (u < cnt && active) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + Num<T>::mul(vv[u], Num<T>::load(bv[u].v[e]));
        }
      }
    }
#endif
  } else {
    // A batch is R * LPR nonzeros: each lane loads R (col, val) pairs coalesced, the group
    // broadcasts them with ds_bpermute.  R > 1 only when more B-row loads are kept in flight
    // than there are lanes in the group (kUnroll > LPR: the small-problem configurations).
    constexpr int R = kUnroll > LPR ? kUnroll / LPR : 1;
    constexpr int BATCH = LPR * R;
    auto load_batch = [&](int64_t jb, I (&c)[R], A (&v)[R]) {
      const int n_ = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c[r] = 0;  // slots past the row end: row 0 (the zero row if k == 0), discarded
        v[r] = 0;
        const int idx = r * LPR + gl;
        if (idx < n_) {
          c[r] = ld_stream<K::NT>(col + jb + idx);
          const int64_t jv = vperm ? (int64_t)ld_stream<K::NT>(vperm + jb + idx) : jb + idx;
          v[r] = Num<T>::load(ld_stream<K::NT>(val + jv));
        }
      }
    };
    I nxc[R];
    A nxv[R];
    if constexpr (K::PF) {
      if (j0 < j1) load_batch(j0, nxc, nxv);
    }
    for (int64_t jb = j0; jb < j1; jb += BATCH) {
      const int cnt = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
      I myc[R];
      A myv[R];
      if constexpr (K::PF) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          myc[r] = nxc[r];
          myv[r] = nxv[r];
        }
        if (jb + BATCH < j1) load_batch(jb + BATCH, nxc, nxv);  // in flight during this batch
      } else {
        load_batch(jb, myc, myv);
      }
      for (int k = 0; k < cnt; k += kUnroll) {
        P bv[kUnroll];
        A vv[kUnroll];
        if constexpr (K::PF) {
          // Branch-free issue for the latency-bound small launches: every broadcast first, then
          // every load (slots past the row end read B row 0, inactive lanes read from B's first
          // columns; both discarded below), so the group pays one LDS wait and one memory round
          // trip per batch instead of one ds_bpermute wait per load.
          I cuv[kUnroll];
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) {
            const int src = gbase + ((k + u) & (LPR - 1));
            const int r = R > 1 ? u / LPR : 0;
            cuv[u] = shfl(myc[r], src);
            vv[u] = shfl(myv[r], src);
          }
#pragma unroll
          for (int u = 0; u < kUnroll; ++u)
            bv[u] = br.template load<K::BNT, P>(k + u < cnt ? cuv[u] : I(0));
        } else {
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) {
            // R > 1: the batch is exactly kUnroll long, so k == 0 and the register is static
            const int src = gbase + ((k + u) & (LPR - 1));
            const int r = R > 1 ? u / LPR : 0;
            const I cu = shfl(myc[r], src);
            vv[u] = shfl(myv[r], src);
            if constexpr (K::BUF) {
              // branch-free issue: a slot past the row end (or a lane past n) loads row k, which
              // lies outside the buffer, so the range check returns zeros with no memory access.
              // Loads under per-slot branches made hipcc wait vmcnt(0) before each bf16 / f16
              // load (one B row in flight per lane instead of U)
              bv[u] = br.template load<K::BNT, P>(k + u < cnt && active ? cu : (I)br.k32);
            } else {
              if (k + u < cnt && active) bv[u] = br.template load<K::BNT, P>(cu);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          if (k + u < cnt && active) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + Num<T>::mul(vv[u], Num<T>::load(bv[u].v[e]));
          }
        }
      }
    }
  }
}

// One work item for the whole wave (LPR < 64): group q = lane / LPR of the G = 64 / LPR groups
// loads the B rows of nonzeros jb + G*u + q of each batch of G*U, forms their products in
// parallel (U loads in flight per lane, the batch's (col, val) prefetched during the previous
// one), then every group adds all G*U products in nonzero order, taking the other groups'
// products through ds_bpermute.  The order (and each product's rounding) is the contract's, so
// the bits equal the one-group traversal; a long row needs G times fewer dependent load rounds.
template <typename T, typename I, typename K>
__device__ __forceinline__ void accumulate_wave(const I* __restrict__ col, const T* __restrict__ val,
                                                const I* __restrict__ vperm,
                                                const BRows<T, K::BUF>& br,
                                                int64_t j0, int64_t j1, int lane, int gl,
                                                typename Num<T>::acc (&acc)[K::VEC]) {
#pragma clang fp contract(off)
  constexpr int VEC = K::VEC, LPR = K::LPR, U = K::UW, G = 64 / LPR;
  constexpr int BATCH = G * U;
  constexpr int R = (BATCH + 63) / 64;  // (col, val) registers per lane for one batch
  static_assert(LPR < 64, "accumulate_wave needs several groups per wave");
  using A = typename Num<T>::acc;
  using P = Pack<T, VEC>;
  const int q = lane / LPR;
  auto load_batch = [&](int64_t jb, I (&c)[R], A (&v)[R]) {
    const int n_ = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      c[r] = 0;
      v[r] = 0;
      const int idx = r * 64 + lane;
      if (idx < n_) {
        c[r] = OFX_LD(col + (jb + idx));
        const int64_t jv = vperm ? (int64_t)OFX_LD(vperm + (jb + idx)) : jb + idx;
        v[r] = Num<T>::load(OFX_LD(val + jv));
      }
    }
  };
  I nxc[R];
  A nxv[R];
  if (j0 < j1) load_batch(j0, nxc, nxv);
  for (int64_t jb = j0; jb < j1; jb += BATCH) {
    const int cnt = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
    I myc[R];
    A myv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      myc[r] = nxc[r];
      myv[r] = nxv[r];
    }
    if (jb + BATCH < j1) load_batch(jb + BATCH, nxc, nxv);  // in flight during this batch
    // this group's nonzeros of the batch: i = G*u + q, held by lane i % 64 in register i / 64
    // G divides 64, so nonzero G*u + q sits in register (G*u) / 64 for every group q
    I cuv[U];
    A vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = G * u + q;
      cuv[u] = shfl(myc[(G * u) >> 6], i & 63);
      vv[u] = shfl(myv[(G * u) >> 6], i & 63);
    }
    P bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      bv[u] = br.template load<K::BNT, P>(G * u + q < cnt ? cuv[u] : I(0));
    // per u: this group's product, the G groups' products fetched with ds_bpermute (all issued
    // before the first add, so their latency overlaps), then added in nonzero order
#pragma unroll
    for (int u = 0; u < U; ++u) {
      A pr[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) pr[e] = Num<T>::mul(vv[u], Num<T>::load(bv[u].v[e]));
      A x[G][VEC];
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2)
#pragma unroll
        for (int e = 0; e < VEC; ++e) x[g2][e] = shfl(pr[e], g2 * LPR + gl);
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2)
        if (G * u + g2 < cnt)
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + x[g2][e];
    }
  }
}

// The wave items with the products exchanged through LDS (Cfg::XL): the same batches as
// accumulate_wave (group q of G loads the B rows of nonzeros G*u + q, u < U), but each lane writes
// its products to the wave's LDS region, nonzero-major, and group 0 alone adds the batch's
// products in nonzero order: the contract's order and roundings, without the G x VEC cross-lane
// moves per nonzero that make narrow groups expensive in accumulate_wave.  Only group 0's
// accumulators hold the sum (the callers store and reduce from lanes < LPR).  The LDS region is
// reused batch to batch: a wave's LDS operations complete in order, so the next batch's writes
// cannot overtake this batch's reads.
template <typename T, typename I, typename K>
__device__ __forceinline__ void accumulate_wave_xl(const I* __restrict__ col, const T* __restrict__ val,
                                                   const I* __restrict__ vperm,
                                                   const BRows<T, K::BUF>& br, int64_t j0, int64_t j1,
                                                   int lane, int gl, typename Num<T>::acc* lds,
                                                   typename Num<T>::acc (&acc)[K::VEC]) {
#pragma clang fp contract(off)
  constexpr int VEC = K::VEC, LPR = K::LPR, U = K::UW, G = 64 / LPR;
  constexpr int BATCH = G * U;
  constexpr int R = (BATCH + 63) / 64;
  constexpr int W = LPR * VEC;  // floats per nonzero in LDS
  static_assert(LPR < 64, "accumulate_wave_xl needs several groups per wave");
  using A = typename Num<T>::acc;
  using P = Pack<T, VEC>;
  const int q = lane / LPR;
  auto load_batch = [&](int64_t jb, I (&c)[R], A (&v)[R]) {
    const int n_ = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      c[r] = 0;
      v[r] = 0;
      const int idx = r * 64 + lane;
      if (idx < n_) {
        c[r] = OFX_LD(col + (jb + idx));
        const int64_t jv = vperm ? (int64_t)OFX_LD(vperm + (jb + idx)) : jb + idx;
        v[r] = Num<T>::load(OFX_LD(val + jv));
      }
    }
  };
  I nxc[R];
  A nxv[R];
  if (j0 < j1) load_batch(j0, nxc, nxv);
  for (int64_t jb = j0; jb < j1; jb += BATCH) {
    const int cnt = (int)((j1 - jb) < BATCH ? (j1 - jb) : BATCH);
    I myc[R];
    A myv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      myc[r] = nxc[r];
      myv[r] = nxv[r];
    }
    if (jb + BATCH < j1) load_batch(jb + BATCH, nxc, nxv);  // in flight during this batch
    I cuv[U];
    A vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = G * u + q;
      cuv[u] = shfl(myc[(G * u) >> 6], i & 63);
      vv[u] = shfl(myv[(G * u) >> 6], i & 63);
    }
    P bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      bv[u] = br.template load<K::BNT, P>(G * u + q < cnt ? cuv[u] : I(0));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = G * u + q;
      if (i < cnt) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) lds[i * W + gl * VEC + e] = Num<T>::mul(vv[u], Num<T>::load(bv[u].v[e]));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (q == 0) {
#pragma unroll 8
      for (int i = 0; i < cnt; ++i)
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + lds[i * W + gl * VEC + e];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename T, int VEC, bool NT>
__device__ __forceinline__ void store_row(T* __restrict__ p, const typename Num<T>::acc (&acc)[VEC],
                                          const T* __restrict__ bias, int act) {
  if (!OFX_DOK(p, sizeof(Pack<T, VEC>)) || (bias && !OFX_DOK(bias, sizeof(T) * VEC))) return;  // debug
  Pack<T, VEC> o;
  if (bias == nullptr && act == OFX_ACT_NONE) {  // uniform: the plain op pays one branch
#pragma unroll
    for (int e = 0; e < VEC; ++e) o.v[e] = Num<T>::store(acc[e]);
  } else {
#pragma unroll
    for (int e = 0; e < VEC; ++e) o.v[e] = epilogue<T>(acc[e], bias, e, act);
  }
  if constexpr (NT && (sizeof(o) == 16 || sizeof(o) == 8 || sizeof(o) == 4 || sizeof(o) == 2)) {
    using R = typename RawVec<sizeof(o)>::type;
    __builtin_nontemporal_store(__builtin_bit_cast(R, o), reinterpret_cast<R*>(p));
  } else {
    *reinterpret_cast<Pack<T, VEC>*>(p) = o;
  }
}

// COH (Cfg::LR): the partial is read back by another work item in the same launch (hub_tail)
template <typename A, int VEC, bool COH = false>
__device__ __forceinline__ void store_partial(A* __restrict__ p, const A (&acc)[VEC]) {
  if constexpr (COH) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) coh_store(p + e, acc[e]);
  } else {
    if (!OFX_DOK(p, sizeof(A) * VEC)) return;  // OFX_DEBUG_BOUNDS builds only
#pragma unroll
    for (int e = 0; e < VEC; ++e) p[e] = acc[e];
  }
}

// In-kernel hub reduce (Cfg::LR).  A chunk item, once its partial row is stored, counts itself in
// at its hub's arrival counter (indexed by the hub's first chunk slot, zeroed by the plan); the last
// of the hub's nc chunks to arrive adds the hub's partial rows in chunk order from +0 and writes the
// C row (epilogue included): the bits of spmm_reduce_kernel, without its launch.  It then resets
// the counter, so a plan built once stays valid for the next launch.  Every lane of the calling
// group calls this after its column passes; `member` lanes hold columns (VEC x L lanes, the
// caller's mapping; SH: the last window shifted to end at column n - 1), `lead_lane` is the group's
// lane 0.  The chunks of one hub run on any XCD: partials are stored, counted and read back
// agent-coherent (store_partial<COH>, coh_load), ordered by waiting for the stores before the count
// (no agent-scope fence: round 4's first cut had two per chunk item, measured +8 us on a 2M-nonzero
// N=16 launch, profiles/r04g_ab.jsonl).
template <typename T, int VEC, int L, bool SH>
__device__ __forceinline__ void hub_tail(unsigned* __restrict__ arrive, int64_t slot0, int64_t nc,
                                         const typename Num<T>::acc* __restrict__ part,
                                         T* __restrict__ C, int64_t ldc, int64_t lr, int64_t n,
                                         int gl, bool member, int lead_lane,
                                         const T* __restrict__ bias, int act) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  wait_stores();  // this group's partial row is at the coherence point before it is counted
  unsigned old = 0;
  if (member && gl == 0)
    old = __hip_atomic_fetch_add(arrive + slot0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, lead_lane);  // waits for the count: the loads below issue after it
  if ((int64_t)old != nc - 1) return;
  if (!member) return;
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)L * VEC) {
    int64_t cc = c0 + (int64_t)gl * VEC;
    if (cc >= n) continue;
    if (SH && cc + VEC > n) cc = n - VEC;
    const A* p = part + slot0 * n + cc;
    A acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = A(0);
    constexpr int kPre = 8;  // partial rows in flight (the adds stay in chunk order)
    int64_t q = 0;
    for (; q + kPre <= nc; q += kPre) {
      A x[kPre][VEC];
#pragma unroll
      for (int u = 0; u < kPre; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) x[u][e] = coh_load(p + (q + u) * n + e);
#pragma unroll
      for (int u = 0; u < kPre; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + x[u][e];
    }
    for (; q < nc; ++q)
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + coh_load(p + q * n + e);
    store_row<T, VEC, false>(C + lr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
  }
  if (gl == 0) coh_store(arrive + slot0, 0u);
}

// Block-engine sizes (compile-time knobs for A/B builds: probes/ab_build.sh): bytes of products
// per LDS buffer, nonzeros per batch, B-row loads per lane per batch.
#ifndef OFX_BE_LDS
#define OFX_BE_LDS 16384
#endif
#ifndef OFX_BE_NB_CAP
#define OFX_BE_NB_CAP 128
#endif
#ifndef OFX_BE_UW_CAP
#define OFX_BE_UW_CAP 8
#endif

// ---- small form: one launch, no plan, no workspace -------------------------------------------
// Launches with few rows and little B-row traffic (use_small_form) run as ONE kernel.  Block b
// owns rows [b*RPB, (b+1)*RPB), one lane-group per row.  A group takes its row when the row has at
// most `light` nonzeros and is not split (accumulate, the group form).  The block's longer rows
// are then taken one at a time by the whole block: each of its GB lane-groups loads the B rows of
// a strided share of a batch of NB nonzeros, the products go to LDS, and the first lane-group of
// wave 0 adds them in nonzero order while the next batch's loads are in flight.  A row longer
// than `split` runs chunk by chunk and its chunk sums are added in chunk order from +0: the bits
// of the planned form's partials + spmm_reduce (and of the CPU kernel).
template <typename T, typename I, typename K>
struct SmallForm {
  using A = typename Num<T>::acc;
  static constexpr int kThreads = 64 * K::WPB;
  static constexpr int W = K::LPR * K::VEC;               // columns per pass
  static constexpr int G = 64 / K::LPR;                   // lane-groups per wave
  static constexpr int GB = G * K::WPB;                   // lane-groups per block
  static constexpr int RPB = GB;                          // rows per block
  static constexpr int D = 4;                             // batches of B-row loads in flight
  static constexpr int S = 8;                             // batches per (col, val) span
  static constexpr int kLdsElems = OFX_BE_LDS / (int)sizeof(A);  // 16 KB of products per buffer
  static constexpr int NB_RAW0 = kLdsElems / W < OFX_BE_NB_CAP ? kLdsElems / W : OFX_BE_NB_CAP;
  static constexpr int UW_RAW = NB_RAW0 / GB;
  static constexpr int UW = UW_RAW > OFX_BE_UW_CAP ? OFX_BE_UW_CAP : (UW_RAW < 1 ? 1 : UW_RAW);  // loads per lane per batch
  static constexpr int NB = UW * GB;                      // nonzeros per batch
  static constexpr int SPAN = S * NB;                     // nonzeros per (col, val) span
  static constexpr int PT = (SPAN + kThreads - 1) / kThreads;  // span entries per thread
  // one element per lane: products column-major ([column][nonzero], rows padded by 4), so the
  // in-order adds read 4 consecutive nonzeros per 16-B LDS read; wider lanes: row-major
  static constexpr bool kColMajor = K::VEC == 1 && sizeof(A) == 4 && NB % 4 == 0;
  static constexpr int NBP = NB + 4;
  static constexpr int kBufElems = kColMajor ? W * NBP : NB * W;
  static_assert(S % D == 0 && S > D, "small form: span must hold whole rounds of the load ring");
  static_assert(kBufElems * (int)sizeof(A) <= OFX_BE_LDS + 4 * W * (int)sizeof(A),
                "small form: LDS batch too large");
};

// Shared memory of the small form: two product buffers and two (col, val) span buffers.
template <typename T, typename I, typename K>
struct SmallLds {
  using SF = SmallForm<T, I, K>;
  using A = typename Num<T>::acc;
  A prod[2 * SF::kBufElems];
  A sval[2 * SF::SPAN];
  I scol[2 * SF::SPAN];
};

// acc[e] (valid in wave 0, group 0) = sum over j in [j0, j1) of val[j] * B[col[j], cc + e], in
// ascending j from +0, computed by the whole block (see above).  Every thread of the block calls
// this with the same j0/j1.
//   (col, val) of S batches (a span) are loaded coalesced by the whole block into LDS, one span
//   ahead; every other load has a fixed place in the schedule (rows past j1 read B row 0 and
//   are dropped), so a wait for one batch's B rows never waits for a younger batch's.
//   B rows: a ring of D batches in flight per lane; batch k + D is issued right after batch k's
//   products are in LDS.
//   Products of consecutive batches alternate between two LDS buffers, so one barrier per batch
//   orders the writes of batch k against the adds of batch k (after it) and of batch k - 1.
// Chunked traversal (kpc > 0): [j0, j1) is a whole split row whose chunks are kpc batches long
// (chunk = kpc * NB) and whose last chunk (nc - 1) takes the remainder.  The adder closes a chunk
// at each chunk boundary (total = total + acc; acc = +0) and returns total + the last chunk's
// sum: the contract's bits (each chunk from +0 in order, the partials in chunk order from +0)
// in one pipelined pass instead of one pass per chunk.
template <typename T, typename I, typename K>
__device__ __forceinline__ void block_accumulate(const I* __restrict__ col,
                                                 const T* __restrict__ val,
                                                 const I* __restrict__ vperm,
                                                 const BRows<T, K::BUF>& br,
                                                 int64_t j0, int64_t j1, int gb, int gl,
                                                 bool chain, SmallLds<T, I, K>& sh,
                                                 typename Num<T>::acc (&acc)[K::VEC],
                                                 int64_t kpc = 0, int64_t nc = 0) {
#pragma clang fp contract(off)
  using SF = SmallForm<T, I, K>;
  using A = typename Num<T>::acc;
  using P = Pack<T, K::VEC>;
  using PA = Pack<A, K::VEC>;
  constexpr int VEC = K::VEC, W = SF::W, GB = SF::GB, UW = SF::UW, NB = SF::NB, NBP = SF::NBP;
  constexpr int D = SF::D, S = SF::S, SPAN = SF::SPAN, PT = SF::PT, NT = SF::kThreads;
  const int tid = threadIdx.x;
  const int64_t nb = (j1 - j0 + NB - 1) / NB;  // batches
  // span s: nonzeros [j0 + s*SPAN, j0 + (s+1)*SPAN)
  auto span_load = [&](int64_t s, I (&c)[PT], A (&v)[PT]) {
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      const int e = p * NT + tid < SPAN ? p * NT + tid : SPAN - 1;
      const int64_t j = j0 + s * SPAN + e;
      // past j1: nonzero j1 - 1 again (a valid row; its products are never added)
      const int64_t jc = j < j1 ? j : j1 - 1;
      c[p] = OFX_LD(col + jc);
      v[p] = Num<T>::load(OFX_LD(val + (vperm ? (int64_t)OFX_LD(vperm + jc) : jc)));
    }
  };
  auto span_store = [&](int64_t s, const I (&c)[PT], const A (&v)[PT]) {
    const int off = (int)(s & 1) * SPAN;
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      if (p * NT + tid < SPAN) {
        sh.scol[off + p * NT + tid] = c[p];
        sh.sval[off + p * NT + tid] = v[p];
      }
    }
  };
  I rc[PT];  // the next span's (col, val), in flight until staged
  A rv[PT];
  A total[VEC];  // chunked traversal: the closed chunks' sum, in chunk order from +0
#pragma unroll
  for (int e = 0; e < VEC; ++e) total[e] = A(0);
  // B rows of batch kb (B row 0 for a batch past the end: its span buffer may hold anything)
  auto issue = [&](int64_t kb, P (&b)[UW]) {
    const int off = (int)((kb / S) & 1) * SPAN + (int)(kb % S) * NB;
    const int64_t live = -(int64_t)(kb < nb);
#pragma unroll
    for (int u = 0; u < UW; ++u) {
      const I c = sh.scol[off + GB * u + gb] & (I)live;
      b[u] = br.template load<K::BNT, P>(c);
    }
  };
  // batch k: products of the B rows in `b` -> LDS; (span staging); barrier; B rows of batch
  // k + D -> `b`; the in-order adds of batch k (wave 0, group 0)
  auto step = [&](int64_t k, P (&b)[UW], bool stage) {
    const int cnt = (int)((j1 - j0 - k * NB) < NB ? (j1 - j0 - k * NB) : NB);
    A* buf = sh.prod + (int)(k & 1) * SF::kBufElems;
    const int voff = (int)((k / S) & 1) * SPAN + (int)(k % S) * NB;
    A vv[UW];
#pragma unroll
    for (int u = 0; u < UW; ++u) vv[u] = sh.sval[voff + GB * u + gb];
#pragma unroll
    for (int u = 0; u < UW; ++u) {
      const int i = GB * u + gb;
      A pr[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) pr[e] = Num<T>::mul(vv[u], Num<T>::load(b[u].v[e]));
      if constexpr (SF::kColMajor) {
        buf[gl * NBP + i] = pr[0];
      } else if constexpr (VEC * sizeof(A) == 16 || VEC * sizeof(A) == 8) {
        PA o;
#pragma unroll
        for (int e = 0; e < VEC; ++e) o.v[e] = pr[e];
        *reinterpret_cast<PA*>(buf + i * W + gl * VEC) = o;
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) buf[i * W + gl * VEC + e] = pr[e];
      }
    }
    // stage (k % S == S - D): batch k + D opens the next span, which goes to LDS now (its loads
    // were issued a span earlier), and the span after it starts loading
    if (stage) span_store((k + D) / S, rc, rv);
    __syncthreads();
    if (stage) span_load((k + D) / S + 1, rc, rv);
    issue(k + D, b);
    if (chain) {
      if (kpc > 0 && k > 0 && k % kpc == 0 && k / kpc < nc) {  // batch k opens a new chunk
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          total[e] = total[e] + acc[e];
          acc[e] = A(0);
        }
      }
      // full rounds of reads in flight, then one guarded round for the rest of the batch (a
      // batch that is not a whole number of rounds pays one LDS wait for its tail, not one per
      // product)
      int i = 0;
      if constexpr (SF::kColMajor) {
        // column gl: 4 consecutive nonzeros per 16-B read, QR reads in flight
        constexpr int QR = 8;
        const A* cp = buf + gl * NBP;
        for (; i + 4 * QR <= cnt; i += 4 * QR) {
          Pack<A, 4> x[QR];
#pragma unroll
          for (int q = 0; q < QR; ++q) x[q] = *reinterpret_cast<const Pack<A, 4>*>(cp + i + 4 * q);
#pragma unroll
          for (int q = 0; q < QR; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[0] = acc[0] + x[q].v[e];
        }
        if (i < cnt) {
          Pack<A, 4> x[QR];
#pragma unroll
          for (int q = 0; q < QR; ++q)
            if (i + 4 * q < cnt) x[q] = *reinterpret_cast<const Pack<A, 4>*>(cp + i + 4 * q);
#pragma unroll
          for (int q = 0; q < QR; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (i + 4 * q + e < cnt) acc[0] = acc[0] + x[q].v[e];
        }
      } else {
        constexpr int QR = 16;
        for (; i + QR <= cnt; i += QR) {
          PA x[QR];
#pragma unroll
          for (int q = 0; q < QR; ++q)
            x[q] = *reinterpret_cast<const PA*>(buf + (i + q) * W + gl * VEC);
#pragma unroll
          for (int q = 0; q < QR; ++q)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + x[q].v[e];
        }
        if (i < cnt) {
          PA x[QR];
#pragma unroll
          for (int q = 0; q < QR; ++q)
            if (i + q < cnt) x[q] = *reinterpret_cast<const PA*>(buf + (i + q) * W + gl * VEC);
#pragma unroll
          for (int q = 0; q < QR; ++q)
            if (i + q < cnt)
#pragma unroll
              for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + x[q].v[e];
        }
      }
    }
  };
  span_load(0, rc, rv);
  span_store(0, rc, rv);
  __syncthreads();
  span_load(1, rc, rv);  // stored when batch S is first issued
  // the ring: four named register sets, so batch k's rows stay in flight until step k
  static_assert(D == 4, "small form: the load ring below is written out for D = 4");
  P b0[UW], b1[UW], b2[UW], b3[UW];
  issue(0, b0);
  issue(1, b1);
  issue(2, b2);
  issue(3, b3);
  // whole spans: no guards, the same loads outstanding at every step of every span (and at the
  // loop entry), so each step's wait covers exactly its own batch
  static_assert(S == 2 * D, "small form: a span is two turns of the ring");
  int64_t k0 = 0;
  for (; k0 + S <= nb; k0 += S) {
    step(k0 + 0, b0, false);
    step(k0 + 1, b1, false);
    step(k0 + 2, b2, false);
    step(k0 + 3, b3, false);
    step(k0 + 4, b0, true);
    step(k0 + 5, b1, false);
    step(k0 + 6, b2, false);
    step(k0 + 7, b3, false);
  }
  // the last, partial span (its batches were staged by the loop or the prologue)
  if (k0 + 0 < nb) step(k0 + 0, b0, false);
  if (k0 + 1 < nb) step(k0 + 1, b1, false);
  if (k0 + 2 < nb) step(k0 + 2, b2, false);
  if (k0 + 3 < nb) step(k0 + 3, b3, false);
  if (k0 + 4 < nb) step(k0 + 4, b0, false);
  if (k0 + 5 < nb) step(k0 + 5, b1, false);
  if (k0 + 6 < nb) step(k0 + 6, b2, false);
  if (kpc > 0) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = total[e] + acc[e];
  }
  __syncthreads();  // the next call's first batch writes buffer 0, which the adds may still read
}

template <typename T, typename I, typename K>
__global__ void __launch_bounds__(64 * K::WPB)
    spmm_small_kernel(const I* __restrict__ rp, const I* __restrict__ col,
                      const T* __restrict__ val, const I* __restrict__ vperm,
                      const T* __restrict__ B, int64_t ldb, int64_t kb, T* __restrict__ C,
                      int64_t ldc, int64_t row_begin, int64_t nrows, int64_t n, int64_t split,
                      int64_t chunk,
                      int64_t light, const T* __restrict__ bias, int act) {
  using SF = SmallForm<T, I, K>;
  using A = typename Num<T>::acc;
  constexpr int VEC = K::VEC, LPR = K::LPR, W = SF::W, RPB = SF::RPB;
  __shared__ __attribute__((aligned(16))) SmallLds<T, I, K> lds;
  __shared__ int heavy_rows[RPB];
  __shared__ int nheavy;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gl = lane & (LPR - 1);
  const int gbase = lane & ~(LPR - 1);
  const int q = LPR == 64 ? 0 : lane / LPR;
  const int gb = wave * SF::G + q;  // lane-group of the block
  const int64_t row0 = (int64_t)blockIdx.x * RPB;
  if (threadIdx.x == 0) nheavy = 0;
  __syncthreads();
  const int64_t lr = row0 + gb;
  if (lr < nrows) {
    const int64_t rs = (int64_t)OFX_LD(rp + (row_begin + lr));
    const int64_t re = (int64_t)OFX_LD(rp + (row_begin + lr + 1));
    const int64_t len = re - rs;
    if (len > light || len > split) {
      if (gl == 0) heavy_rows[atomicAdd(&nheavy, 1)] = gb;
    } else {
      for (int64_t c0 = 0; c0 < n; c0 += W) {
        const int64_t cc = c0 + (int64_t)gl * VEC;
        const bool active = cc < n;
        A acc[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = A(0);
        accumulate<T, I, K>(col, val, vperm, brows<T, K::BUF>(B, c0, cc, active, ldb, kb), rs, re, gl, gbase,
                            active, acc);
        if (active) store_row<T, VEC, K::NT>(C + lr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
      }
    }
  }
  __syncthreads();
  const int nh = nheavy;
  const bool chain = wave == 0 && q == 0;
  for (int h = 0; h < nh; ++h) {
    const int64_t hr = row0 + heavy_rows[h];
    const int64_t rs = (int64_t)OFX_LD(rp + (row_begin + hr));
    const int64_t re = (int64_t)OFX_LD(rp + (row_begin + hr + 1));
    const bool split_row = re - rs > split;
    const int64_t nc = split_row ? num_chunks(re - rs, chunk) : 1;
    // chunks of whole batches: the row in one chunked pass (block_accumulate)
    const bool one_pass = split_row && chunk % SF::NB == 0;
    for (int64_t c0 = 0; c0 < n; c0 += W) {
      const int64_t cc = c0 + (int64_t)gl * VEC;
      const bool active = cc < n;
      const BRows<T, K::BUF> br = brows<T, K::BUF>(B, c0, cc, active, ldb, kb);
      A total[VEC], acc[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) total[e] = A(0);
      if (one_pass) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = A(0);
        block_accumulate<T, I, K>(col, val, vperm, br, rs, re, gb, gl, chain, lds, acc,
                                  chunk / SF::NB, nc);
        if (chain && active) store_row<T, VEC, K::NT>(C + hr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
        continue;
      }
      for (int64_t ci = 0; ci < nc; ++ci) {
        int64_t j0 = rs, j1 = re;
        if (split_row) {
          j0 = rs + ci * chunk;
          j1 = (re - j0 - chunk < chunk) ? re : j0 + chunk;
        }
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = A(0);
        block_accumulate<T, I, K>(col, val, vperm, br, j0, j1, gb, gl, chain, lds, acc);
        if (split_row) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) total[e] = total[e] + acc[e];
        }
      }
      if (chain && active)
        store_row<T, VEC, K::NT>(C + hr * ldc + cc, split_row ? total : acc,
                                 bias ? bias + cc : nullptr, act);
    }
  }
}

// ---- main kernel: one work list = hub chunks, then rows in bin order ------------------------
// Without a plan (`order` == nullptr) the list is simply the rows in index order.
#ifdef OFX_AB_WPE  // A/B builds only (probes/ab_build.sh): waves per SIMD the registers must allow
#define OFX_MAIN_WPE __attribute__((amdgpu_waves_per_eu(OFX_AB_WPE)))
#else
#define OFX_MAIN_WPE
#endif
// C[0, nrows) x [0, n) (row stride ldc) = the canonical quiet NaN, grid-stride over this launch.
// The first consumer of an invalid plan runs it instead of its rows (spmm_plan.h plan_valid).
template <typename T>
__device__ __attribute__((noinline)) void poison_output(T* __restrict__ C, int64_t ldc,
                                                        int64_t nrows, int64_t n) {
  const T p = poison_value<T>();
  const int64_t total = nrows * n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride)
    C[(e / n) * ldc + e % n] = p;
}

template <typename T, typename I, typename K>
__global__ void __launch_bounds__(64 * K::WPB) OFX_MAIN_WPE
    spmm_main_kernel(const I* __restrict__ rp, const I* __restrict__ col,
                     const T* __restrict__ val, const I* __restrict__ vperm,
                     const T* __restrict__ B, int64_t ldb, int64_t kb,
                     T* __restrict__ C, int64_t ldc, int64_t row_begin, int64_t nrows, int64_t n,
                     int64_t split, int64_t chunk, int64_t heavy,
                     const unsigned long long* __restrict__ counters,
                     const int64_t* __restrict__ items, const int64_t* __restrict__ order,
                     typename Num<T>::acc* __restrict__ part, const T* __restrict__ bias,
                     int act, int64_t wave_blocks, int64_t block_base,
                     unsigned* __restrict__ arrive, unsigned* err) {
  using A = typename Num<T>::acc;
  constexpr int VEC = K::VEC, LPR = K::LPR, kWaves = K::WPB;
  const int64_t bid = block_base + (int64_t)blockIdx.x;  // launches of > 2^31 threads are cut
  // a plan that failed, was superseded or never built: poison the output, loudly (spmm_plan.h);
  // every launch of a cut grid poisons all of C (idempotent) and spmm_reduce then writes nothing
  if (counters != nullptr && !plan::plan_valid(counters)) {
    if (bid == 0 && threadIdx.x == 0) plan::raise_device_error(err, plan::kErrPlanInvalid);
    poison_output<T>(C, ldc, nrows, n);
    return;
  }
  constexpr int GPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gl = lane & (LPR - 1);
  const int gbase = lane & ~(LPR - 1);
  const int gsub = LPR == 64 ? 0 : lane / LPR;
  if constexpr (K::WH && LPR < 64) {
    // blocks [0, wave_blocks): one wave per hub chunk / heavy row (the plan's first items)
    using KW = WaveMap<K>;
    constexpr int WV = KW::VEC, WL = KW::LPR;
    if (bid < wave_blocks) {
      // the wave_blocks * WPB waves stride over the items (the grid bound is an estimate; the
      // plan's counters hold the count), so the launch carries no blocks that only exit
      const int wgl = lane & (WL - 1);
      const int64_t nchunks = (int64_t)OFX_LD(counters + 0);
      const int64_t nheavy = (int64_t)OFX_LD(counters + 3) - (int64_t)OFX_LD(counters + 2);  // bin 0
      for (int64_t w = bid * kWaves + wave; w < nchunks + nheavy; w += wave_blocks * kWaves) {
        int64_t wr, wc = -1;
        if (w < nchunks) {
          wr = OFX_LD(items + (2 * w + 0));
          wc = OFX_LD(items + (2 * w + 1));
        } else {
          wr = plan::order_row(order, nrows, nheavy, w - nchunks);  // a heavy row
        }
        wr = uniform64(wr);
        wc = uniform64(wc);
        const int64_t rs = (int64_t)OFX_LD(rp + (row_begin + wr));
        const int64_t re = (int64_t)OFX_LD(rp + (row_begin + wr + 1));
        int64_t j0 = rs, j1 = re;
        if (wc >= 0) {
          j0 = rs + wc * chunk;
          j1 = (re - j0 - chunk < chunk) ? re : j0 + chunk;
        }
        for (int64_t c0 = 0; c0 < n; c0 += (int64_t)WL * WV) {
          int64_t cc = c0 + (int64_t)wgl * WV;
          const bool active = cc < n;
          if constexpr (K::SH && WV > 1) {
            if (active && cc + WV > n) cc = n - WV;  // the window ending at column n - 1
          }
          A acc[WV];
#pragma unroll
          for (int e = 0; e < WV; ++e) acc[e] = A(0);
          if constexpr (K::XL) {
            __shared__ A xl_lds[K::WPB][KW::XL_FLOATS];
            accumulate_wave_xl<T, I, KW>(col, val, vperm, brows<T, K::BUF>(B, c0, cc, active, ldb, kb),
                                         j0, j1, lane, wgl, xl_lds[wave], acc);
          } else {
            accumulate_wave<T, I, KW>(col, val, vperm, brows<T, K::BUF>(B, c0, cc, active, ldb, kb),
                                      j0, j1, lane, wgl, acc);
          }
          if (active && lane < WL) {
            if (wc >= 0)
              store_partial<A, WV, K::LR>(part + w * n + cc, acc);
            else
              store_row<T, WV, K::NT>(C + wr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
          }
        }
        if constexpr (K::LR) {
          if (wc >= 0)
            hub_tail<T, WV, WL, K::SH && (WV > 1)>(arrive, w - wc, num_chunks(re - rs, chunk), part, C, ldc,
                                       wr, n, wgl, lane < WL, 0, bias, act);
        }
      }
      return;
    }
  }
  if constexpr (K::BI) {
    // blocks [0, wave_blocks): one block per hub chunk / heavy row (the plan's first items).
    // A block returns or runs its item as a whole, so block_accumulate's barriers are uniform.
    if (bid < wave_blocks) {
      __shared__ __attribute__((aligned(16))) SmallLds<T, I, K> lds;
      constexpr int W = SmallForm<T, I, K>::W;
      const int64_t w = bid;
      const int64_t nchunks = (int64_t)OFX_LD(counters + 0);
      const int64_t nheavy = (int64_t)OFX_LD(counters + 3) - (int64_t)OFX_LD(counters + 2);  // bin 0
      if (w >= nchunks + nheavy) return;
      int64_t wr, wc = -1;
      if (w < nchunks) {
        wr = OFX_LD(items + (2 * w + 0));
        wc = OFX_LD(items + (2 * w + 1));
      } else {
        wr = plan::order_row(order, nrows, nheavy, w - nchunks);  // a heavy row
      }
      wr = uniform64(wr);
      wc = uniform64(wc);
      const int64_t rs = (int64_t)OFX_LD(rp + (row_begin + wr));
      const int64_t re = (int64_t)OFX_LD(rp + (row_begin + wr + 1));
      int64_t j0 = rs, j1 = re;
      if (wc >= 0) {
        j0 = rs + wc * chunk;
        j1 = (re - j0 - chunk < chunk) ? re : j0 + chunk;
      }
      const int gb = wave * GPW + gsub;  // lane-group of the block
      const bool chain = wave == 0 && gsub == 0;
      for (int64_t c0 = 0; c0 < n; c0 += W) {
        const int64_t cc = c0 + (int64_t)gl * VEC;
        const bool active = cc < n;
        A acc[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = A(0);
        block_accumulate<T, I, K>(col, val, vperm, brows<T, K::BUF>(B, c0, cc, active, ldb, kb), j0, j1, gb, gl,
                                  chain, lds, acc);
        if (chain && active) {
          if (wc >= 0)
            store_partial<A, VEC, K::LR>(part + w * n + cc, acc);
          else
            store_row<T, VEC, K::NT>(C + wr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
        }
      }
      if constexpr (K::LR) {
        if (wc >= 0 && chain)  // the chain group (wave 0, group 0) holds the partial row
          hub_tail<T, VEC, LPR, K::SH>(arrive, w - wc, num_chunks(re - rs, chunk), part, C, ldc, wr,
                                       n, gl, true, gbase, bias, act);
      }
      return;
    }
  }
  // one lane-group per work item; in the WH / BI forms these are the light rows after the wave /
  // block items
  int64_t g = ((bid - ((K::WH || K::BI) ? wave_blocks : 0)) * kWaves + wave) * GPW +
              gsub;
  if constexpr ((K::WH && LPR < 64) || K::BI) {
    if (order != nullptr)
      g += (int64_t)OFX_LD(counters + 0) + (int64_t)OFX_LD(counters + 3) -
           (int64_t)OFX_LD(counters + 2);
  }
  // Work items with a plan: hub chunks, then the heavy rows (bin 0 of `order`), then the light
  // rows in index order, taken one of two ways (the same rows, the same bits):
  //   by index  every row index gets a group, and a group whose row is a hub or heavy row (done
  //             by the items before) exits.  No order[q] load in the light row's chain (order ->
  //             row_ptr -> (col, val) -> B rows), which is what bounds the short rows of a
  //             latency-bound launch; but an exited group leaves its lanes idle while the other
  //             groups of its wave work, so it pays only when few rows are excluded;
  //   by order  the plan's light bin (order[q]), dense.
  // By index when hubs + heavy rows are at most 1/kIdxExcluded of the rows (power-law graphs:
  // 1.7-1.8%; Reddit-shaped: 53% hubs, where it cost 9%).
  constexpr int64_t kIdxExcluded = 16;
#if defined(OFX_LIGHT_ORDER)
  constexpr bool kIdx = false;  // A/B builds only (probes/ab_build.sh)
#else
  constexpr bool kIdx = true;
#endif
  int64_t lr, c = -1;  // local row; chunk index or -1 for a whole row
  bool by_index = false;
  if (order == nullptr) {
    if (g >= nrows) return;
    lr = g;
  } else {
    const int64_t nchunks = (int64_t)OFX_LD(counters + 0);
    const int64_t nhubs = (int64_t)OFX_LD(counters + 1);
    const int64_t nheavy = (int64_t)OFX_LD(counters + 3) - (int64_t)OFX_LD(counters + 2);  // bin 0
#if defined(OFX_LIGHT_INDEX)
    const bool idx = true;
#else
    const bool idx = kIdx && (nhubs + nheavy) * kIdxExcluded <= nrows;
#endif
    if (g < nchunks) {
      lr = OFX_LD(items + (2 * g + 0));
      c = OFX_LD(items + (2 * g + 1));
    } else if (g < nchunks + nheavy || !idx) {
      const int64_t q = g - nchunks;
      if (q >= nrows - nhubs) return;
      lr = plan::order_row(order, nrows, nheavy, q);
    } else {
      lr = g - nchunks - nheavy;
      if (lr >= nrows) return;
      by_index = true;
    }
  }
  if constexpr (LPR == 64) {
    lr = uniform64(lr);
    c = uniform64(c);
  }
  const int64_t rs = (int64_t)OFX_LD(rp + (row_begin + lr));
  const int64_t re = (int64_t)OFX_LD(rp + (row_begin + lr + 1));
  if (by_index && (re - rs > split || re - rs > heavy)) return;  // a hub or a heavy row
  int64_t j0 = rs, j1 = re;
  if (c >= 0) {
    // chunk c of num_chunks(len, chunk) = len / chunk; the last one (fewer than 2 * chunk
    // nonzeros left from its start) takes the remainder.  No 64-bit division per work item.
    j0 = rs + c * chunk;
    j1 = (re - j0 - chunk < chunk) ? re : j0 + chunk;
  }
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)LPR * VEC) {
    int64_t cc = c0 + (int64_t)gl * VEC;
    const bool active = cc < n;
    if constexpr (K::SH) {
      // n not a multiple of VEC: the lane holding the row's last columns takes the window ending
      // at column n - 1; its first columns repeat its neighbour's (the same sums in the same order,
      // written twice with the same bits)
      if (active && cc + VEC > n) cc = n - VEC;
    }
    A acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = A(0);
    accumulate<T, I, K>(col, val, vperm, brows<T, K::BUF>(B, c0, cc, active, ldb, kb), j0, j1, gl, gbase, active,
                        acc);
    if (active) {
      if (c >= 0)
        store_partial<A, VEC, K::LR>(part + g * n + cc, acc);
      else
        store_row<T, VEC, K::NT>(C + lr * ldc + cc, acc, bias ? bias + cc : nullptr, act);
    }
  }
  if constexpr (K::LR) {
    if (c >= 0)
      hub_tail<T, VEC, LPR, K::SH>(arrive, g - c, num_chunks(re - rs, chunk), part, C, ldc, lr, n,
                                   gl, true, gbase, bias, act);
  }
}

// ---- hub reduce: C[hub row] = ((0 + part[chunk 0]) + part[chunk 1]) + ... (chunk order) ---------
// One group of L lanes per hub (64/L hubs per wave); each lane owns VEC consecutive columns and
// reads them as one 16-B vector per partial row, kPre partial rows in flight before the in-order
// adds.  Memory-level parallelism is what bounds this pass (Reddit: ~450k chunk partials of 1 KB):
// a 256-thread block per hub with 4-B loads ran at 3.1 TB/s; 16-B loads over 64/L hubs per wave
// keep 4x the bytes in flight (Reddit 148 -> 125 us, products unchanged at 33 us; a separate
// one-lane-per-column kernel with 64 partials in flight for hubs of > 64 chunks measured slower
// for both, 45 / 147 us, and was dropped).

template <typename T, int VEC, int L>
__global__ void __launch_bounds__(kBlock)
    spmm_reduce_kernel(const unsigned long long* __restrict__ counters,
                       const int64_t* __restrict__ hubs,
                       const typename Num<T>::acc* __restrict__ part, T* __restrict__ C,
                       int64_t ldc, int64_t n, const T* __restrict__ bias, int act) {
#pragma clang fp contract(off)
  using A = typename Num<T>::acc;
  using P = Pack<A, VEC>;
  constexpr int kPre = 16;  // partial rows in flight per lane (the adds stay in chunk order)
  if (!plan::plan_valid(counters)) return;  // spmm_main reported it and poisoned C
  const int64_t nhubs = (int64_t)OFX_LD(counters + 1);
  const int gl = threadIdx.x % L;
  const int64_t groups = (int64_t)gridDim.x * (kBlock / L);
  for (int64_t h = (int64_t)blockIdx.x * (kBlock / L) + threadIdx.x / L; h < nhubs; h += groups) {
    const int64_t lr = OFX_LD(hubs + (3 * h + 0));
    const int64_t slot = OFX_LD(hubs + (3 * h + 1));
    const int64_t nc = OFX_LD(hubs + (3 * h + 2));
    for (int64_t c = (int64_t)gl * VEC; c < n; c += (int64_t)L * VEC) {
      const A* p = part + slot * n + c;
      A acc[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] = A(0);
      int64_t q = 0;
      for (; q + kPre <= nc; q += kPre) {
        P v[kPre];
#pragma unroll
        for (int u = 0; u < kPre; ++u) v[u] = OFX_LD(reinterpret_cast<const P*>(p + (q + u) * n));
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + v[u].v[e];
        }
      }
      for (; q < nc; ++q) {
        const P v = OFX_LD(reinterpret_cast<const P*>(p + q * n));
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] = acc[e] + v.v[e];
      }
      if (bias && !OFX_DOK(bias + c, sizeof(T) * VEC)) continue;  // OFX_DEBUG_BOUNDS builds only
#pragma unroll
      for (int e = 0; e < VEC; ++e) OFX_ST(&C[lr * ldc + c + e], epilogue<T>(acc[e], bias, c + e, act));
    }
  }
}

template <typename T, int VEC>
int launch_reduce_vec(hipStream_t s, int64_t max_hubs, int64_t n,
                      const unsigned long long* counters, const int64_t* hubs,
                      const typename Num<T>::acc* part, T* C, int64_t ldc, const T* bias, int act) {
  const int64_t lanes = (n + VEC - 1) / VEC;
  int l = 4;
  while (l < 64 && l < lanes) l *= 2;
  const int64_t per_block = kBlock / l;
  int64_t grid = (max_hubs + per_block - 1) / per_block;
  if (grid > kMaxReduceBlocks) grid = kMaxReduceBlocks;
#define OFX_REDUCE(LL)                                                                        \
  hipLaunchKernelGGL((spmm_reduce_kernel<T, VEC, LL>), dim3((unsigned)grid), dim3(kBlock), 0, s, \
                     counters, hubs, part, C, ldc, n, bias, act)
  switch (l) {
    case 4: OFX_REDUCE(4); break;
    case 8: OFX_REDUCE(8); break;
    case 16: OFX_REDUCE(16); break;
    case 32: OFX_REDUCE(32); break;
    default: OFX_REDUCE(64); break;
  }
#undef OFX_REDUCE
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

// 16-B partial loads when every partial row starts 16-B aligned (the workspace base is 256-B
// aligned and rows are n accumulators apart), else one accumulator per lane.
template <typename T>
int launch_reduce(hipStream_t s, int64_t max_hubs, int64_t n, const unsigned long long* counters,
                  const int64_t* hubs, const typename Num<T>::acc* part, T* C, int64_t ldc,
                  const T* bias, int act) {
  using A = typename Num<T>::acc;
  constexpr int kVec = 16 / (int)sizeof(A);
  if ((n * (int64_t)sizeof(A)) % 16 == 0)
    return launch_reduce_vec<T, kVec>(s, max_hubs, n, counters, hubs, part, C, ldc, bias, act);
  return launch_reduce_vec<T, 1>(s, max_hubs, n, counters, hubs, part, C, ldc, bias, act);
}

int pick_vec(int elem_bytes, const Launch& L, int forced_vec, int cap = 16) {
  const int maxvec = std::min(16 / elem_bytes, cap);
  for (int v = maxvec; v >= 1; v /= 2) {
    if (forced_vec && v != forced_vec) continue;
    const size_t vb = (size_t)v * elem_bytes;
    if (L.n % v == 0 && L.ldb % v == 0 && L.ldc % v == 0 &&
        ((uintptr_t)L.b % vb) == 0 && ((uintptr_t)L.c % vb) == 0)
      return v;
  }
  return 0;
}

int pick_lpr(int64_t n, int vec) {
  const int64_t lanes = (n + vec - 1) / vec;
  int l = 4;
  while (l < 64 && l < lanes) l *= 2;
  return l;
}

// ofx_spmm_csr_describe: the configuration a launch takes (kind = "main" for the planned forms'
// spmm_main_kernel, "small" for spmm_small_kernel), written instead of launching.  The form names
// follow DESIGN.md §3: small, mid (block items), narrow (wave items of HL lanes), prefetch (PF
// without block items), bandwidth (the rest).
template <typename T, typename I, typename K>
int describe_cfg(const Launch& L, const char* kind) {
  const char* form = std::strcmp(kind, "small") == 0 ? "small"
                     : K::BI                         ? "mid"
                     : (K::WH && K::HL > 0)          ? "narrow"
                     : K::PF                         ? "prefetch"
                                                     : "bandwidth";
  // the workspace this launch lays out (<= ofx_spmm_csr_workspace_size over the matrix's m)
  const size_t ws = std::strcmp(kind, "small") == 0
                        ? 0
                        : ws_layout(L.nrows, L.nnz, L.n, sizeof(typename Num<T>::acc), L.sched).total;
  std::snprintf(L.describe, L.describe_bytes,
                "form=%s kernel=%s VEC=%d LPR=%d U=%d WPB=%d NT=%d PF=%d WH=%d BI=%d BUF=%d SH=%d "
                "HL=%d HU=%d HV=%d XL=%d LR=%d elem=%d idx=%d ws=%zu",
                form, kind, K::VEC, K::LPR, K::U, K::WPB, (int)K::NT, (int)K::PF, (int)K::WH,
                (int)K::BI, (int)K::BUF, (int)K::SH, K::HL, K::HU, K::HV, (int)K::XL, (int)K::LR,
                (int)sizeof(T),
                (int)sizeof(I), ws);
  return OFX_OK;
}

#ifdef OFX_DEBUG_BOUNDS
// OFX_DEBUG_BOUNDS builds: the launch's allocations (dbg_bounds.h), published on its stream before
// its kernels, and its configuration as the tag recorded with a violation:
// VEC | LPR << 8 | U << 16 | flags << 24 (NT PF BNT WH BI BUF SH LR) | HL << 32 | HU << 40 |
// kind << 48
template <typename T, typename I, typename K>
int debug_publish(const Launch& L, unsigned long long kind) {
  dbg::HostBounds hb;
  const int64_t si = (int64_t)sizeof(I), st = (int64_t)sizeof(T);
  hb.add(L.rp, (uint64_t)((L.row_begin + L.nrows + 1) * si));
  hb.add(L.col, (uint64_t)(L.nnz * si));
  hb.add(L.val, (uint64_t)(L.nnz * st));
  hb.add(L.vperm, (uint64_t)(L.nnz * si));
  if (L.b_rows > 0) hb.add(L.b, (uint64_t)(((L.b_rows - 1) * L.ldb + L.n) * st));
  hb.add(L.c, (uint64_t)(((L.nrows - 1) * L.ldc + L.n) * st));
  hb.add(L.ws, L.ws_bytes);
  hb.add(L.bias, (uint64_t)(L.n * st));
  void* zero = nullptr;
  OFX_HIP_CHECK(hipGetSymbolAddress(&zero, HIP_SYMBOL(g_zero_row)));
  hb.add(zero, kZeroRowBytes);
  const unsigned long long flags = (unsigned long long)K::NT | (unsigned long long)K::PF << 1 |
                                   (unsigned long long)K::BNT << 2 | (unsigned long long)K::WH << 3 |
                                   (unsigned long long)K::BI << 4 | (unsigned long long)K::BUF << 5 |
                                   (unsigned long long)K::SH << 6 | (unsigned long long)K::LR << 7;
  const unsigned long long tag = (unsigned long long)K::VEC | (unsigned long long)K::LPR << 8 |
                                 (unsigned long long)K::U << 16 | flags << 24 |
                                 (unsigned long long)K::HL << 32 | (unsigned long long)K::HU << 40 |
                                 kind << 48;
  OFX_REQUIRE(hb.publish(L.stream, tag) == 0, OFX_EDEVICE, "spmm_csr: debug bounds not published");
  return OFX_OK;
}
#endif

template <typename T, typename I, typename K>
int launch_cfg(const Launch& L) {
  if (L.describe != nullptr) return describe_cfg<T, I, K>(L, "main");
  using A = typename Num<T>::acc;
  constexpr int GPW = 64 / K::LPR;
  constexpr int64_t GPB = (int64_t)K::WPB * GPW;  // lane-groups per block
  const I* rp = static_cast<const I*>(L.rp);
  const I* col = static_cast<const I*>(L.col);
  const T* val = static_cast<const T*>(L.val);
  const T* B = static_cast<const T*>(L.b);
  T* C = static_cast<T*>(L.c);
  const WsLayout w = ws_layout(L.nrows, L.nnz, L.n, sizeof(A), L.sched);
  const bool plan = w.total > 0;
#ifdef OFX_DEBUG_BOUNDS
  if (const int rc = debug_publish<T, I, K>(L, 1)) return rc;
#endif
  WorkList wl{};
  if (plan) {
    OFX_REQUIRE(L.ws != nullptr && L.ws_bytes >= w.total, OFX_EWORKSPACE,
                "spmm_csr: workspace of %zu bytes is smaller than the %zu bytes required",
                L.ws_bytes, w.total);
    if (L.sched.planned) {
      plan::worklist_of(w, static_cast<char*>(L.ws), &wl);
    } else {
      const int rc = launch_plan<I>(L.stream, rp, L.row_begin, L.nrows, L.nnz_est, L.sched, w,
                                    static_cast<char*>(L.ws), &wl);
      if (rc) return rc;
    }
  }
  unsigned long long* counters = wl.counters;
  int64_t *hub = wl.hubs, *items = wl.items, *order = wl.order;
  A* part = reinterpret_cast<A*>(wl.part);
  // Work items: hub chunks, heavy rows, then every row by index (surplus groups exit at once).
  // The WH / BI forms put one wave / block per hub chunk and heavy row first (upper bound: every
  // chunk and every row longer than the heavy threshold), then the groups of the rows.
  const int64_t heavy = L.sched.heavy == 0 ? auto_heavy(L.nrows, L.nnz_est) : L.sched.heavy;
  const int64_t heavy_bound =
      heavy == INT64_MAX ? 0 : std::min<int64_t>(L.nrows, L.nnz / (heavy + 1) + 1);
  const int64_t bi_items = w.max_chunks + heavy_bound;
  // wave items (one wave each) and block items (one block each) are bounded alike: hub chunks
  // plus the rows above the heavy threshold.  The wave items loop (a wave strides over them), so
  // their blocks are capped at kWaveItemBlocks; the light rows then need one group per row.
  constexpr int64_t kWaveItemBlocks = 2048;
  const bool wh = K::WH && K::LPR < 64 && plan;
  const int64_t wave_blocks = wh ? std::min<int64_t>((bi_items + K::WPB - 1) / K::WPB, kWaveItemBlocks)
                              : (K::BI && plan) ? bi_items
                                                : 0;
  const int64_t work = L.nrows + (plan && !wh && !K::BI ? bi_items : 0);
  const int64_t grid = wave_blocks + (work + GPB - 1) / GPB;
  // A launch holds fewer than 2^32 threads (papers-scale: 111M rows + items at 8 groups per block
  // would not): the grid goes out in pieces of kLaunchBlocks, each told its first block.
  constexpr int64_t kLaunchBlocks = ((int64_t)1 << 31) / (64 * K::WPB);
  for (int64_t b0 = 0; b0 < grid; b0 += kLaunchBlocks) {
    const int64_t nb = std::min(kLaunchBlocks, grid - b0);
    hipLaunchKernelGGL((spmm_main_kernel<T, I, K>), dim3((unsigned)nb), dim3(64 * K::WPB), 0,
                       L.stream, rp, col, val, static_cast<const I*>(L.vperm), B, L.ldb, L.b_rows,
                       C, L.ldc, L.row_begin, L.nrows, L.n, plan ? L.sched.split : INT64_MAX,
                       plan ? L.sched.chunk : INT64_MAX, heavy, counters, items, order, part,
                       static_cast<const T*>(L.bias), L.act, wave_blocks, b0, wl.arrive,
                       plan ? device_error_words() : nullptr);
    OFX_HIP_CHECK(hipGetLastError());
  }
  if (plan && w.max_hubs > 0 && !K::LR)  // LR: the main kernel added the hubs (hub_tail)
    return launch_reduce<T>(L.stream, w.max_hubs, L.n, counters, hub, part, C, L.ldc,
                            static_cast<const T*>(L.bias), L.act);
  return OFX_OK;
}


template <typename T, typename I, typename K>
int launch_small(const Launch& L) {
  if (L.describe != nullptr) return describe_cfg<T, I, K>(L, "small");
  using SF = SmallForm<T, I, K>;
  // options.heavy_threshold > 0 overrides the light/whole-block cut (tuning; no numeric effect)
  const int64_t light =
      (L.sched.heavy > 0 && L.sched.heavy != INT64_MAX) ? L.sched.heavy : (int64_t)kSmallLight * K::U;
  const int64_t grid = (L.nrows + SF::RPB - 1) / SF::RPB;
#ifdef OFX_DEBUG_BOUNDS
  if (const int rc = debug_publish<T, I, K>(L, 2)) return rc;
#endif
  OFX_REQUIRE(grid < (int64_t)UINT32_MAX, OFX_EINVAL, "spmm_csr: too many rows (%lld)",
              (long long)L.nrows);
  hipLaunchKernelGGL((spmm_small_kernel<T, I, K>), dim3((unsigned)grid), dim3(64 * K::WPB), 0,
                     L.stream, static_cast<const I*>(L.rp), static_cast<const I*>(L.col),
                     static_cast<const T*>(L.val), static_cast<const I*>(L.vperm),
                     static_cast<const T*>(L.b), L.ldb, L.b_rows, static_cast<T*>(L.c), L.ldc,
                     L.row_begin,
                     L.nrows, L.n, L.sched.split, L.sched.chunk, light,
                     static_cast<const T*>(L.bias), L.act);
  OFX_HIP_CHECK(hipGetLastError());
  return OFX_OK;
}

template <typename T, typename I, typename K>
int launch_small_or_planned(const Launch& L) {
  if (use_small_form(L.nrows, L.nnz_est, L.n, L.sched)) return launch_small<T, I, K>(L);
  return launch_cfg<T, I, K>(L);
}

// B far larger than the Infinity Cache (> 1 GiB): the col/val/C streams are loaded and stored
// non-temporally so they do not evict the hot (hub) B rows that still hit on-die.  Measured
// (scripts/ab.py, bit-identical): papers-scale -1.8%, products -0.3%; with B at cache size
// (1M power-law, 256 MB) the same hint costs +8%, hence the threshold.
constexpr int64_t kNtBytes = int64_t(1) << 30;

// Small problems (<= kSmallRows rows: too few lane-groups to be bandwidth-bound) run as long as
// their longest non-split row, a chain of len / U dependent B-row load rounds; these launches keep
// 32 (16 for 8-16 B lanes) loads in flight per lane instead of 8.  A Cora-shaped layer (max row
// 253 nonzeros, N=16) took 25 us with U=8.  Same bits: U only changes how many loads are issued
// ahead of the in-order adds.  Below kSmallFormElems products the launch is the small form.
template <typename T, typename I, int VEC>
int launch_vec_small(const Launch& L, int lpr) {
  constexpr int U = VEC * sizeof(T) <= 4 ? 32 : 16;
  switch (lpr) {
    case 4: return launch_small_or_planned<T, I, Cfg<VEC, 4, U, 4, false, true, false, true>>(L);
    case 8: return launch_small_or_planned<T, I, Cfg<VEC, 8, U, 4, false, true, false, true>>(L);
    case 16: return launch_small_or_planned<T, I, Cfg<VEC, 16, U, 4, false, true, false, true>>(L);
    case 32: return launch_small_or_planned<T, I, Cfg<VEC, 32, U, 4, false, true, false, true>>(L);
    case 64: return launch_small_or_planned<T, I, Cfg<VEC, 64, U, 4, false, false, false, false>>(L);
    default: return fail(OFX_EINVAL, "spmm_csr: unsupported lanes-per-row %d", lpr);
  }
}

// The prefetching form (use_prefetch_form): U = 32 / 16 loads in flight per lane, the next batch's
// (col, val) prefetched; WH: hub chunks and heavy rows take a whole wave (wave items).  Tuning
// variants 30004 (WH) / 30005 force it at any size.
template <typename T, typename I, int VEC, bool WH>
int launch_vec_pf(const Launch& L, int lpr) {
  constexpr int U = VEC * sizeof(T) <= 4 ? 32 : 16;
  switch (lpr) {
    case 4: return launch_cfg<T, I, Cfg<VEC, 4, U, 4, false, true, false, WH, false, true, 0, 16, false, kLR>>(L);
    case 8: return launch_cfg<T, I, Cfg<VEC, 8, U, 4, false, true, false, WH, false, true, 0, 16, false, kLR>>(L);
    case 16: return launch_cfg<T, I, Cfg<VEC, 16, U, 4, false, true, false, WH, false, true, 0, 16, false, kLR>>(L);
    case 32: return launch_cfg<T, I, Cfg<VEC, 32, U, 4, false, true, false, WH, false, true, 0, 16, false, kLR>>(L);
    case 64: return launch_cfg<T, I, Cfg<VEC, 64, U, 4, false, false, false, false, false, true, 0, 16, false, kLR>>(L);
    default: return fail(OFX_EINVAL, "spmm_csr: unsupported lanes-per-row %d", lpr);
  }
}

// Mid form (use_mid_form): block items first, then one lane-group per light row.  SR: the light
// rows run the small-launch configuration (U = 32 / 16 loads in flight, next batch prefetched)
// instead of the big-launch one (U = 8, 16 for one-element fp32 lanes).
template <typename T, typename I, int VEC, bool SR>
int launch_vec_mid(const Launch& L, int lpr) {
  constexpr int U = SR ? (VEC * sizeof(T) <= 4 ? 32 : 16) : (VEC == 1 && sizeof(T) == 4 ? 16 : 8);
  switch (lpr) {
    case 4: return launch_cfg<T, I, Cfg<VEC, 4, U, 4, false, SR, false, false, true, true, 0, 16, false, kLR>>(L);
    case 8: return launch_cfg<T, I, Cfg<VEC, 8, U, 4, false, SR, false, false, true, true, 0, 16, false, kLR>>(L);
    case 16: return launch_cfg<T, I, Cfg<VEC, 16, U, 4, false, SR, false, false, true, true, 0, 16, false, kLR>>(L);
    case 32: return launch_cfg<T, I, Cfg<VEC, 32, U, 4, false, SR, false, false, true, true, 0, 16, false, kLR>>(L);
    case 64: return launch_cfg<T, I, Cfg<VEC, 64, U, 4, false, SR, false, false, true, true, 0, 16, false, kLR>>(L);
    default: return fail(OFX_EINVAL, "spmm_csr: unsupported lanes-per-row %d", lpr);
  }
}

// B's byte offsets fit the buffer descriptor's 32 bits (BRows): row k (the zero row) included.
template <typename T>
bool buffer_rows_ok(const Launch& L) {
  return (unsigned __int128)(L.b_rows + 1) * (unsigned __int128)L.ldb * sizeof(T) <
         ((unsigned __int128)1 << 32);
}

// B of 4 GiB or more (papers-scale): the bandwidth configurations with global loads (BUF = false).
template <typename T, typename I, int VEC>
int launch_vec_global(const Launch& L, int lpr, bool nt) {
  switch (lpr) {
    case 4: return launch_cfg<T, I, Cfg<VEC, 4, 8, 4, false, false, false, false, false, false>>(L);
    case 8: return launch_cfg<T, I, Cfg<VEC, 8, 8, 4, false, false, false, false, false, false>>(L);
    case 16:
      if constexpr (VEC == 1 && sizeof(T) == 4)
        return launch_cfg<T, I, Cfg<1, 16, 16, 4, false, false, false, false, false, false>>(L);
      return launch_cfg<T, I, Cfg<VEC, 16, 8, 4, false, false, false, false, false, false>>(L);
    case 32:
      return nt ? launch_cfg<T, I, Cfg<VEC, 32, 8, 4, true, false, false, false, false, false>>(L)
                : launch_cfg<T, I, Cfg<VEC, 32, 8, 4, false, false, false, false, false, false>>(L);
    case 64:
      return nt ? launch_cfg<T, I, Cfg<VEC, 64, 8, 4, true, false, false, false, false, false>>(L)
                : launch_cfg<T, I, Cfg<VEC, 64, 8, 4, false, false, false, false, false, false>>(L);
    default: return fail(OFX_EINVAL, "spmm_csr: unsupported lanes-per-row %d", lpr);
  }
}

template <typename T, typename I, int VEC>
int launch_vec(const Launch& L, int lpr, bool nt) {
  const int v = L.sched.variant;
  if (!buffer_rows_ok<T>(L)) {
    OFX_REQUIRE(v == 0 || v == kForceBigVariant || v == kForceGlobalVariant || (v > 0 && v < 10000),
                OFX_EINVAL,
                "spmm_csr: variant %d needs B under 4 GiB (k=%lld, ldb=%lld)", v,
                (long long)L.b_rows, (long long)L.ldb);
    return launch_vec_global<T, I, VEC>(L, lpr, nt);
  }
  if (v == kForceSmallVariant || (v == 0 && use_small_form(L.nrows, L.nnz_est, L.n, L.sched)))
    return launch_vec_small<T, I, VEC>(L, lpr);
  if (v == kForceMidSmallVariant) return launch_vec_mid<T, I, VEC, true>(L, lpr);
  if (v == kForceMidVariant) return launch_vec_mid<T, I, VEC, false>(L, lpr);
  if (v == kForceWaveVariant) return launch_vec_pf<T, I, VEC, true>(L, lpr);
  if (v == kForcePrefetchVariant) return launch_vec_pf<T, I, VEC, false>(L, lpr);
  if (v == kForceGlobalVariant) return launch_vec_global<T, I, VEC>(L, lpr, nt);
  // light rows of the mid form: the prefetching small-launch configuration above N = 16 (5-12%
  // faster at N = 64 / 128 on 20k-170k-row power-law graphs), the big-launch one at N <= 16
  // (profiles/r02n_probe_mid.json)
  if (v == 0 && use_mid_form(L.nrows, L.nnz_est, L.n, L.sched)) {
    return L.n > 16 ? launch_vec_mid<T, I, VEC, true>(L, lpr) : launch_vec_mid<T, I, VEC, false>(L, lpr);
  }
  // prefetching form: wave items at 16 < N <= 64 only (profiles/r03d_probe_forms.jsonl: at N = 16
  // they cost more than they save, arxiv-shaped 206 against 96 us; at N = 32 / 64 they win or tie,
  // 100 / 124 against 155 / 135 us; at N = 128 the form without them is 4-8% faster)
  if (v == 0 && use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched))
    return (L.n > 16 && L.n <= 64) ? launch_vec_pf<T, I, VEC, true>(L, lpr)
                                   : launch_vec_pf<T, I, VEC, false>(L, lpr);
  // the bandwidth configuration (forced variants keep it at every size)
#ifdef OFX_AB_GLOBAL_LOADS  // A/B builds only (probes/ab_build.sh): global loads, not buffer loads
  return launch_vec_global<T, I, VEC>(L, lpr, nt);
#endif
  switch (lpr) {
    case 4: return launch_cfg<T, I, Cfg<VEC, 4>>(L);
    case 8: return launch_cfg<T, I, Cfg<VEC, 8>>(L);
    case 16:
      // fp32 rows of <= 64 B (one element per lane): 16 loads in flight instead of 8, -1.2% on
      // products-shaped N = 16 (tuning variant 10021, profiles/r02_ab_n16_bnt.log), same bits
      if constexpr (VEC == 1 && sizeof(T) == 4) return launch_cfg<T, I, Cfg<1, 16, 16>>(L);
      return launch_cfg<T, I, Cfg<VEC, 16>>(L);
    case 32:
      return nt ? launch_cfg<T, I, Cfg<VEC, 32, 8, 4, true>>(L) : launch_cfg<T, I, Cfg<VEC, 32>>(L);
    case 64:
      return nt ? launch_cfg<T, I, Cfg<VEC, 64, 8, 4, true>>(L) : launch_cfg<T, I, Cfg<VEC, 64>>(L);
    default: return fail(OFX_EINVAL, "spmm_csr: unsupported lanes-per-row %d", lpr);
  }
}

// fp32 rows whose width is not a multiple of 4 above N = 64 in the bandwidth configuration:
// 16-B lanes with the last window shifted (Cfg::SH) instead of one element per lane, which needs
// several 64-lane passes there: products N = 99 / 301 10.6 / 31.2 -> 8.5 / 25.2 ms.  At 17-63
// columns one pass of single elements is as fast or faster (N = 41 / 47 / 63: 4.6 / 5.0 / 6.1 ms
// against 4.8 / 5.2 / 6.2; such rows cost whole 128-B lines either way); profiles/r03ad_sweep.jsonl.
// Round 5: 16-bit rows whose width is not a multiple of 8 above N = 64 the same way (8-element
// windows at 2-B alignment, probes/unaligned_probe.hip) instead of one element per lane over 64
// lanes: 1M power-law bf16 N = 99 / 127 / 255 1,490 / 1,556 / 3,031 -> 917 / 1,040 / 1,799 us
// (tuning entries 10122 / 10123, gpurun_out/r05h_2_py.txt; N = 128 / 256: 853 / 1,489).
// And 16-bit rows of 17-63 columns (but 32) in the bandwidth form, where the N / 16-element
// lanes left them one element per lane over 32-64 lanes: 4-element windows over 8 lanes up to 31
// columns, 8-element windows over 8 lanes above (entries 10175 / 10177, gpurun_out/r05t_1_py.txt,
// 1M power-law bf16 N = 17 / 31 / 33 / 47 / 63: 521 / 551 / 823 / 841 / 862 -> 403 / 487 / 555 /
// 609 / 674 us; N = 32 / 64 369 / 465 keep their layouts).  fp32 there stays one element per
// lane: shifted windows moved it by -6..+3% on that graph and +4% on products (round 3).
template <typename T, typename I>
int launch_shift(const Launch& L, bool nt) {
  constexpr int V = 16 / (int)sizeof(T);
  if constexpr (sizeof(T) == 2) {
    if (L.n < 32)
      return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
  }
  const int lpr = pick_lpr(L.n, V);
  switch (lpr) {
    case 4: return launch_cfg<T, I, Cfg<V, 4, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
    case 8: return launch_cfg<T, I, Cfg<V, 8, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
    case 16: return launch_cfg<T, I, Cfg<V, 16, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
    case 32:
      return nt ? launch_cfg<T, I, Cfg<V, 32, 8, 4, true, false, false, false, false, true, 0, 16, true>>(L)
                : launch_cfg<T, I, Cfg<V, 32, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
    default:
      return nt ? launch_cfg<T, I, Cfg<V, 64, 8, 4, true, false, false, false, false, true, 0, 16, true>>(L)
                : launch_cfg<T, I, Cfg<V, 64, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L);
  }
}

// The prefetching form's (mid-size graphs) odd fp32 widths above 16: 16-B lanes with the shifted
// last window, U = 16 loads in flight and the next (col, val) batch prefetched, instead of one
// element per lane (N <= 64: up to 64 lanes, one row per wave).  Hubs added in the kernel (LR), as
// in the rest of the prefetching form.
// (Round 5: rows up to 128 / 256 columns take launch_mid_width_pf; this serves the wider ones,
// and 16-bit rows in 8-element windows the same way.)
template <typename T, typename I>
int launch_shift_pf(const Launch& L) {
  constexpr int V = 16 / (int)sizeof(T);
  switch (pick_lpr(L.n, V)) {
    case 4: return launch_cfg<T, I, Cfg<V, 4, 16, 4, false, true, false, false, false, true, 0, 16, true, kLR>>(L);
    case 8: return launch_cfg<T, I, Cfg<V, 8, 16, 4, false, true, false, false, false, true, 0, 16, true, kLR>>(L);
    case 16: return launch_cfg<T, I, Cfg<V, 16, 16, 4, false, true, false, false, false, true, 0, 16, true, kLR>>(L);
    case 32: return launch_cfg<T, I, Cfg<V, 32, 16, 4, false, true, false, false, false, true, 0, 16, true, kLR>>(L);
    default: return launch_cfg<T, I, Cfg<V, 64, 16, 4, false, false, false, false, false, true, 0, 16, true, kLR>>(L);
  }
}

bool use_shift_pf_form(const Launch& L, int elem_bytes) {
  const bool odd = (elem_bytes == 4 && L.n % 4 != 0) || (elem_bytes == 2 && L.n % 8 != 0);
  return L.sched.variant == 0 && (elem_bytes == 4 || elem_bytes == 2) && L.n > 16 && odd &&
         use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         ((uintptr_t)L.b % elem_bytes) == 0 && ((uintptr_t)L.c % elem_bytes) == 0;
}

bool use_shift_form(const Launch& L, int elem_bytes) {
  const bool odd = (elem_bytes == 4 && L.n > 64 && L.n % 4 != 0) ||
                   (elem_bytes == 2 && L.n > 64 && L.n % 8 != 0) ||
                   (elem_bytes == 2 && L.n > 16 && L.n < 64 && L.n != 32);
  return L.sched.variant == 0 && (elem_bytes == 4 || elem_bytes == 2) && odd &&
         !use_small_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         !use_mid_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         !use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         ((uintptr_t)L.b % elem_bytes) == 0 && ((uintptr_t)L.c % elem_bytes) == 0;
}

// Rows of 64 B in fp32 (N = 16) above the mid form: four lanes of float4 per light row (16 rows
// per wave, few registers, so many rows in flight: what bounds these launches) and the hub chunks
// and heavy rows as wave items in 16-lane one-element groups (HL), so a 512-nonzero chunk is not
// one 4-lane chain.  Up to kPrefetchNnz: U = 4 with 16 wave-item loads in flight per lane (arxiv-
// shaped 71 -> 46 us, 2M nonzeros 65 -> 56 us); past it 2-lane float2 groups of U = 8 with 8 (5M
// 111 -> 92 us, 1M power-law 406 -> 353 us, products 2,241 -> 2,184 us; a uniform-degree 20M graph
// 396 -> 402 us).  profiles/r03n_graph.jsonl.  Same bits: only who adds changes.
template <typename T, typename I>
int launch_narrow(const Launch& L) {
  // past kPrefetchNnz only (round 4's U = 8 in-kernel-reduce shape below it, entry 10082, gave
  // way to launch_mid_width_pf's LDS-exchanged wave items in round 5)
  return launch_cfg<T, I, Cfg<2, 8, 8, 4, false, true, false, true, false, true, 16, 8>>(L);
}

bool use_narrow_form(const Launch& L, int elem_bytes) {
  // up to kPrefetchNnz the mid-width shape (its LDS-exchanged wave items) is faster since round 5
  return L.sched.variant == 0 && elem_bytes == 4 && L.n == 16 && pick_vec(4, L, 0) == 4 &&
         !use_small_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         !use_mid_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         !use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched);
}

// Narrow rows of mid-size launches (round 4, launch_narrow_pf, removed in round 5): 16-bit rows
// of 8 or 16 columns and fp32 rows of 8 took four lanes per light row (8 B per lane) with 16-lane
// one-element wave items (entries 10050-10063, profiles/r04k_variants.jsonl); the LDS-exchanged
// wave items of launch_mid_width_pf below replaced it at every such width.

// Rows of 17-64 columns of mid-size launches (round 5): the narrow form's
// shape for every width -- shifted windows (Cfg::SH, any N; 2-B-aligned 8 / 16-B accesses are
// exact and as fast on gfx950, probes/unaligned_probe.hip) over 8 lanes, hubs added in the
// kernel -- with the wave items (hub chunks, heavy rows) in 32-lane groups, one column pass
// (the reference gather's word choice, gather_kernel_util.cu:69-104, falls to 2-B words at odd
// 16-bit widths; the shifted window keeps 8 / 16-B words at any width):
// 1-element lanes up to 32 columns, 2-element lanes up to 64 (Cfg::HV).  The wave items' column
// passes were what held these widths: the round-4 layouts ran 16-lane one-element wave items, two
// to four passes per chunk.  Tuning entries 10100 / 10110 / 10117 / 10112 (profiles/
// r05_width_sweep_midsize.jsonl), arxiv-shaped 169k x 1.17M: fp32 N = 17-32 77 -> 58 us, fp32
// 33-64 97-103 -> 79-82, bf16 17 / 24 94 / 84 -> 68 / 66, bf16 33-63 125-160 -> 81-82 and N = 64
// 94 -> 79; 60k x 1.5M fp32 N = 17 72 -> 55, bf16 N = 47 / 63 118 / -> 79.  Same bits: only who
// adds changes.
// The same shape either side (entries 10130-10142, gpurun_out/r05i_1_py.txt, arxiv-shaped):
// rows of 1-15 columns (8 and 16 keep the narrow forms when aligned) in 4-lane groups, one
// element per lane below 4 columns and shifted 4-element windows above, with 16-lane wave items
// -- fp32 N = 1 / 4 / 12 / 15 75 / 86 / 73 / 83 -> 45 / 46 / 47 / 49 us, bf16 100 / 105 / 83 / 92
// -> 47 / 48 / 50 / 50; rows of 65-128 columns in 8-element windows over 16 lanes with 4-element
// wave lanes -- fp32 N = 65 / 99 / 128 143 / 148 / 147 -> 110 / 113 / 114, bf16 N = 65 / 99 / 128
// 463 / 467 / 151 -> 111 / 112 / 109; and 16-bit rows of 129-256 columns, 8-element wave lanes
// with 8 in flight -- bf16 N = 129 / 200 / 255 / 256 656 / 166 / 857 / 164 -> 155 / 150 / 158 /
// 150.  fp32 rows above 128 columns keep their layouts (as fast: 173-210 us either way).
// Up to 64 columns the wave items exchange their products through LDS (Cfg::XL,
// accumulate_wave_xl): 8- / 16-lane groups of 2-4 elements, 32-64 nonzeros per round of B-row
// loads without the cross-lane moves that made narrow groups lose (entries 10183-10198,
// gpurun_out/r05aa_2_py.txt / r05z_2_py.txt, arxiv-shaped / 60k x 1.5M): fp32 N = 8 / 12 / 16
// 43 / 44 / 44 -> 38 / 39 / 39 us, fp32 17-32 56 -> 48, fp32 47 / 64 78 -> 73 / 72 (76 -> 70),
// bf16 17 / 24 57 -> 54 / 53, bf16 47 / 64 80 / 78 -> 71 / 65 (80 / 79 -> 77 / 74); and 16-bit
// rows of 4-16 columns, aligned 8 / 16 included (round 4's narrow shape, launch_narrow_pf, is
// gone; entries 10199-10202, gpurun_out/r05ae_1_py.txt): bf16 N = 4 / 8 / 12 / 16 44 / 46 / 47 /
// 47 -> 37 / 40 / 42 / 42 us (60k x 1.5M 45 -> 43); fp32 rows of 65-128 columns too, two
// 32-lane groups of 8 nonzeros (entry 10204, gpurun_out/r05ag_2_py.txt): N = 65 / 99 / 128 107 /
// 111 / 112 -> 101 / 106 / 107 us (60k x 1.5M 101 / 106 / 107 -> 97 / 103 / 105); 16-bit rows
// there gained nothing from it (-1..+3%) and keep the cross-lane groups.  Rows of 1-3 columns:
// 16 four-lane groups of 8 nonzeros, 128 nonzeros per round of B-row loads (entry 10207,
// gpurun_out/r05aj_2_py.txt): fp32 / bf16 N = 1-3 42-45 -> 29-31 us on both mid-size graphs.
template <typename T, typename I>
int launch_mid_width_pf(const Launch& L) {
  if (L.n < 4)
    return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, true, false, true, false, true, 4, 8, false, kLR, 1, true>>(L);
  if (L.n <= 16)
    return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, true, false, true, false, true, 8, 8, true, kLR, 2, true>>(L);
  if (L.n <= 32)
    return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, true, false, true, false, true, 8, 8, true, kLR, 4, true>>(L);
  if (L.n <= 64) {
    if constexpr (sizeof(T) == 2)
      return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, true, false, true, false, true, 16, 8, true, kLR, 4, true>>(L);
    else
      return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, true, false, true, false, true, 16, 8, true, kLR, 4, true>>(L);
  }
  if constexpr (sizeof(T) == 2) {
    if (L.n > 128)
      return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, true, false, true, false, true, 32, 8, true, kLR, 8>>(L);
    return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, true, false, true, false, true, 32, 16, true, kLR, 4>>(L);
  } else {
    return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, true, false, true, false, true, 32, 8, true, kLR, 4, true>>(L);
  }
}

bool use_mid_width_pf_form(const Launch& L, int elem_bytes) {
  const int64_t top = elem_bytes == 2 ? 256 : 128;
  return L.sched.variant == 0 && (elem_bytes == 2 || elem_bytes == 4) && L.n >= 1 && L.n <= top &&
         use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched) &&
         ((uintptr_t)L.b % elem_bytes) == 0 && ((uintptr_t)L.c % elem_bytes) == 0;
}


}  // namespace

template <typename T, typename I>
int launch_typed(const Launch& L) {
  const bool form = is_form_variant(L.sched.variant);  // auto configuration, forced form
  if (L.sched.variant >= 10000 && !form) {
    OFX_REQUIRE(buffer_rows_ok<T>(L), OFX_EINVAL,
                "spmm_csr: tuning variant %d needs B under 4 GiB", L.sched.variant);
    return launch_tuned<T, I>(L, L.sched.variant - 10000);
  }
  // the narrow form (fp32 N = 16 past kPrefetchNnz), then every width of a mid-size launch up
  // to 128 (fp32) / 256 (16-bit) columns
  if constexpr (sizeof(T) == 4) {
    if (use_narrow_form(L, (int)sizeof(T)) && buffer_rows_ok<T>(L)) return launch_narrow<T, I>(L);
  }
  if constexpr (sizeof(T) == 2 || sizeof(T) == 4) {
    if (use_mid_width_pf_form(L, (int)sizeof(T)) && buffer_rows_ok<T>(L))
      return launch_mid_width_pf<T, I>(L);
    if (use_shift_form(L, (int)sizeof(T)) && buffer_rows_ok<T>(L))
      return launch_shift<T, I>(L, (L.b_rows * L.ldb * (int64_t)sizeof(T)) > kNtBytes);
  }
  if constexpr (sizeof(T) == 2 || sizeof(T) == 4) {
#ifndef OFX_AB_NO_SHIFT_PF  // A/B builds only (probes/ab_build.sh)
    if (use_shift_pf_form(L, (int)sizeof(T)) && buffer_rows_ok<T>(L)) return launch_shift_pf<T, I>(L);
#endif
  }
  // variant = VEC * 100 + LPR forces a configuration (tuning / tests); 0 = auto.
  const int forced_vec = (L.sched.variant > 0 && !form) ? L.sched.variant / 100 : 0;
  const int forced_lpr = (L.sched.variant > 0 && !form) ? L.sched.variant % 100 : 0;
  // fp32 rows of <= 64 B outside the narrow form (the small / mid forms, N < 16, forced forms):
  // one element per lane over 16 lanes (+9% against 4 lanes of float4 in the round-2 bandwidth
  // configuration, scripts/ab.py); wider rows keep the widest vector
  // 16-bit rows of at most 128 B (N <= 64) in the bandwidth configuration: at least 16 lanes per
  // row (VEC = N / 16: 2-8 B per lane) instead of the widest vector over 4-8 lanes; products bf16
  // N = 8 / 16 / 32 / 64 -8 / -7 / -6 / -13%, Reddit-shaped N = 16 / 32 / 64 -27 / -19 / -6%
  // (profiles/r03y_lanes_*.jsonl; fp32 keeps its layouts, DESIGN.md §3 tuning record)
  // The prefetching form too (mid-size graphs): arxiv-shaped bf16 N = 16 took 214 us with 8-element
  // lanes (two active lanes per 4-lane group) against 49 us for fp32 (profiles/r03ah_*.jsonl).
  // The small and mid forms too (round 4, profiles/r04y_small16.jsonl, interleaved A/B): PubMed-
  // shaped bf16 / f16 N = 8-32 33 -> 23 us, N = 64 36 -> 29; 20k rows x 400k N = 8-64 -4..-30%;
  // Cora-shaped (host-bound) -1..-8%.
  const bool narrow16 = !forced_vec && sizeof(T) == 2 && L.n <= 64 && L.sched.variant == 0;
  int cap16 = 1;  // the largest power of two <= N / 16
  while (cap16 * 32 <= L.n) cap16 *= 2;
  const int vec = (!forced_vec && sizeof(T) == 4 && L.n <= 16) ? 1
                  : narrow16 ? pick_vec((int)sizeof(T), L, 0, cap16)
                             : pick_vec((int)sizeof(T), L, forced_vec);
  OFX_REQUIRE(vec > 0, OFX_EINVAL,
              "spmm_csr: variant %d not applicable (n=%lld ldb=%lld ldc=%lld or pointer alignment)",
              L.sched.variant, (long long)L.n, (long long)L.ldb, (long long)L.ldc);
  int lpr = forced_lpr ? forced_lpr : pick_lpr(L.n, vec);
  // rows of fewer than 8 single-element lanes in the bandwidth configuration: 8-lane groups (idle
  // lanes included), not 4-lane ones; fp32 N = 1 / 2 / 3 / 4 on products -11 / -9 / -8 / -9%, on
  // the 1M power-law graph N = 1 / 4 -10 / -22%.  16 lanes won on products at N = 2-8 by 2-8% but
  // lost on the power-law graph by 4-48% (profiles/r03af_sweep.jsonl)
  if (!forced_lpr && vec == 1 && lpr < 8 && L.sched.variant == 0 &&
      !use_small_form(L.nrows, L.nnz_est, L.n, L.sched) &&
      !use_mid_form(L.nrows, L.nnz_est, L.n, L.sched) &&
      !use_prefetch_form(L.nrows, L.nnz_est, L.n, L.sched))
    lpr = 8;
  const bool nt = (L.b_rows * L.ldb * (int64_t)sizeof(T)) > kNtBytes;
  switch (vec) {
    case 1: return launch_vec<T, I, 1>(L, lpr, nt);
    case 2: return launch_vec<T, I, 2>(L, lpr, nt);
    case 4:
      if constexpr (sizeof(T) <= 4) return launch_vec<T, I, 4>(L, lpr, nt);
      break;
    case 8:
      if constexpr (sizeof(T) == 2) return launch_vec<T, I, 8>(L, lpr, nt);
      break;
  }
  return fail(OFX_EINVAL, "spmm_csr: unsupported vector width %d", vec);
}

}  // namespace ofx

#define OFX_SPMM_INSTANTIATE(T, I) template int ofx::launch_typed<T, I>(const ofx::Launch& L);

#endif  // OFX_SPMM_CSR_IMPL_H_
