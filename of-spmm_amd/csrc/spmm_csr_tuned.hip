// spmm_csr_tuned.hip — the tuning table of the SpMM forward (variant = 10000 + id): forced
// configurations for A/B runs (scripts/ab.py) and the tuning-table parity tests.
//
// No automatic rule launches through this table (the rules in spmm_csr_impl.h call launch_cfg
// directly), so the release library is built without it: only
// `make -C of-spmm_amd tuning` compiles it (-DOFX_TUNING_TABLE, oneflow_spmm/libofx_spmm_tuning.so,
// selected with OFX_SPMM_LIB), and ofx_version() then ends in "+tuning".  The tuning-table
// tests skip on a library without it.
#pragma clang fp contract(off)

#include "spmm_csr_impl.h"

namespace ofx {

#ifndef OFX_TUNING_TABLE
template <typename T, typename I>
int launch_tuned(const Launch& L, int) {
  return fail(OFX_EUNSUPPORTED,
              "spmm_csr: tuning variant %d: this library was built without the tuning table "
              "(make -C of-spmm_amd tuning; OFX_SPMM_LIB=.../libofx_spmm_tuning.so)",
              L.sched.variant);
}
#else
// Tuning table (variant = 10000 + id), float values / int32 indices only; every entry computes the
// same bits (the accumulation order does not depend on the launch shape).
template <typename T, typename I>
int launch_tuned(const Launch& L, int id) {
  // rows of VEC-element lanes: n, the strides and both pointers a multiple of VEC elements
  auto rows_of = [&](int vec) {
    const uintptr_t a = (uintptr_t)vec * sizeof(T);
    return L.n % vec == 0 && L.ldb % vec == 0 && L.ldc % vec == 0 && ((uintptr_t)L.b % a) == 0 &&
           ((uintptr_t)L.c % a) == 0;
  };
  // Round 4: narrow rows of mid-size launches (the prefetching form's share of the narrow form:
  // VEC x LPR light-row layouts with HL-lane one-element wave items, hubs added in the kernel).
  // 16-bit N = 16 / 8 and fp32 N = 8 (profiles/r04i_sweep.jsonl: 73-98 us against fp32 N = 16's
  // 47 us in the narrow form on the arxiv-shaped graph).
  if constexpr (sizeof(T) == 2 && std::is_same<I, int32_t>::value) {
    constexpr bool P = true, W = true;
    switch (id) {
      case 50: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 51: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 52: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 8, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 53: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 8, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 54: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, P, false, W, false, true, 16, 8, false, kLR>>(L); break;
      case 55: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 4, 4, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L); break;
      case 56: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 4, 8, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L); break;
      case 57: return launch_cfg<T, I, Cfg<1, 8, 8, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L);
      case 58: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, false, false, true, 0, 16, false, kLR>>(L); break;
      case 59: if (rows_of(8)) return launch_cfg<T, I, Cfg<8, 4, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      // odd 16-bit widths (no vector layout): one element per lane in 16 / 32-lane groups with
      // several column passes, instead of one 64-lane row per wave
      case 64: return launch_cfg<T, I, Cfg<1, 16, 32, 4, false, P, false, W, false, true, 0, 16, false, kLR>>(L);
      case 65: return launch_cfg<T, I, Cfg<1, 32, 32, 4, false, P, false, W, false, true, 0, 16, false, kLR>>(L);
      case 66: return launch_cfg<T, I, Cfg<1, 16, 32, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L);
      case 67: return launch_cfg<T, I, Cfg<1, 16, 16, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L);
      case 68: return launch_cfg<T, I, Cfg<1, 32, 16, 4, false, P, false, W, false, true, 32, 16, false, kLR>>(L);
      // 16-bit rows of 24-32 columns (round 4: bf16 N = 32 took 220 us on the arxiv-shaped graph,
      // the 2-element lanes' wave items unrolled to 259 VGPRs): 8 / 16-B lanes with 16-lane
      // one-element wave items
      case 73: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 74: if (rows_of(8)) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 75: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 8, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 76: if (rows_of(8)) return launch_cfg<T, I, Cfg<8, 4, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 77: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 16, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      // 16-bit rows of 33-64 columns: 16 / 8-B lanes with 16-lane wave items
      case 78: if (rows_of(8)) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 79: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      default: break;
    }
  }
  if constexpr (std::is_same<T, float>::value && std::is_same<I, int32_t>::value) {
    constexpr bool P = true, W = true;
    switch (id) {
      case 60: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 4, 4, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L); break;
      case 61: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 4, 8, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L); break;
      case 62: return launch_cfg<T, I, Cfg<1, 8, 8, 4, false, P, false, W, false, true, 8, 16, false, kLR>>(L);
      case 63: if (rows_of(2)) return launch_cfg<T, I, Cfg<2, 4, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      // fp32 N = 17-32 of mid-size launches (round 4: N = 17 took 113 us against 49 at N = 16 in
      // the shifted-window prefetching configuration): one-element 16 / 32-lane groups with column
      // passes, and the shifted window with 16-lane wave items
      case 69: return launch_cfg<T, I, Cfg<1, 16, 16, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L);
      case 70: return launch_cfg<T, I, Cfg<1, 32, 16, 4, false, P, false, W, false, true, 32, 16, false, kLR>>(L);
      case 71: if (((uintptr_t)L.b % 4) == 0 && ((uintptr_t)L.c % 4) == 0 && L.n >= 4)
                 return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L);
               break;
      case 72: if (((uintptr_t)L.b % 4) == 0 && ((uintptr_t)L.c % 4) == 0 && L.n >= 4)
                 return launch_cfg<T, I, Cfg<4, 8, 4, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L);
               break;
      // fp32 rows of 33-64 columns: 16-B lanes with 16-lane wave items
      case 80: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 81: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 16, 4, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      // fp32 N = 16 narrow form of mid-size launches with the in-kernel reduce (the automatic
      // pick is U = 4, HU = 16): U = 8, HU = 8 / 32
      case 82: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L); break;
      case 83: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, P, false, W, false, true, 16, 8, false, kLR>>(L); break;
      case 84: if (rows_of(4)) return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, P, false, W, false, true, 16, 32, false, kLR>>(L); break;
      // round 5: 8-element (32-B) lanes with the shifted window, so that rows of 17-32 columns
      // take 4 lanes (16 rows per wave, the N = 16 narrow form's packing) and rows of 33-64 take 8
      case 90: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 91: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 4, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 92: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 93: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 4, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 94: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 16, 8, true, kLR>>(L); break;
      // the wave items (hub chunks, heavy rows) in 32-lane groups: one column pass at N <= 32
      case 100: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      case 101: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      case 102: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR>>(L); break;
      case 103: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 32, 32, true, kLR>>(L); break;
      case 104: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 4, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      // rows of 33-64 columns: 32-lane wave items of 2-element (8-B) lanes, one pass
      case 117: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      case 118: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      case 119: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 4, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      // the same shape either side of 17-64 columns: 65-128 (4-element wave lanes), 129-256
      // (8-element, 32-B wave lanes), and 1-15 columns (16-lane one-element wave items)
      case 126: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 32, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4>>(L); break;
      case 127: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 32, 4, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4>>(L); break;
      case 128: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4>>(L); break;
      case 129: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 8>>(L); break;
      case 130: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 131: return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L);
      case 132: if (L.n >= 2) return launch_cfg<T, I, Cfg<2, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 139: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR, 8>>(L); break;
      case 141: return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 4, 16, false, kLR>>(L);
      // wave items in more, narrower groups (more nonzeros per batch: fewer dependent B-load
      // rounds per 512-nonzero hub chunk): light rows of the round-5 rule, wave HL x HV, HU
      case 143: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 2>>(L); break;
      case 144: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 16, true, kLR, 4>>(L); break;
      case 145: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 4>>(L); break;
      case 146: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 32, true, kLR, 2>>(L); break;
      case 147: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 4>>(L); break;
      case 148: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 8>>(L); break;
      case 149: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 8>>(L); break;
      case 150: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 4, 16, true, kLR, 4>>(L); break;
      case 151: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 8, 16, true, kLR, 2>>(L); break;
      // the bandwidth form (above kPrefetchNnz) at widths between the multiples of 16: shifted
      // windows (170-172), and the wave-item shape without the in-kernel reduce (173, 174)
      case 170: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 171: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 172: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 173: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 32, 8, true>>(L); break;
      case 174: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 32, 8, true, false, 2>>(L); break;
      case 180: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 8, true>>(L); break;
      // wave items with the products exchanged through LDS (Cfg::XL): narrow groups, many
      // nonzeros per round of B-row loads
      case 183: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 4, true>>(L); break;
      case 184: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 16, true, kLR, 4, true>>(L); break;
      case 185: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 4, 16, true, kLR, 4, true>>(L); break;
      case 186: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 8, true>>(L); break;
      case 187: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 4, true>>(L); break;
      case 191: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 2, true>>(L); break;
      case 192: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 8, 4, true, kLR, 8, true>>(L); break;
      case 193: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 8, true, kLR, 4, true>>(L); break;
      case 196: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 4, true, kLR, 4, true>>(L); break;
      case 197: if (L.n >= 2) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 2, true>>(L); break;
      // 65-128 columns: LDS-exchanged wave items (203-205)
      case 203: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 16, 8, true, kLR, 8, true>>(L); break;
      case 204: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR, 4, true>>(L); break;
      case 205: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4, true>>(L); break;
      // 1-3 columns: LDS-exchanged one-element wave items (206-207)
      case 206: if (L.n >= 1) return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 8, 8, false, kLR, 1, true>>(L); break;
      case 207: if (L.n >= 1) return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 4, 8, false, kLR, 1, true>>(L); break;
      // 4-32 columns: 16 four-lane LDS-exchanged groups (208-209)
      case 208: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 4, 8, true, kLR, 2, true>>(L); break;
      case 209: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 4, 8, true, kLR, 4, true>>(L); break;
      default: break;
    }
  }
  // round 5: 16-bit rows of odd widths with the shifted window (windows at 2-B alignment:
  // probes/unaligned_probe.hip) -- 4- and 8-element lanes over 4-16 lanes
  if constexpr (sizeof(T) == 2 && std::is_same<I, int32_t>::value) {
    constexpr bool P = true, W = true;
    switch (id) {
      case 95: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 96: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 97: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 98: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 99: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 16, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      // the prefetching form's layout without wave items (the N = 64 automatic one), shifted
      case 105: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 16, 4, false, P, false, false, false, true, 0, 16, true, kLR>>(L); break;
      case 106: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 16, 4, false, P, false, false, false, true, 0, 16, true, kLR>>(L); break;
      case 107: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 16, 4, false, P, false, false, false, true, 0, 16, true, kLR>>(L); break;
      // 32-lane wave items
      case 108: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      case 109: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      case 110: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      case 111: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR>>(L); break;
      // 32-lane wave items of 2-element (4-B) lanes: one pass up to 64 columns
      case 112: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      case 113: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      case 114: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR, 2>>(L); break;
      case 115: if (L.n >= 8) return launch_cfg<T, I, Cfg<4, 16, 16, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      case 116: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 4, 4, false, P, false, W, false, true, 32, 16, true, kLR, 2>>(L); break;
      // 16-bit rows of more than 64 columns, any width: shifted 16-B windows (the fp32 shifted
      // configurations' shape), prefetching (120, 121, 125) and bandwidth (122-124) forms
      case 120: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 16, 4, false, P, false, false, false, true, 0, 16, true, kLR>>(L); break;
      case 121: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 16, 4, false, P, false, false, false, true, 0, 16, true, kLR>>(L); break;
      case 122: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 123: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 124: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 64, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 125: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4>>(L); break;
      case 134: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 8>>(L); break;
      case 135: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 136: return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 16, 16, false, kLR>>(L);
      case 137: if (L.n >= 2) return launch_cfg<T, I, Cfg<2, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR>>(L); break;
      case 138: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 4, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4>>(L); break;
      case 140: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 32, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR, 8>>(L); break;
      case 142: return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 4, 16, false, kLR>>(L);
      case 152: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 4>>(L); break;
      case 153: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 8, 16, true, kLR, 8>>(L); break;
      case 154: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 8>>(L); break;
      case 155: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 16, true, kLR, 4>>(L); break;
      case 156: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 2>>(L); break;
      case 157: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 8>>(L); break;
      case 175: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 176: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 4, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 177: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 178: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 32, 8, true, false, 2>>(L); break;
      case 179: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, false, false, false, false, true, 0, 16, true>>(L); break;
      case 181: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 16, 8, true, false, 2>>(L); break;
      case 182: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 8, true>>(L); break;
      case 188: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 4, true>>(L); break;
      case 189: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 8, true>>(L); break;
      case 190: if (L.n >= 4) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 4, true>>(L); break;
      case 194: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 8, 4, true, kLR, 8, true>>(L); break;
      case 195: if (L.n >= 4) return launch_cfg<T, I, Cfg<8, 8, 8, 4, false, P, false, W, false, true, 16, 8, true, kLR, 4, true>>(L); break;
      case 198: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 8, 4, true, kLR, 4, true>>(L); break;
      // 16-bit, 16 columns and fewer: narrow LDS-exchanged wave items (199-202)
      case 199: if (L.n >= 2) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 2, true>>(L); break;
      case 200: if (L.n >= 2) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 16, 16, true, kLR, 2, true>>(L); break;
      case 201: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 4, 16, true, kLR, 4, true>>(L); break;
      case 202: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 8, 8, true, kLR, 4, true>>(L); break;
      // 65-128 columns: LDS-exchanged wave items (203-205)
      case 203: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 16, 8, true, kLR, 8, true>>(L); break;
      case 204: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 8, true, kLR, 4, true>>(L); break;
      case 205: if (L.n >= 8) return launch_cfg<T, I, Cfg<8, 16, 8, 4, false, P, false, W, false, true, 32, 16, true, kLR, 4, true>>(L); break;
      // 1-3 columns: LDS-exchanged one-element wave items (206-207)
      case 206: if (L.n >= 1) return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 8, 8, false, kLR, 1, true>>(L); break;
      case 207: if (L.n >= 1) return launch_cfg<T, I, Cfg<1, 4, 8, 4, false, P, false, W, false, true, 4, 8, false, kLR, 1, true>>(L); break;
      // 4-32 columns: 16 four-lane LDS-exchanged groups (208-209)
      case 208: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, P, false, W, false, true, 4, 8, true, kLR, 2, true>>(L); break;
      case 209: if (L.n >= 4) return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, P, false, W, false, true, 4, 8, true, kLR, 4, true>>(L); break;
      default: break;
    }
  }
  if constexpr (std::is_same<T, float>::value && std::is_same<I, int32_t>::value) {
    OFX_REQUIRE(L.n % 4 == 0 && L.ldb % 4 == 0 && L.ldc % 4 == 0 && ((uintptr_t)L.b % 16) == 0 &&
                    ((uintptr_t)L.c % 16) == 0,
                OFX_EINVAL, "spmm_csr: tuning variant %d needs 16-B aligned rows", L.sched.variant);
    switch (id) {
      case 1: return launch_cfg<T, I, Cfg<4, 32, 8, 4, false>>(L);
      case 2: return launch_cfg<T, I, Cfg<4, 32, 8, 4, true>>(L);
      case 3: return launch_cfg<T, I, Cfg<4, 32, 8, 1, false>>(L);
      case 4: return launch_cfg<T, I, Cfg<4, 32, 16, 4, false>>(L);
      case 5: return launch_cfg<T, I, Cfg<4, 32, 4, 4, false>>(L);
      case 6: return launch_cfg<T, I, Cfg<4, 32, 8, 2, true>>(L);
      case 7: return launch_cfg<T, I, Cfg<4, 32, 8, 8, false>>(L);
      case 8: return launch_cfg<T, I, Cfg<4, 32, 16, 4, true>>(L);
      case 9: return launch_cfg<T, I, Cfg<4, 16, 8, 4, false>>(L);
      case 10: return launch_cfg<T, I, Cfg<4, 16, 8, 4, true>>(L);
      // prefetch + branch-free issue (the small-launch form) at products scale
      case 11: return launch_cfg<T, I, Cfg<4, 32, 8, 4, true, true>>(L);
      case 12: return launch_cfg<T, I, Cfg<4, 32, 16, 4, true, true>>(L);
      case 13: return launch_cfg<T, I, Cfg<4, 32, 32, 4, true, true>>(L);
      case 14: return launch_cfg<T, I, Cfg<4, 32, 8, 4, false, true>>(L);
      // small launches at N = 16 (VEC 1, 16 lanes per row): loads in flight per lane
      case 15: return launch_cfg<T, I, Cfg<1, 16, 32, 4, false, true>>(L);
      case 16: return launch_cfg<T, I, Cfg<1, 16, 64, 4, false, true>>(L);
      case 17: return launch_cfg<T, I, Cfg<1, 16, 128, 4, false, true>>(L);
      // B-row loads non-temporal (request size / cache-policy probe at N = 16 and N = 128)
      case 18: return launch_cfg<T, I, Cfg<1, 16, 8, 4, false, false, true>>(L);
      case 19: return launch_cfg<T, I, Cfg<1, 16, 8, 4, true, false, true>>(L);
      case 20: return launch_cfg<T, I, Cfg<4, 32, 8, 4, false, false, true>>(L);
      case 21: return launch_cfg<T, I, Cfg<1, 16, 16, 4, false, false>>(L);
      // small launches without / with the wave-item form (N = 16: VEC 1, N = 64: VEC 4)
      case 22: return launch_cfg<T, I, Cfg<1, 16, 32, 4, false, true>>(L);
      case 23: return launch_cfg<T, I, Cfg<1, 16, 32, 4, false, true, false, true>>(L);
      case 24: return launch_cfg<T, I, Cfg<4, 16, 16, 4, false, true>>(L);
      case 25: return launch_cfg<T, I, Cfg<4, 16, 16, 4, false, true, false, true>>(L);
      // mid-size launches at N = 16: four lanes of float4 per row (16 rows per wave) instead of
      // sixteen one-element lanes, with / without the prefetch and wave items
      case 26: return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, true>>(L);
      case 27: return launch_cfg<T, I, Cfg<4, 4, 16, 4, false, true>>(L);
      case 28: return launch_cfg<T, I, Cfg<2, 8, 8, 4, false, true>>(L);
      case 29: return launch_cfg<T, I, Cfg<4, 4, 16, 4, false, true, false, true>>(L);
      case 30: return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, true>>(L);
      // ... and with wave items in 16-lane one-element groups (HL = 16, HU loads in flight)
      case 31: return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, true, false, true, false, true, 16, 16>>(L);
      case 32: return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, true, false, true, false, true, 16, 16>>(L);
      case 33: return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, true, false, true, false, true, 16, 8>>(L);
      case 34: return launch_cfg<T, I, Cfg<2, 8, 8, 4, false, true, false, true, false, true, 16, 16>>(L);
      case 35: return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, false, false, true, false, true, 16, 16>>(L);
      case 36: return launch_cfg<T, I, Cfg<4, 4, 4, 4, false, true, false, true, false, true, 16, 32>>(L);
      case 37: return launch_cfg<T, I, Cfg<2, 8, 8, 4, false, true, false, true, false, true, 16, 8>>(L);
      case 38: return launch_cfg<T, I, Cfg<4, 4, 8, 4, false, true, false, true, false, true, 16, 8>>(L);
      // N = 32 / 64: float4 light rows in 8 / 16 lanes with HL wave items (16 or 32 lanes)
      case 39: return launch_cfg<T, I, Cfg<4, 8, 4, 4, false, true, false, true, false, true, 16, 16>>(L);
      case 40: return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, true, false, true, false, true, 32, 8>>(L);
      case 41: return launch_cfg<T, I, Cfg<4, 16, 4, 4, false, true, false, true, false, true, 16, 16>>(L);
      case 42: return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, true, false, true, false, true, 32, 8>>(L);
      case 43: return launch_cfg<T, I, Cfg<4, 8, 8, 4, false, true>>(L);
      case 44: return launch_cfg<T, I, Cfg<4, 16, 8, 4, false, true>>(L);
      default: break;
    }
  }
  return fail(OFX_EINVAL, "spmm_csr: unknown tuning variant %d for this dtype", L.sched.variant);
}
#endif  // OFX_TUNING_TABLE

#define OFX_TUNED(T, I) template int launch_tuned<T, I>(const Launch& L, int id);
OFX_TUNED(float, int32_t)
OFX_TUNED(float, int64_t)
OFX_TUNED(double, int32_t)
OFX_TUNED(double, int64_t)
OFX_TUNED(bf16, int32_t)
OFX_TUNED(bf16, int64_t)
OFX_TUNED(f16, int32_t)
OFX_TUNED(f16, int64_t)
#undef OFX_TUNED

}  // namespace ofx
