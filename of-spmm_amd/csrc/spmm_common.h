// spmm_common.h — numeric contract shared by the HIP kernels (spmm_csr.hip) and the CPU kernel
// (spmm_cpu.cpp): storage types, conversions, schedule (split) resolution, counter-based RNG.
//
// The accumulation contract restates the reference composition gather -> multiply ->
// unsorted_segment_sum (oneflow/user/kernels/gather_kernel_util.cpp:72-92,
// oneflow/user/kernels/unsorted_segment_sum_kernel_util.cpp:29-45: `out` zero-filled, then
// `to = to + from` per index in ascending order, i.e. one multiply rounding then one add
// rounding per nonzero; half/bf16 accumulate in fp32 as in
// oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:146-205).
#ifndef OFX_SPMM_COMMON_H_
#define OFX_SPMM_COMMON_H_

#include <stdint.h>
#include <string.h>

#include "ofx_spmm.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define OFX_HD __host__ __device__ __forceinline__
#else
#define OFX_HD static inline
#endif

namespace ofx {

// 16-bit storage types (bit containers; arithmetic always happens in fp32).
struct bf16 {
  uint16_t x;
};
struct f16 {
  uint16_t x;
};

OFX_HD float bits_to_f32(uint32_t u) { return __builtin_bit_cast(float, u); }
OFX_HD uint32_t f32_to_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

OFX_HD float bf16_to_f32(uint16_t h) { return bits_to_f32(uint32_t(h) << 16); }
// Round-to-nearest-even; NaN stays NaN (quiet bit forced).
// On the device this is gfx950's v_cvt_pk_bf16_f32 (emitted for the conversion to __bf16), which
// gives the same bits as the software rounding for all 2^32 f32 inputs, NaNs included
// (probes/bf16_cvt_probe.hip, profiles/r02_bf16_cvt_probe.json); the host (CPU kernel) keeps
// the software form.
OFX_HD uint16_t f32_to_bf16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(uint16_t, (__bf16)f);
#else
  const uint32_t u = f32_to_bits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return uint16_t((u >> 16) | 0x40u);
  return uint16_t((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
#endif
}
OFX_HD float f16_to_f32(uint16_t h) { return float(__builtin_bit_cast(_Float16, h)); }
OFX_HD uint16_t f32_to_f16(float f) { return __builtin_bit_cast(uint16_t, _Float16(f)); }

// bf16 rounding of an fp32 value, returned as fp32 (round-to-nearest-even, NaN quieted): the
// same bits as bf16_to_f32(f32_to_bf16(f)) without the 16-bit round trip.
// Device: one v_cvt_pk_bf16_f32 (per two values) and a shift instead of ~7 integer ops; the
// software form made the bf16 N=256 Reddit-shaped SpMM ALU-bound (7.2 -> 12.5 ms).
OFX_HD float round_bf16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (float)(__bf16)f;
#else
  const uint32_t u = f32_to_bits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return bits_to_f32((u & 0xffff0000u) | 0x400000u);
  return bits_to_f32((u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
#endif
}

// Accumulator type, load/store conversions and the multiply per storage type.
//
// mul(v, b) is the elementwise multiply of the reference composition, whose output tensor has
// the storage type T: BinaryFunctor<kMul> is `static_cast<Dst>(src0 * src1)`
// (oneflow/core/ep/common/primitive/binary_functor.h:46-51), i.e. the product is rounded to T
// before unsorted_segment_sum adds it.  For bf16/f16 the fp32 product of two 16-bit values is
// exact (8+8 / 11+11 significand bits), so rounding it once to T is the correctly rounded 16-bit
// product (for bf16, except where the product falls below fp32's normal range, ~1e-38, where
// the fp32 step can round first).  The fp32 sum of the rounded products is then
// rounded once at the end (unsorted_segment_sum_kernel.cpp:146-205).
template <typename T>
struct Num;
template <>
struct Num<float> {
  using acc = float;
  OFX_HD static float load(float v) { return v; }
  OFX_HD static float store(float a) { return a; }
  OFX_HD static float mul(float v, float b) { return v * b; }
};
template <>
struct Num<double> {
  using acc = double;
  OFX_HD static double load(double v) { return v; }
  OFX_HD static double store(double a) { return a; }
  OFX_HD static double mul(double v, double b) { return v * b; }
};
template <>
struct Num<bf16> {
  using acc = float;
  OFX_HD static float load(bf16 v) { return bf16_to_f32(v.x); }
  OFX_HD static bf16 store(float a) { return bf16{f32_to_bf16(a)}; }
  OFX_HD static float mul(float v, float b) { return round_bf16(v * b); }
};
template <>
struct Num<f16> {
  using acc = float;
  OFX_HD static float load(f16 v) { return f16_to_f32(v.x); }
  OFX_HD static f16 store(float a) { return f16{f32_to_f16(a)}; }
  OFX_HD static float mul(float v, float b) { return float(_Float16(v * b)); }
};

// Epilogue of the fused op (include/ofx_spmm.h ofx_spmm_csr_fused): the composition
// spmm_csr -> bias_add -> relu, each step rounding to T as the separate ops would
// (bias_add: oneflow/user/kernels/bias_add_kernel.cpp:25-53; relu:
// oneflow/core/ep/common/primitive/unary_functor.h:146-156, x <= 0 -> +0, NaN passes).
template <typename T>
OFX_HD T epilogue(typename Num<T>::acc acc, const T* bias, int64_t c, int act) {
  T y = Num<T>::store(acc);
  if (bias) y = Num<T>::store(Num<T>::load(y) + Num<T>::load(bias[c]));
  if (act == OFX_ACT_RELU && Num<T>::load(y) <= typename Num<T>::acc(0))
    y = Num<T>::store(typename Num<T>::acc(0));
  return y;
}

// The poison a launch with no valid work plan writes over its whole output:
// one canonical quiet NaN of T (f32 0x7fc00000, f64 0x7ff8000000000000, bf16 0x7fc0,
// f16 0x7e00), so no stale or uninitialised value can be read as a result.
template <typename T>
OFX_HD T poison_value() {
  return Num<T>::store(typename Num<T>::acc(__builtin_nan("")));
}

OFX_HD int dtype_size(int dt) {
  switch (dt) {
    case OFX_DT_FLOAT: return 4;
    case OFX_DT_DOUBLE: return 8;
    case OFX_DT_INT32: return 4;
    case OFX_DT_INT64: return 8;
    case OFX_DT_FLOAT16: return 2;
    case OFX_DT_BFLOAT16: return 2;
    default: return 0;
  }
}
OFX_HD bool is_index_dtype(int dt) { return dt == OFX_DT_INT32 || dt == OFX_DT_INT64; }
OFX_HD bool is_value_dtype(int dt) {
  return dt == OFX_DT_FLOAT || dt == OFX_DT_DOUBLE || dt == OFX_DT_FLOAT16 ||
         dt == OFX_DT_BFLOAT16;
}

// ---- schedule ---------------------------------------------------------------------------
// Default split threshold: rows with more than T nonzeros are cut into chunks of T, where
// T = clamp(65536 / n, 128, 512) rounded down to a power of two (T*n <= 64K multiply-adds
// per chunk).  This is a fixed function of n and part of the numeric contract.
// The 512 cap (round 3; was 8192) bounds a chunk's in-order chain at every width: at N = 16 a
// 4096-8191-nonzero chunk was one lane-group's chain of 256-512 dependent load rounds, which
// set the time of power-law launches of modest size (1M rows at N = 16 ran slower than N = 64).
// N >= 128 keeps its threshold (512 at N = 128, 256 at N = 256).
OFX_HD int64_t default_split(int64_t n) {
  int64_t t = n > 0 ? (int64_t)65536 / n : 512;
  if (t < 128) t = 128;
  if (t > 512) t = 512;
  int64_t p = 128;
  while (p * 2 <= t) p *= 2;
  return p;
}

struct Schedule {
  int64_t split;  // rows with len > split are chunked; INT64_MAX = never
  int64_t chunk;  // chunk length (the last chunk of a row takes the remainder: [chunk, 2*chunk))
  int64_t heavy;  // degree-bin threshold for the device work order (no numeric effect);
                  // 0 = auto, INT64_MAX = off
  int32_t variant;
  int32_t planned;  // the workspace holds this launch's plan (ofx_spmm_csr_plan): skip planning
  int32_t force_bin;  // plan a binned work list even for few rows (the mid form's block items)
};

static inline Schedule resolve_schedule(int64_t n, const ofx_spmm_options* o) {
  Schedule s;
  s.variant = o ? o->variant : 0;
  s.planned = o ? o->planned : 0;
  s.force_bin = 0;
  const int64_t h = o ? o->heavy_threshold : 0;
  s.heavy = h > 0 ? h : (h < 0 ? INT64_MAX : 0);  // 0 = auto (device launch: 5x mean degree)
  if (o && o->ordered) {
    s.split = INT64_MAX;
    s.chunk = INT64_MAX;
    return s;
  }
  s.split = (o && o->split_threshold > 0) ? o->split_threshold : default_split(n);
  s.chunk = (o && o->chunk > 0) ? o->chunk : s.split;
  if (s.chunk > s.split) s.chunk = s.split;  // every split row then has >= 1 full chunk
  return s;
}

// The automatic heavy-bin threshold of the device work order (no numeric effect): 5x the mean
// degree of the launch's rows, at least 16 (products and the 1M power-law config both peak at
// 4-6x the mean).
OFX_HD int64_t auto_heavy(int64_t nrows, int64_t nnz) {
  const int64_t mean = nrows > 0 ? (nnz + nrows - 1) / nrows : 1;
  return 5 * mean < 16 ? 16 : 5 * mean;
}

// Number of chunks of a split row of length len (> split): floor(len / chunk) — the last
// chunk absorbs the remainder, so chunk k covers [k*chunk, (k+1)*chunk) for k < nc-1 and
// [(nc-1)*chunk, len) for the last one.
OFX_HD int64_t num_chunks(int64_t len, int64_t chunk) { return len / chunk; }

// ---- counter-based RNG (synthetic inputs; identical on host and device) -----------------
OFX_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
OFX_HD uint64_t hash2(uint64_t seed, uint64_t i) { return splitmix64(splitmix64(seed) ^ i); }
// U[-1, 1) with 24 random bits: exactly representable in fp32.
OFX_HD float u_pm1(uint64_t h) { return float((int64_t)(h >> 40) - (1 << 23)) * (1.0f / (1 << 23)); }
// exact-mode draws: values in {-2,-1,1,2}, dense in integers [-8, 8].
OFX_HD float exact_val(uint64_t h) {
  const float t[4] = {-2.f, -1.f, 1.f, 2.f};
  return t[(h >> 33) & 3];
}
OFX_HD float exact_dense(uint64_t h) { return float((int)((h >> 33) % 17) - 8); }

}  // namespace ofx

#endif  // OFX_SPMM_COMMON_H_
