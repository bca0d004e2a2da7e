/*
 * spmm_oracle.c — CPU restatement of the reference's SpMM semantics.  TEST INFRASTRUCTURE ONLY:
 * imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker;
 * never linked into, or called by, the product (of-spmm_amd/).
 *
 * Parity status: the reference (OneFlow v0.8.1-dev) contains no SpMM and no test pinning one
 * (SURVEY.md §0, §8c).  Its two building blocks are pinned by the reference's own golden vectors
 * (the embedding test python/oneflow/test/modules/test_sparse.py:76-134: row gather and
 * index-order segment sum, embedding_kernel_util.cpp:48-88; tests/test_reference_fixtures.py),
 * whose sums are exact -> "parity partially pinned": the rounding order of longer sums rests on
 * the restatement below and the cross-checks against scipy.sparse and torch.sparse_csr in
 * tests/golden/make_golden.py:
 *
 *   gather     oneflow/user/kernels/gather_kernel_util.cpp:72-92
 *              out[i,:] = in[idx[i],:]   (CHECK_GE(idx, 0) -> error here; an index >= the table
 *              size gathers a zero-filled row, :84-89, so its nonzero adds val * 0.  The CUDA
 *              gather, gather_kernel_util.cu:36, zero-fills negative indices too: orc_* take
 *              `neg_zero` = 1 for that semantics, the device kernel's)
 *   multiply   elementwise val[i] * out[i,:]  (one fp rounding)
 *   segsum     oneflow/user/kernels/unsorted_segment_sum_kernel_util.cpp:29-45
 *              out zero-filled (Memset, unsorted_segment_sum_kernel.cpp:95-96), then for i in
 *              ascending order: to = to + from  (std::transform with std::plus<T>)
 *   split      BalancedSplitter::At, oneflow/core/common/balanced_splitter.cpp:20-40
 *
 * Composed over a CSR (segment id of nonzero j = its row): C[r,:] = sum_j val[j]*B[col[j],:],
 * accumulated from +0 in ascending j with a multiply rounding and an add rounding per term.
 * `split`/`chunk` reproduce the operator's documented hub-row schedule so the
 * device result can be checked bit-for-bit; split = INT64_MAX is the pure reference order.
 *
 * Build: `make -C oracle` (gcc, OpenMP) -> oracle/liboracle.so.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#pragma GCC optimize("no-fast-math")

/* balanced_splitter.cpp:20-40: first (total % parts) parts get one extra element. */
void orc_balanced_range(int64_t total, int64_t parts, int64_t idx, int64_t* lo, int64_t* hi) {
  const int64_t base = total / parts;
  const int64_t rem = total % parts;
  if (idx < rem) {
    *lo = (base + 1) * idx;
    *hi = *lo + base + 1;
  } else {
    *lo = (base + 1) * rem + base * (idx - rem);
    *hi = *lo + base;
  }
}

/* Rounding of an fp32 value to the 16-bit storage types, returned as fp32 (round to nearest
 * even).  The multiply of the reference composition stores its product in the tensor's dtype:
 * BinaryFunctor<kMul> is `static_cast<Dst>(src0 * src1)`
 * (oneflow/core/ep/common/primitive/binary_functor.h:46-51), so for bf16/f16 inputs each
 * product is rounded to 16 bits before the fp32 segment sum (unsorted_segment_sum_kernel.cpp:
 * 146-205) adds it.  The fp32 product of two 16-bit values is exact, so one rounding here is
 * the 16-bit product. */
enum { ORC_R_NONE = 0, ORC_R_BF16 = 1, ORC_R_F16 = 2 };

static float orc_round_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u)
    u = (u & 0xffff0000u) | 0x400000u; /* NaN: quiet, payload truncated */
  else
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
  memcpy(&f, &u, 4);
  return f;
}

static float orc_round_f16(float f) {
  if (isnan(f)) return f;
  const float a = fabsf(f);
  float r;
  if (a < 0x1p-14f) {
    r = nearbyintf(a * 0x1p24f) * 0x1p-24f; /* subnormal f16: multiples of 2^-24 */
  } else {
    uint32_t u;
    memcpy(&u, &a, 4);
    u = (u + 0xfffu + ((u >> 13) & 1u)) & ~0x1fffu; /* 11 significant bits */
    memcpy(&r, &u, 4);
    if (r > 65504.0f) r = INFINITY;
  }
  return copysignf(r, f);
}

static inline float orc_mul(float v, float b, int round16) {
  const float p = v * b;
  if (round16 == ORC_R_BF16) return orc_round_bf16(p);
  if (round16 == ORC_R_F16) return orc_round_f16(p);
  return p;
}

/* exported for the tests: rounding of n fp32 values (in place) as the multiply does */
void orc_round16(float* x, int64_t n, int round16) {
  for (int64_t i = 0; i < n; ++i) x[i] = orc_mul(x[i], 1.0f, round16);
}

/* The gathered row of column c: B's row, or the zero-filled row of an index outside [0, k). */
#define ORC_ROW(b, c, ldb, k, zero) (((uint64_t)(c) < (uint64_t)(k)) ? (b) + (c) * (ldb) : (zero))

/* One segment [j0, j1) of row sums, f32 mul-then-add, from +0 (gather -> mul -> segsum). */
static void seg_f32(const int64_t* col, const float* val, const float* b, int64_t ldb, int64_t k,
                    const float* zero, int64_t n, int64_t j0, int64_t j1, float* acc, int round16) {
  for (int64_t c = 0; c < n; ++c) acc[c] = 0.0f;
  if (round16 == ORC_R_NONE) { /* fp32: a branch-free loop the compiler vectorises over c */
    for (int64_t j = j0; j < j1; ++j) {
      const float* from = ORC_ROW(b, col[j], ldb, k, zero); /* gather */
      const float v = val[j];
      for (int64_t c = 0; c < n; ++c) {
        const float prod = v * from[c]; /* multiply (rounded; built -ffp-contract=off) */
        acc[c] = acc[c] + prod;         /* segment-sum */
      }
    }
    return;
  }
  if (round16 == ORC_R_BF16) { /* the same rounding as orc_round_bf16, written as a select */
    for (int64_t j = j0; j < j1; ++j) {
      const float* from = ORC_ROW(b, col[j], ldb, k, zero);
      const float v = val[j];
      for (int64_t c = 0; c < n; ++c) {
        const float p = v * from[c];
        uint32_t u;
        memcpy(&u, &p, 4);
        const uint32_t rne = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
        const uint32_t qnan = (u & 0xffff0000u) | 0x400000u;
        u = ((u & 0x7fffffffu) > 0x7f800000u) ? qnan : rne;
        float prod;
        memcpy(&prod, &u, 4);
        acc[c] = acc[c] + prod;
      }
    }
    return;
  }
  for (int64_t j = j0; j < j1; ++j) {
    const float* from = ORC_ROW(b, col[j], ldb, k, zero); /* gather */
    for (int64_t c = 0; c < n; ++c) {
      const float prod = orc_mul(val[j], from[c], round16); /* multiply, stored in T */
      acc[c] = acc[c] + prod;                                /* segment-sum */
    }
  }
}

static void seg_f64(const int64_t* col, const double* val, const double* b, int64_t ldb,
                    int64_t k, const double* zero, int64_t n, int64_t j0, int64_t j1, double* acc) {
  for (int64_t c = 0; c < n; ++c) acc[c] = 0.0;
  for (int64_t j = j0; j < j1; ++j) {
    const double* from = ORC_ROW(b, col[j], ldb, k, zero);
    for (int64_t c = 0; c < n; ++c) {
      const double prod = val[j] * from[c];
      acc[c] = acc[c] + prod;
    }
  }
}

/* C (rows [row_begin,row_end), written from C[0]) = A @ B in f32 with the given schedule.
 * Returns 0, or -1 on a negative column (the reference's CHECK_GE) unless neg_zero; a column
 * >= k gathers a zero row. */
int orc_spmm_f32(int64_t m, int64_t k, int64_t n, const int64_t* rp, const int64_t* col,
                 const float* val, const float* b, int64_t ldb, float* c, int64_t ldc,
                 int64_t row_begin, int64_t row_end, int64_t split, int64_t chunk,
                 int nthreads, int round16, int neg_zero) {
  (void)m;
  if (!neg_zero)
    for (int64_t j = rp[row_begin]; j < rp[row_end]; ++j)
      if (col[j] < 0) return -1;
  float* zero = (float*)calloc((size_t)(n > 0 ? n : 1), sizeof(float));
  if (!zero) return -2;
#pragma omp parallel num_threads(nthreads)
  {
    float* part = (float*)__builtin_alloca(sizeof(float) * (n > 0 ? n : 1));
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
      float* out = c + (r - row_begin) * ldc;
      const int64_t j0 = rp[r], j1 = rp[r + 1], len = j1 - j0;
      if (len <= split) {
        seg_f32(col, val, b, ldb, k, zero, n, j0, j1, out, round16);
      } else {
        const int64_t nc = len / chunk;
        for (int64_t x = 0; x < n; ++x) out[x] = 0.0f;
        for (int64_t q = 0; q < nc; ++q) {
          const int64_t a = j0 + q * chunk;
          const int64_t e = (q == nc - 1) ? j1 : a + chunk;
          seg_f32(col, val, b, ldb, k, zero, n, a, e, part, round16);
          for (int64_t x = 0; x < n; ++x) out[x] = out[x] + part[x];
        }
      }
    }
  }
  free(zero);
  return 0;
}

int orc_spmm_f64(int64_t m, int64_t k, int64_t n, const int64_t* rp, const int64_t* col,
                 const double* val, const double* b, int64_t ldb, double* c, int64_t ldc,
                 int64_t row_begin, int64_t row_end, int64_t split, int64_t chunk,
                 int nthreads, int neg_zero) {
  (void)m;
  if (!neg_zero)
    for (int64_t j = rp[row_begin]; j < rp[row_end]; ++j)
      if (col[j] < 0) return -1;
  double* zero = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  if (!zero) return -2;
#pragma omp parallel num_threads(nthreads)
  {
    double* part = (double*)__builtin_alloca(sizeof(double) * (n > 0 ? n : 1));
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
      double* out = c + (r - row_begin) * ldc;
      const int64_t j0 = rp[r], j1 = rp[r + 1], len = j1 - j0;
      if (len <= split) {
        seg_f64(col, val, b, ldb, k, zero, n, j0, j1, out);
      } else {
        const int64_t nc = len / chunk;
        for (int64_t x = 0; x < n; ++x) out[x] = 0.0;
        for (int64_t q = 0; q < nc; ++q) {
          const int64_t a = j0 + q * chunk;
          const int64_t e = (q == nc - 1) ? j1 : a + chunk;
          seg_f64(col, val, b, ldb, k, zero, n, a, e, part);
          for (int64_t x = 0; x < n; ++x) out[x] = out[x] + part[x];
        }
      }
    }
  }
  free(zero);
  return 0;
}

/* fp64 reference of an f32 problem (C64) and the |.|-sum bound sum_j |val_j|*|B_col_j,c|,
 * used by the tolerance check |C - C64| <= rtol * absum. */
void orc_spmm_f32_ref64(int64_t n, const int64_t* rp, const int64_t* col, const float* val,
                        const float* b, int64_t ldb, double* c64, double* absum,
                        int64_t row_begin, int64_t row_end, int nthreads, int64_t k) {
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
  for (int64_t r = row_begin; r < row_end; ++r) {
    double* o = c64 + (r - row_begin) * n;
    double* a = absum + (r - row_begin) * n;
    for (int64_t x = 0; x < n; ++x) o[x] = a[x] = 0.0;
    for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
      if ((uint64_t)col[j] >= (uint64_t)k) continue; /* a zero-filled row: adds (+-)0 */
      const float* from = b + col[j] * ldb;
      for (int64_t x = 0; x < n; ++x) {
        o[x] += (double)val[j] * (double)from[x];
        a[x] += fabs((double)val[j]) * fabs((double)from[x]);
      }
    }
  }
}

/* SDDMM (the values-gradient of C = A @ B): out[j] = <a[row(j) - row_begin, :], b[col[j], :]>
 * in the operator's documented order (of-spmm_amd/csrc/spmm_backward.hip header): products
 * rounded, 8-element leaves summed sequentially from +0, leaves zero-padded to a power of two
 * and added pairwise level by level.  No SDDMM exists in the reference; the order is ours. */
static int64_t pow2_at_least(int64_t x) {
  int64_t p = 1;
  while (p < x) p *= 2;
  return p;
}

void orc_sddmm_f32(int64_t n, const int64_t* rp, const int64_t* col, const float* a, int64_t lda,
                   const float* b, int64_t ldb, float* out, int64_t row_begin, int64_t row_end,
                   int nthreads, int64_t k) {
  const int64_t leaves = (n + 7) / 8, padded = pow2_at_least(leaves);
  float* zero = (float*)calloc((size_t)(n > 0 ? n : 1), sizeof(float));
  if (!zero) return;
#pragma omp parallel num_threads(nthreads)
  {
    float* leaf = (float*)__builtin_alloca(sizeof(float) * padded);
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
      const float* ar = a + (r - row_begin) * lda;
      for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
        const float* br = ORC_ROW(b, col[j], ldb, k, zero); /* the forward's gathered row */
        for (int64_t l = 0; l < padded; ++l) {
          float s = 0.0f;
          for (int64_t e = 8 * l; e < 8 * l + 8 && e < n; ++e) {
            const float p = ar[e] * br[e];
            s = s + p;
          }
          leaf[l] = s;
        }
        for (int64_t w = 1; w < padded; w *= 2)
          for (int64_t l = 0; l < padded; l += 2 * w) leaf[l] = leaf[l] + leaf[l + w];
        out[j] = leaf[0];
      }
    }
  }
  free(zero);
}

void orc_sddmm_f64(int64_t n, const int64_t* rp, const int64_t* col, const double* a, int64_t lda,
                   const double* b, int64_t ldb, double* out, int64_t row_begin, int64_t row_end,
                   int nthreads, int64_t k) {
  const int64_t leaves = (n + 7) / 8, padded = pow2_at_least(leaves);
  double* zero = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  if (!zero) return;
#pragma omp parallel num_threads(nthreads)
  {
    double* leaf = (double*)__builtin_alloca(sizeof(double) * padded);
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
      const double* ar = a + (r - row_begin) * lda;
      for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
        const double* br = ORC_ROW(b, col[j], ldb, k, zero);
        for (int64_t l = 0; l < padded; ++l) {
          double s = 0.0;
          for (int64_t e = 8 * l; e < 8 * l + 8 && e < n; ++e) {
            const double p = ar[e] * br[e];
            s = s + p;
          }
          leaf[l] = s;
        }
        for (int64_t w = 1; w < padded; w *= 2)
          for (int64_t l = 0; l < padded; l += 2 * w) leaf[l] = leaf[l] + leaf[l + w];
        out[j] = leaf[0];
      }
    }
  }
  free(zero);
}
