// synth.cpp — deterministic synthetic power-law CSR and dense inputs.
//
// The benchmark configs of BASELINE.json are dataset-*shaped* (Cora / ogbn-products / Reddit /
// papers100M); the datasets themselves are not available offline, so inputs are generated:
//   degrees   Chung–Lu weights w_i = (i+1)^(-1/(gamma-1)) over ranks, d_i = floor(nnz*w_i/W),
//             remainder +1 to the heaviest ranks (cap k), ranks mapped to rows by a seeded
//             Fisher–Yates permutation pi.
//   columns   per row, d stratified draws u_j = (j + U_j)/d of the column CDF (same weights,
//             same permutation when k == m), pushed forward to stay strictly increasing in rank
//             (so no duplicates), mapped through pi and sorted: canonical CSR.
//   values    U[-1,1) with 24 random bits (exact in fp32) from splitmix64(seed, j), or the
//             exact mode {+-1, +-2} / integers in [-8, 8] (all partial sums exact in fp32).
// Everything is a pure function of (shape, seed) — identical across thread counts and ranks.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "ofx_internal.h"
#include "spmm_common.h"

namespace ofx {
namespace {

std::vector<int64_t> permutation(int64_t m, uint64_t seed) {
  std::vector<int64_t> p(m);
  for (int64_t i = 0; i < m; ++i) p[i] = i;
  const uint64_t s = splitmix64(seed ^ 0x7065726d75746eull);
  for (int64_t i = m - 1; i > 0; --i) {
    const int64_t j = (int64_t)(hash2(s, (uint64_t)i) % (uint64_t)(i + 1));
    std::swap(p[i], p[j]);
  }
  return p;
}

double weight(int64_t rank, double gamma) { return std::pow((double)(rank + 1), -1.0 / (gamma - 1.0)); }

template <typename I>
void fill_columns(int64_t k, double gamma, uint64_t seed, const int64_t* rp, int64_t row_begin,
                  int64_t row_end, I* out, int nthreads) {
  std::vector<double> cdf(k);
  double acc = 0.0;
  for (int64_t c = 0; c < k; ++c) {
    acc += weight(c, gamma);
    cdf[c] = acc;
  }
  const double W = acc;
  // Bucket index over the CDF: bucket q covers targets [q*W/NB, (q+1)*W/NB); lo[q] = the first
  // rank whose cdf exceeds the bucket's lower edge, so a search starts at lo[q] and ends by
  // lo[q+1] + 1.  Same answer as a full binary search, O(1) expected steps on huge k.
  const int64_t NB = k < (1 << 22) ? (k > 0 ? k : 1) : (1 << 22);
  std::vector<int64_t> blo(NB + 1);
  for (int64_t q = 0, r = 0; q <= NB; ++q) {
    const double edge = (double)q / (double)NB * W;
    while (r < k && cdf[r] <= edge) ++r;
    blo[q] = r;
  }
  const std::vector<int64_t> perm = permutation(k, seed);
  const uint64_t cs = splitmix64(seed ^ 0x636f6c756d6e73ull);
  const int64_t base = rp[row_begin];
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<int64_t> tmp;
#pragma omp for schedule(dynamic, 256)
    for (int64_t r = row_begin; r < row_end; ++r) {
      const int64_t d = rp[r + 1] - rp[r];
      if (d == 0) continue;
      tmp.resize(d);
      const uint64_t rs = hash2(cs, (uint64_t)r);
      int64_t prev = -1;
      for (int64_t j = 0; j < d; ++j) {
        const double uj = (double)(hash2(rs, (uint64_t)j) >> 11) * (1.0 / 9007199254740992.0);
        const double target = ((double)j + uj) / (double)d * W;
        int64_t q = (int64_t)(target / W * (double)NB);
        if (q < 0) q = 0;
        if (q > NB - 1) q = NB - 1;
        // first rank with cdf > target: search the bucket (one rank of slack on each side for
        // edge rounding), fall back to the whole table if the bucket does not bracket it
        const int64_t lo = blo[q] > 0 ? blo[q] - 1 : 0;
        const int64_t hi = blo[q + 1] + 1 < k ? blo[q + 1] + 1 : k;
        int64_t rank = (int64_t)(std::upper_bound(cdf.begin() + lo, cdf.begin() + hi, target) -
                                 cdf.begin());
        if (!((rank == 0 || cdf[rank - 1] <= target) && (rank == k || cdf[rank] > target)))
          rank = (int64_t)(std::upper_bound(cdf.begin(), cdf.end(), target) - cdf.begin());
        if (rank > k - 1) rank = k - 1;
        if (rank < prev + 1) rank = prev + 1;
        if (rank > k - d + j) rank = k - d + j;
        prev = rank;
        tmp[j] = perm[rank];
      }
      std::sort(tmp.begin(), tmp.end());
      I* o = out + (rp[r] - base);
      for (int64_t j = 0; j < d; ++j) o[j] = (I)tmp[j];
    }
  }
}

template <typename T>
void fill_values(int64_t j_begin, int64_t j_end, uint64_t seed, int exact, T* out) {
#pragma omp parallel for schedule(static)
  for (int64_t j = j_begin; j < j_end; ++j) {
    const uint64_t h = hash2(seed, (uint64_t)j);
    const float f = exact ? exact_val(h) : u_pm1(h);
    out[j - j_begin] = Num<T>::store((typename Num<T>::acc)f);
  }
}

template <typename T>
void fill_dense(int64_t r_begin, int64_t r_end, int64_t n, int64_t ld, uint64_t seed, int exact,
                T* out) {
#pragma omp parallel for schedule(static)
  for (int64_t r = r_begin; r < r_end; ++r)
    for (int64_t c = 0; c < n; ++c) {
      const uint64_t h = hash2(seed, (uint64_t)(r * n + c));
      const float f = exact ? exact_dense(h) : u_pm1(h);
      out[(r - r_begin) * ld + c] = Num<T>::store((typename Num<T>::acc)f);
    }
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_synth_row_ptr(int64_t m, int64_t k, int64_t nnz, double gamma, uint64_t seed,
                                 int64_t* row_ptr_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(m >= 0 && k >= 0 && nnz >= 0 && row_ptr_out && gamma > 1.0, OFX_EINVAL,
                "synth_row_ptr: bad arguments");
    OFX_REQUIRE(m == 0 || (double)nnz <= (double)m * (double)k, OFX_EINVAL,
                "synth_row_ptr: nnz=%lld exceeds m*k", (long long)nnz);
    row_ptr_out[0] = 0;
    if (m == 0) return OFX_OK;
    std::vector<double> w(m);
    double W = 0.0;
    for (int64_t i = 0; i < m; ++i) {
      w[i] = weight(i, gamma);
      W += w[i];
    }
    std::vector<int64_t> d(m);
    int64_t total = 0;
    for (int64_t i = 0; i < m; ++i) {
      int64_t di = (int64_t)std::floor((double)nnz * w[i] / W);
      if (di > k) di = k;
      d[i] = di;
      total += di;
    }
    int64_t rem = nnz - total;
    while (rem > 0) {
      for (int64_t i = 0; i < m && rem > 0; ++i)
        if (d[i] < k) {
          ++d[i];
          --rem;
        }
    }
    while (rem < 0) {  // floor() never overshoots, kept for completeness
      for (int64_t i = m - 1; i >= 0 && rem < 0; --i)
        if (d[i] > 0) {
          --d[i];
          ++rem;
        }
    }
    const std::vector<int64_t> perm = permutation(m, seed);
    std::vector<int64_t> deg(m);
    for (int64_t i = 0; i < m; ++i) deg[perm[i]] = d[i];
    for (int64_t r = 0; r < m; ++r) row_ptr_out[r + 1] = row_ptr_out[r] + deg[r];
    return OFX_OK;
  });
}

extern "C" int ofx_synth_columns(int64_t m, int64_t k, double gamma, uint64_t seed,
                                 const int64_t* row_ptr, int64_t row_begin, int64_t row_end,
                                 int idx_dtype, void* col_out, int num_threads) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(row_ptr && 0 <= row_begin && row_begin <= row_end && row_end <= m && k >= 0,
                OFX_EINVAL, "synth_columns: bad arguments");
    OFX_REQUIRE(is_index_dtype(idx_dtype), OFX_EUNSUPPORTED, "synth_columns: bad index dtype");
    if (row_end == row_begin || row_ptr[row_end] == row_ptr[row_begin]) return OFX_OK;
    OFX_REQUIRE(col_out && k > 0, OFX_EINVAL, "synth_columns: NULL output or k == 0");
    const int nt = num_threads > 0 ? num_threads : omp_get_max_threads();
    if (idx_dtype == OFX_DT_INT32)
      fill_columns<int32_t>(k, gamma, seed, row_ptr, row_begin, row_end,
                            static_cast<int32_t*>(col_out), nt);
    else
      fill_columns<int64_t>(k, gamma, seed, row_ptr, row_begin, row_end,
                            static_cast<int64_t*>(col_out), nt);
    return OFX_OK;
  });
}

extern "C" int ofx_synth_values_host(int val_dtype, int64_t j_begin, int64_t j_end, uint64_t seed,
                                     int exact, void* out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(j_begin <= j_end && (out || j_begin == j_end), OFX_EINVAL,
                "synth_values_host: bad arguments");
    switch (val_dtype) {
      case OFX_DT_FLOAT: fill_values(j_begin, j_end, seed, exact, static_cast<float*>(out)); break;
      case OFX_DT_DOUBLE: fill_values(j_begin, j_end, seed, exact, static_cast<double*>(out)); break;
      case OFX_DT_BFLOAT16: fill_values(j_begin, j_end, seed, exact, static_cast<bf16*>(out)); break;
      case OFX_DT_FLOAT16: fill_values(j_begin, j_end, seed, exact, static_cast<f16*>(out)); break;
      default: return fail(OFX_EUNSUPPORTED, "synth_values_host: bad dtype %d", val_dtype);
    }
    return OFX_OK;
  });
}

extern "C" int ofx_synth_dense_host(int val_dtype, int64_t r_begin, int64_t r_end, int64_t n,
                                    int64_t ld, uint64_t seed, int exact, void* out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(r_begin <= r_end && ld >= n && n >= 0, OFX_EINVAL, "synth_dense_host: bad shape");
    switch (val_dtype) {
      case OFX_DT_FLOAT: fill_dense(r_begin, r_end, n, ld, seed, exact, static_cast<float*>(out)); break;
      case OFX_DT_DOUBLE: fill_dense(r_begin, r_end, n, ld, seed, exact, static_cast<double*>(out)); break;
      case OFX_DT_BFLOAT16: fill_dense(r_begin, r_end, n, ld, seed, exact, static_cast<bf16*>(out)); break;
      case OFX_DT_FLOAT16: fill_dense(r_begin, r_end, n, ld, seed, exact, static_cast<f16*>(out)); break;
      default: return fail(OFX_EUNSUPPORTED, "synth_dense_host: bad dtype %d", val_dtype);
    }
    return OFX_OK;
  });
}
