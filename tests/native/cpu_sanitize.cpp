// cpu_sanitize.cpp — the host-side kernels (csrc/spmm_cpu.cpp, csrc/synth.cpp, csrc/errors.cpp)
// compiled from source with -fsanitize=address,undefined and driven over the edge cases of the
// op (empty matrix, empty rows, N = 0/1/odd, hub rows that split, row ranges, int32/int64,
// every value dtype, strided views, COO duplicates, bad arguments).  Results are cross-checked
// against naive loops written here, so a sanitizer-clean run is also a correctness run.
// SURVEY.md §5 ("race detection / sanitizers"): the CPU kernel under ASan/UBSan.
// Built and run by tests/test_native_abi.py::test_cpu_kernels_under_sanitizers.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ofx_spmm.h"

namespace {

int g_fail = 0;
#define EXPECT(cond, ...)                        \
  do {                                           \
    if (!(cond)) {                               \
      ++g_fail;                                  \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);                  \
      std::printf("\n");                         \
    }                                            \
  } while (0)

uint64_t g_state = 0x9e3779b97f4a7c15ull;
uint64_t next_u64() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}
int64_t next_int(int64_t n) { return n > 0 ? (int64_t)(next_u64() % (uint64_t)n) : 0; }
float next_f32() { return (float)((int64_t)(next_u64() >> 40) - (1 << 23)) / (float)(1 << 23); }

struct Csr {
  int64_t m, k;
  std::vector<int64_t> rp, ci;
};

// Random CSR with sorted unique columns; `hub` gives one row `hub_len` nonzeros.
Csr random_csr(int64_t m, int64_t k, int64_t max_deg, int64_t hub_row, int64_t hub_len) {
  Csr a{m, k, std::vector<int64_t>(m + 1, 0), {}};
  std::vector<char> used(k > 0 ? k : 1);
  for (int64_t r = 0; r < m; ++r) {
    int64_t d = r == hub_row ? hub_len : next_int(max_deg + 1);
    if (d > k) d = k;
    std::fill(used.begin(), used.end(), 0);
    int64_t got = 0;
    while (got < d) {
      const int64_t c = next_int(k);
      if (!used[c]) used[c] = 1, ++got;
    }
    for (int64_t c = 0; c < k; ++c)
      if (used[c]) a.ci.push_back(c);
    a.rp[r + 1] = (int64_t)a.ci.size();
  }
  return a;
}

template <typename I>
std::vector<I> as(const std::vector<int64_t>& v) {
  return std::vector<I>(v.begin(), v.end());
}

// Reference order with the chunk split of the contract (include/ofx_spmm.h), fp64 storage.
void ref_spmm(const Csr& a, const std::vector<double>& val, const std::vector<double>& b,
              int64_t ldb, int64_t n, int64_t split, int64_t chunk, int64_t r0, int64_t r1,
              std::vector<double>& out) {
  out.assign((size_t)(r1 - r0) * (size_t)n, 0.0);
  for (int64_t r = r0; r < r1; ++r)
    for (int64_t c = 0; c < n; ++c) {
      const int64_t j0 = a.rp[r], j1 = a.rp[r + 1], len = j1 - j0;
      double acc = 0.0;
      if (len > split) {
        const int64_t nc = len / chunk;
        for (int64_t q = 0; q < nc; ++q) {
          const int64_t a0 = j0 + q * chunk, a1 = q == nc - 1 ? j1 : a0 + chunk;
          double p = 0.0;
          for (int64_t j = a0; j < a1; ++j) p = p + val[j] * b[a.ci[j] * ldb + c];
          acc = acc + p;
        }
      } else {
        for (int64_t j = j0; j < j1; ++j) acc = acc + val[j] * b[a.ci[j] * ldb + c];
      }
      out[(r - r0) * n + c] = acc;
    }
}

template <typename I>
void check_spmm_f64(int idx_dt, int64_t m, int64_t k, int64_t n, int64_t max_deg, int64_t hub,
                    int threads) {
  Csr a = random_csr(m, k, max_deg, m > 0 ? m / 2 : -1, hub);
  const int64_t nnz = a.rp[m];
  std::vector<I> rp = as<I>(a.rp), ci = as<I>(a.ci);
  std::vector<double> val(nnz), b((size_t)k * (n + 3)), out, got;
  for (auto& x : val) x = next_f32();
  for (auto& x : b) x = next_f32();
  const int64_t ldb = n + 3, ldc = n + 1;
  ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
  o.split_threshold = 16;
  o.chunk = 8;
  const int64_t r0 = m > 2 ? 1 : 0, r1 = m;
  got.assign((size_t)(r1 - r0) * (size_t)ldc + 1, -7.0);
  const int rc = ofx_spmm_csr_cpu(threads, idx_dt, OFX_DT_DOUBLE, m, k, n, nnz, rp.data(),
                                  nnz ? ci.data() : nullptr, nnz ? val.data() : nullptr,
                                  k ? b.data() : nullptr, ldb, got.data(), ldc, r0, r1, &o);
  EXPECT(rc == OFX_OK, "spmm_csr_cpu rc=%d (%s)", rc, ofx_last_error());
  ref_spmm(a, val, b, ldb, n, 16, 8, r0, r1, out);
  for (int64_t r = 0; r < r1 - r0; ++r)
    for (int64_t c = 0; c < n; ++c)
      EXPECT(got[r * ldc + c] == out[r * n + c], "f64 m=%lld n=%lld row %lld col %lld",
             (long long)m, (long long)n, (long long)r, (long long)c);
  EXPECT(got.back() == -7.0, "wrote past the last row");
}

void check_spmm_all_dtypes(int threads) {
  // every value dtype and the fused epilogue, int64 indices, a split hub row
  const int64_t m = 37, k = 29, n = 5;
  Csr a = random_csr(m, k, 9, 3, 28);
  const int64_t nnz = a.rp[m];
  const int dts[] = {OFX_DT_FLOAT, OFX_DT_DOUBLE, OFX_DT_FLOAT16, OFX_DT_BFLOAT16};
  const size_t sz[] = {4, 8, 2, 2};
  for (int t = 0; t < 4; ++t) {
    std::vector<unsigned char> val(nnz * sz[t] + 1), b(k * n * sz[t] + 1), bias(n * sz[t] + 1),
        c(m * n * sz[t] + 1);
    for (auto& x : val) x = (unsigned char)(next_u64() & 0x3f);  // small finite values
    for (auto& x : b) x = (unsigned char)(next_u64() & 0x3f);
    for (auto& x : bias) x = (unsigned char)(next_u64() & 0x3f);
    for (int act = 0; act < 2; ++act) {
      const int rc = ofx_spmm_csr_fused_cpu(threads, OFX_DT_INT64, dts[t], m, k, n, nnz,
                                            a.rp.data(), a.ci.data(), val.data(), b.data(), n,
                                            c.data(), n, 0, m, act ? bias.data() : nullptr,
                                            act ? OFX_ACT_RELU : OFX_ACT_NONE, nullptr);
      EXPECT(rc == OFX_OK, "fused dtype %d rc=%d (%s)", dts[t], rc, ofx_last_error());
    }
  }
}

void check_transpose_sddmm(int threads) {
  const int64_t m = 41, k = 23, n = 7;
  Csr a = random_csr(m, k, 6, 5, 20);
  const int64_t nnz = a.rp[m];
  std::vector<int32_t> rp = as<int32_t>(a.rp), ci = as<int32_t>(a.ci);
  std::vector<int32_t> trp(k + 1), tci(nnz + 1), perm(nnz + 1);
  int rc = ofx_csr_transpose_cpu(OFX_DT_INT32, m, k, nnz, rp.data(), ci.data(), trp.data(),
                                 tci.data(), perm.data());
  EXPECT(rc == OFX_OK, "transpose rc=%d (%s)", rc, ofx_last_error());
  EXPECT(trp[0] == 0 && trp[k] == nnz, "transpose row_ptr ends");
  for (int64_t t = 0; t < k; ++t)
    for (int64_t j = trp[t]; j < trp[t + 1]; ++j) {
      const int64_t src = perm[j];
      EXPECT(ci[src] == t, "transpose column mismatch at %lld", (long long)j);
      EXPECT(j == trp[t] || tci[j - 1] < tci[j], "transpose rows not ascending at %lld",
             (long long)j);
    }
  std::vector<float> A((size_t)m * n), B((size_t)k * n), out(nnz + 1, -3.f);
  for (auto& x : A) x = next_f32();
  for (auto& x : B) x = next_f32();
  rc = ofx_sddmm_csr_cpu(threads, OFX_DT_INT32, OFX_DT_FLOAT, m, k, n, nnz, rp.data(), ci.data(),
                         A.data(), n, B.data(), n, out.data(), 0, m);
  EXPECT(rc == OFX_OK, "sddmm rc=%d (%s)", rc, ofx_last_error());
  for (int64_t r = 0; r < m; ++r)
    for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
      double d = 0;
      for (int64_t c = 0; c < n; ++c) d += (double)A[r * n + c] * (double)B[ci[j] * n + c];
      EXPECT(std::fabs(d - out[j]) <= 1e-5, "sddmm value at %lld", (long long)j);
    }
  EXPECT(out[nnz] == -3.f, "sddmm wrote past nnz");
}

void check_coo() {
  const int64_t m = 13, k = 11, nnz = 90;  // many duplicates
  std::vector<int64_t> row(nnz), col(nnz);
  std::vector<float> val(nnz);
  for (int64_t i = 0; i < nnz; ++i) row[i] = next_int(m), col[i] = next_int(k), val[i] = next_f32();
  for (int merge = 0; merge < 2; ++merge) {
    std::vector<int64_t> orp(m + 1), oci(nnz + 1);
    std::vector<float> ov(nnz + 1);
    int64_t out_nnz = -1;
    const int rc = ofx_coo_to_csr_cpu(OFX_DT_INT64, OFX_DT_FLOAT, m, k, nnz, row.data(),
                                      col.data(), val.data(), merge, orp.data(), oci.data(),
                                      ov.data(), &out_nnz);
    EXPECT(rc == OFX_OK, "coo rc=%d (%s)", rc, ofx_last_error());
    EXPECT(merge ? out_nnz <= nnz : out_nnz == nnz, "coo nnz %lld", (long long)out_nnz);
    EXPECT(orp[m] == out_nnz, "coo row_ptr end");
    double s_in = 0, s_out = 0;
    for (auto x : val) s_in += x;
    for (int64_t j = 0; j < out_nnz; ++j) s_out += ov[j];
    EXPECT(std::fabs(s_in - s_out) < 1e-4, "coo value sum");
  }
  row[3] = m;  // out of range
  std::vector<int64_t> orp(m + 1), oci(nnz);
  int64_t out_nnz = 0;
  EXPECT(ofx_coo_to_csr_cpu(OFX_DT_INT64, OFX_DT_FLOAT, m, k, nnz, row.data(), col.data(),
                            nullptr, 1, orp.data(), oci.data(), nullptr, &out_nnz) != OFX_OK,
         "coo accepted a row out of range");
}

void check_partition_synth() {
  for (int64_t total : {0, 1, 7, 1001})
    for (int64_t parts : {1, 2, 3, 8}) {
      int64_t prev = 0;
      for (int64_t i = 0; i < parts; ++i) {
        int64_t b = -1, e = -1;
        EXPECT(ofx_balanced_range(total, parts, i, &b, &e) == OFX_OK, "balanced_range");
        EXPECT(b == prev && e >= b, "balanced_range not contiguous");
        prev = e;
      }
      EXPECT(prev == total, "balanced_range does not cover");
    }
  Csr a = random_csr(20, 20, 5, -1, 0);
  std::vector<int64_t> out(8);
  int64_t j0 = -1, j1 = -1;
  EXPECT(ofx_csr_row_slice_host(OFX_DT_INT64, a.rp.data(), 4, 11, out.data(), &j0, &j1) == OFX_OK,
         "row_slice");
  EXPECT(j0 == a.rp[4] && j1 == a.rp[11] && out[0] == 0 && out[7] == a.rp[11] - a.rp[4],
         "row_slice values");
  const int64_t m = 300, k = 200, nnz = 4000;
  std::vector<int64_t> rp(m + 1);
  EXPECT(ofx_synth_row_ptr(m, k, nnz, 2.5, 0, rp.data()) == OFX_OK, "synth_row_ptr");
  EXPECT(rp[0] == 0 && rp[m] == nnz, "synth_row_ptr ends");
  std::vector<int32_t> cols(nnz);
  EXPECT(ofx_synth_columns(m, k, 2.5, 0, rp.data(), 0, m, OFX_DT_INT32, cols.data(), 2) == OFX_OK,
         "synth_columns");
  for (int64_t r = 0; r < m; ++r)
    for (int64_t j = rp[r] + 1; j < rp[r + 1]; ++j) EXPECT(cols[j - 1] < cols[j], "columns sorted");
  std::vector<uint16_t> v(nnz);
  EXPECT(ofx_synth_values_host(OFX_DT_BFLOAT16, 0, nnz, 1, 0, v.data()) == OFX_OK, "synth_values");
  std::vector<float> d(7 * 9);
  EXPECT(ofx_synth_dense_host(OFX_DT_FLOAT, 3, 10, 5, 9, 2, 1, d.data()) == OFX_OK, "synth_dense");
}

void check_errors() {
  int32_t rp[3] = {0, 1, 2}, ci[2] = {0, 1};
  float v[2] = {1, 2}, b[4] = {1, 2, 3, 4}, c[4];
  EXPECT(ofx_spmm_csr_cpu(1, 99, OFX_DT_FLOAT, 2, 2, 2, 2, rp, ci, v, b, 2, c, 2, 0, 2, nullptr) ==
             OFX_EUNSUPPORTED, "bad index dtype accepted");
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 2, 2, 2, rp, ci, v, b, 1, c, 2, 0, 2,
                          nullptr) == OFX_EINVAL, "ldb < n accepted");
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 2, 2, 2, rp, ci, v, b, 2, c, 2, 1, 3,
                          nullptr) == OFX_EINVAL, "row range past m accepted");
  EXPECT(std::strlen(ofx_last_error()) > 0, "no error message");
}

}  // namespace

int main() {
  for (int threads : {1, 3}) {
    check_spmm_f64<int32_t>(OFX_DT_INT32, 0, 0, 4, 0, 0, threads);      // empty matrix
    check_spmm_f64<int32_t>(OFX_DT_INT32, 9, 6, 0, 3, 0, threads);      // n = 0
    check_spmm_f64<int32_t>(OFX_DT_INT32, 50, 40, 1, 6, 39, threads);   // n = 1, hub row
    check_spmm_f64<int64_t>(OFX_DT_INT64, 64, 70, 17, 8, 65, threads);  // odd n, hub row
    check_spmm_f64<int64_t>(OFX_DT_INT64, 5, 300, 3, 0, 250, threads);  // empty rows + one hub
    check_spmm_all_dtypes(threads);
    check_transpose_sddmm(threads);
  }
  check_coo();
  check_partition_synth();
  check_errors();
  if (g_fail) {
    std::printf("FAILED %d checks\n", g_fail);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
