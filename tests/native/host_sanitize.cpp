// host_sanitize.cpp — the library's whole host side under AddressSanitizer + UBSan
// (`make -C of-spmm_amd asan`: every translation unit, HIP units host-only; nothing runs on a GPU).
// the r03ai SIGABRT was raised on the host, inside the synchronous
// ofx_functional_spmm_csr_global call, so the host path that call takes is driven here:
//   - the OneFlow mirror: functional entry -> op inference (spmm_op.cpp) -> kernel choice
//     (registry + HOB) -> InitOpKernelCache -> Compute, on the kCPU device, for local, 1-D and 2-D
//     placements, the fused op, SDDMM, CSR transpose and the gathered op;
//   - ofx_spmm_csr_describe over every form and lane layout (the configuration choice of a launch,
//     including launch_shift_pf at LPR 16 / 32 / 64 and the prefetching form's 16-bit narrow lanes
//     that the r03ai patch added), every tuning entry, forced variants and row ranges;
//   - the error paths: bad arguments, exceptions thrown inside Compute (ofx_debug_set), and the
//     versioned structs.
// Results of the kCPU runs are checked against naive loops on exact-mode inputs (small integers:
// every order of the sums gives the same bits), so a clean run is also a correctness run.
// Built and run by tests/test_native_abi.py::test_host_path_under_sanitizers.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ofx_spmm.h"

namespace {

int g_fail = 0;
int64_t g_checks = 0;
#define EXPECT(cond, ...)                                \
  do {                                                   \
    ++g_checks;                                          \
    if (!(cond)) {                                       \
      ++g_fail;                                          \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__);    \
      std::printf(__VA_ARGS__);                          \
      std::printf("  [%s]\n", ofx_last_error());         \
    }                                                    \
  } while (0)

uint64_t g_state = 0x2545f4914f6cdd1dull;
uint64_t next_u64() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}
int64_t next_int(int64_t n) { return n > 0 ? (int64_t)(next_u64() % (uint64_t)n) : 0; }

struct Csr {
  int64_t m, k;
  std::vector<int32_t> rp, ci;
  std::vector<float> val;
};

// exact-mode values: nonzeros in {-2, -1, 1, 2}, one hub row longer than every split threshold
Csr exact_csr(int64_t m, int64_t k, int64_t max_deg, int64_t hub_row, int64_t hub_len) {
  Csr a{m, k, std::vector<int32_t>(m + 1, 0), {}, {}};
  std::vector<char> used(k);
  for (int64_t r = 0; r < m; ++r) {
    int64_t d = r == hub_row ? hub_len : next_int(max_deg + 1);
    if (d > k) d = k;
    std::fill(used.begin(), used.end(), 0);
    for (int64_t got = 0; got < d;) {
      const int64_t c = next_int(k);
      if (!used[c]) used[c] = 1, ++got;
    }
    for (int64_t c = 0; c < k; ++c)
      if (used[c]) {
        a.ci.push_back((int32_t)c);
        const float t[4] = {-2.f, -1.f, 1.f, 2.f};
        a.val.push_back(t[next_u64() & 3]);
      }
    a.rp[r + 1] = (int32_t)a.ci.size();
  }
  return a;
}

std::vector<float> exact_dense(int64_t rows, int64_t n) {
  std::vector<float> x((size_t)(rows * n));
  for (auto& v : x) v = (float)((int)next_int(17) - 8);
  return x;
}

ofx_tensor_desc vec_desc(int dt, int64_t len, const void* p) {
  ofx_tensor_desc d = OFX_TENSOR_DESC_INIT;
  d.dtype = dt;
  d.device = -1;
  d.ndim = 1;
  d.shape[0] = len;
  d.stride[0] = 1;
  d.data = const_cast<void*>(p);
  return d;
}
ofx_tensor_desc mat_desc(int dt, int64_t r, int64_t c, int64_t ld, const void* p) {
  ofx_tensor_desc d = OFX_TENSOR_DESC_INIT;
  d.dtype = dt;
  d.device = -1;
  d.ndim = 2;
  d.shape[0] = r;
  d.shape[1] = c;
  d.stride[0] = ld;
  d.stride[1] = 1;
  d.data = const_cast<void*>(p);
  return d;
}

// naive C[r, c] for rows [r0, r1) and columns [c0, c1) of A @ B (+ bias, relu)
std::vector<float> naive(const Csr& a, const std::vector<float>& b, int64_t n, int64_t r0,
                         int64_t r1, int64_t c0, int64_t c1, const float* bias = nullptr,
                         bool relu = false) {
  std::vector<float> out((size_t)((r1 - r0) * (c1 - c0)));
  for (int64_t r = r0; r < r1; ++r)
    for (int64_t c = c0; c < c1; ++c) {
      double s = 0;
      for (int32_t j = a.rp[r]; j < a.rp[r + 1]; ++j) s += (double)a.val[j] * b[a.ci[j] * n + c];
      float f = (float)s;
      if (bias) f = f + bias[c];
      if (relu && !(f > 0.f)) f = 0.f;
      out[(r - r0) * (c1 - c0) + (c - c0)] = f;
    }
  return out;
}

// ---- the OneFlow mirror on kCPU ---------------------------------------------------------------
void check_functional_placements() {
  const int64_t m = 302, k = 257, n = 24;  // N-D placements need even splits (nd_sbp_util.cpp)
  Csr a = exact_csr(m, k, 12, 77, 250);
  const std::vector<float> b = exact_dense(k, n);
  const int64_t nnz = a.rp[m];
  ofx_tensor_desc rp = vec_desc(OFX_DT_INT32, m + 1, a.rp.data());
  ofx_tensor_desc ci = vec_desc(OFX_DT_INT32, nnz, a.ci.data());
  ofx_tensor_desc v = vec_desc(OFX_DT_FLOAT, nnz, a.val.data());
  // local op
  {
    std::vector<float> out((size_t)(m * n), -7.f);
    ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, n, n, b.data());
    ofx_tensor_desc od = mat_desc(OFX_DT_FLOAT, m, n, n, out.data());
    size_t tmp = 1;
    EXPECT(ofx_functional_spmm_csr_tmp_size(&rp, &ci, &v, m, k, &bd, &tmp) == OFX_OK, "tmp size");
    EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &ci, &v, m, k, &bd, &od, nullptr, 0) == OFX_OK,
           "local functional");
    EXPECT(out == naive(a, b, n, 0, m, 0, n), "local result");
  }
  // 1-D row splits: every rank's out rows = its BalancedSplitter range
  for (int64_t P : {2, 3, 8}) {
    for (int64_t pid = 0; pid < P; ++pid) {
      int64_t lo = 0, hi = 0;
      EXPECT(ofx_balanced_range(m, P, pid, &lo, &hi) == OFX_OK, "range");
      std::vector<float> out((size_t)((hi - lo) * n) + 1, -7.f);
      ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, n, n, b.data());
      ofx_tensor_desc od = mat_desc(OFX_DT_FLOAT, hi - lo, n, n, out.data());
      EXPECT(ofx_functional_spmm_csr_ex(nullptr, &rp, &ci, &v, m, k, &bd, &od, nullptr, 0, pid, P,
                                        0, 2) == OFX_OK,
             "1-D P=%lld pid=%lld", (long long)P, (long long)pid);
      const std::vector<float> want = naive(a, b, n, lo, hi, 0, n);
      EXPECT(std::equal(want.begin(), want.end(), out.begin()), "1-D rows P=%lld", (long long)P);
      EXPECT(out.back() == -7.f, "1-D wrote past its rows");
    }
  }
  // 2-D {2, 2} with (S(0), S(1)): a row half and a column half per rank (b is the column slice)
  {
    const int64_t hier[2] = {2, 2};
    const int32_t axes[2] = {0, 1};
    for (int64_t pid = 0; pid < 4; ++pid) {
      int64_t lo = 0, hi = 0, c0 = 0, c1 = 0;
      ofx_balanced_range(m, 2, pid / 2, &lo, &hi);
      ofx_balanced_range(n, 2, pid % 2, &c0, &c1);
      std::vector<float> bs((size_t)(k * (c1 - c0)));
      for (int64_t r = 0; r < k; ++r)
        for (int64_t c = c0; c < c1; ++c) bs[r * (c1 - c0) + (c - c0)] = b[r * n + c];
      std::vector<float> out((size_t)((hi - lo) * (c1 - c0)), -7.f);
      ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, c1 - c0, c1 - c0, bs.data());
      ofx_tensor_desc od = mat_desc(OFX_DT_FLOAT, hi - lo, c1 - c0, c1 - c0, out.data());
      size_t tmp = 0;
      EXPECT(ofx_functional_spmm_csr_global(nullptr, &rp, &ci, &v, m, k, &bd, n, &od, nullptr, 0, 2,
                                            hier, axes, pid, 1, &tmp) == OFX_OK,
             "2-D tmp size");
      EXPECT(ofx_functional_spmm_csr_global(nullptr, &rp, &ci, &v, m, k, &bd, n, &od, nullptr, 0, 2,
                                            hier, axes, pid, 1, nullptr) == OFX_OK,
             "2-D pid %lld", (long long)pid);
      EXPECT(out == naive(a, b, n, lo, hi, c0, c1), "2-D result pid %lld", (long long)pid);
    }
  }
  // fused op: relu(A @ b + bias)
  {
    std::vector<float> bias(n), out((size_t)(m * n), -7.f);
    for (auto& x : bias) x = (float)((int)next_int(9) - 4);
    ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, n, n, b.data());
    ofx_tensor_desc bsd = vec_desc(OFX_DT_FLOAT, n, bias.data());
    ofx_tensor_desc od = mat_desc(OFX_DT_FLOAT, m, n, n, out.data());
    size_t tmp = 0;
    EXPECT(ofx_functional_fused_spmm_csr(nullptr, &rp, &ci, &v, &bd, &bsd, m, k, 1, &od, nullptr,
                                         0, &tmp) == OFX_OK,
           "fused tmp");
    EXPECT(ofx_functional_fused_spmm_csr(nullptr, &rp, &ci, &v, &bd, &bsd, m, k, 1, &od, nullptr,
                                         0, nullptr) == OFX_OK,
           "fused");
    EXPECT(out == naive(a, b, n, 0, m, 0, n, bias.data(), true), "fused result");
  }
  // gradient ops: transpose, SDDMM, gathered
  {
    std::vector<int32_t> trp(k + 1), tci(nnz), perm(nnz);
    ofx_tensor_desc trpd = vec_desc(OFX_DT_INT32, k + 1, trp.data());
    ofx_tensor_desc tcid = vec_desc(OFX_DT_INT32, nnz, tci.data());
    ofx_tensor_desc permd = vec_desc(OFX_DT_INT32, nnz, perm.data());
    size_t tmp = 0;
    EXPECT(ofx_functional_csr_transpose(nullptr, &rp, &ci, m, k, &trpd, &tcid, &permd, nullptr, 0,
                                        &tmp) == OFX_OK,
           "transpose tmp");
    std::vector<char> tbuf(tmp + 1);
    EXPECT(ofx_functional_csr_transpose(nullptr, &rp, &ci, m, k, &trpd, &tcid, &permd, tbuf.data(),
                                        tmp, nullptr) == OFX_OK,
           "transpose");
    EXPECT(trp[k] == nnz, "transpose row_ptr end");
    const std::vector<float> dc = exact_dense(m, n);
    std::vector<float> dv(nnz, -7.f);
    ofx_tensor_desc dcd = mat_desc(OFX_DT_FLOAT, m, n, n, dc.data());
    ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, n, n, b.data());
    ofx_tensor_desc dvd = vec_desc(OFX_DT_FLOAT, nnz, dv.data());
    EXPECT(ofx_functional_sddmm_csr(nullptr, &rp, &ci, &dcd, &bd, m, k, &dvd, nullptr, 0,
                                    &tmp) == OFX_OK,
           "sddmm tmp");
    std::vector<char> sbuf(tmp + 1);
    EXPECT(ofx_functional_sddmm_csr(nullptr, &rp, &ci, &dcd, &bd, m, k, &dvd, sbuf.data(), tmp,
                                    nullptr) == OFX_OK,
           "sddmm");
    for (int64_t r = 0; r < m; ++r)
      for (int32_t j = a.rp[r]; j < a.rp[r + 1]; ++j) {
        double s = 0;
        for (int64_t c = 0; c < n; ++c) s += (double)dc[r * n + c] * b[a.ci[j] * n + c];
        EXPECT(dv[j] == (float)s, "sddmm value %d", (int)j);
      }
    // d(b) = A^T @ dC through spmm_csr_gathered (A's values read through perm)
    std::vector<float> db((size_t)(k * n), -7.f);
    ofx_tensor_desc dbd = mat_desc(OFX_DT_FLOAT, k, n, n, db.data());
    EXPECT(ofx_functional_spmm_csr_gathered(nullptr, &trpd, &tcid, &v, &permd, &dcd, k, m, &dbd,
                                            nullptr, 0, &tmp) == OFX_OK,
           "gathered tmp");
    std::vector<char> gbuf(tmp + 1);
    EXPECT(ofx_functional_spmm_csr_gathered(nullptr, &trpd, &tcid, &v, &permd, &dcd, k, m, &dbd,
                                            gbuf.data(), tmp, nullptr) == OFX_OK,
           "gathered");
    for (int64_t c = 0; c < k; ++c)
      for (int64_t col = 0; col < n; col += 5) {
        double s = 0;
        for (int64_t r = 0; r < m; ++r)
          for (int32_t j = a.rp[r]; j < a.rp[r + 1]; ++j)
            if (a.ci[j] == c) s += (double)a.val[j] * dc[r * n + col];
        EXPECT(db[c * n + col] == (float)s, "gathered (%lld, %lld)", (long long)c, (long long)col);
      }
  }
}

void check_error_paths() {
  const int64_t m = 20, k = 16, n = 4;
  Csr a = exact_csr(m, k, 5, -1, 0);
  const std::vector<float> b = exact_dense(k, n);
  const int64_t nnz = a.rp[m];
  std::vector<float> out((size_t)(m * n));
  ofx_tensor_desc rp = vec_desc(OFX_DT_INT32, m + 1, a.rp.data());
  ofx_tensor_desc ci = vec_desc(OFX_DT_INT32, nnz, a.ci.data());
  ofx_tensor_desc v = vec_desc(OFX_DT_FLOAT, nnz, a.val.data());
  ofx_tensor_desc bd = mat_desc(OFX_DT_FLOAT, k, n, n, b.data());
  ofx_tensor_desc od = mat_desc(OFX_DT_FLOAT, m, n, n, out.data());
  // exceptions thrown inside Compute come back as status codes
  const int want[4] = {OFX_OK, OFX_EINTERNAL, OFX_ENOMEM, OFX_EINTERNAL};
  for (int kind = 1; kind <= 3; ++kind) {
    EXPECT(ofx_debug_set(OFX_DEBUG_THROW_IN_COMPUTE, kind) == OFX_OK, "knob");
    EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &ci, &v, m, k, &bd, &od, nullptr, 0) == want[kind],
           "exception kind %d", kind);
    EXPECT(std::strstr(ofx_last_error(), "ofx_functional_spmm_csr") != nullptr, "names the entry");
  }
  ofx_debug_set(OFX_DEBUG_THROW_IN_COMPUTE, -1);
  EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &ci, &v, m, k, &bd, &od, nullptr, 0) == OFX_OK,
         "after the exceptions");
  // bad arguments are status codes with a message
  EXPECT(ofx_functional_spmm_csr(nullptr, nullptr, &ci, &v, m, k, &bd, &od, nullptr, 0) == OFX_EINVAL,
         "NULL row_ptr");
  ofx_tensor_desc bad = v;
  bad.dtype = OFX_DT_DOUBLE;
  EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &ci, &bad, m, k, &bd, &od, nullptr, 0) != OFX_OK,
         "values dtype mismatch");
  ofx_tensor_desc od_wrong = mat_desc(OFX_DT_FLOAT, m - 1, n, n, out.data());
  EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &ci, &v, m, k, &bd, &od_wrong, nullptr, 0) == OFX_EINVAL,
         "out rows");
  ofx_tensor_desc unversioned = ci;
  unversioned.struct_size = 0;
  EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &unversioned, &v, m, k, &bd, &od, nullptr, 0) ==
             OFX_EINVAL,
         "struct_size 0");
  const int64_t hier[1] = {4};
  const int32_t axes[1] = {0};
  EXPECT(ofx_functional_spmm_csr_global(nullptr, &rp, &ci, &v, m, k, &bd, -1, &od, nullptr, 0, 1,
                                        hier, axes, 7, 1, nullptr) == OFX_EINVAL,
         "parallel_id outside the placement");
  // options: an older (48-byte) layout is read with defaults for range_nnz; an unset one refused
  ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
  std::vector<float> c((size_t)(m * n));
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, m, k, n, nnz, a.rp.data(), a.ci.data(),
                          a.val.data(), b.data(), n, c.data(), n, 0, m, &o) == OFX_OK,
         "options");
  unsigned char* old = static_cast<unsigned char*>(std::malloc(OFX_SPMM_OPTIONS_MIN_SIZE));
  std::memcpy(old, &o, OFX_SPMM_OPTIONS_MIN_SIZE);
  const uint32_t old_size = OFX_SPMM_OPTIONS_MIN_SIZE;  // the field is the first 4 bytes
  std::memcpy(old, &old_size, sizeof(old_size));
  // ASan: reading range_nnz (bytes 48-55) of this 48-byte block would be a heap overflow
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, m, k, n, nnz, a.rp.data(), a.ci.data(),
                          a.val.data(), b.data(), n, c.data(), n, 2, m,
                          reinterpret_cast<const ofx_spmm_options*>(old)) == OFX_OK,
         "older options layout");
  char buf[512];
  EXPECT(ofx_spmm_csr_describe(OFX_DT_INT32, OFX_DT_FLOAT, 1 << 20, 1 << 20, 64, 20 << 20,
                               (void*)256, 64, (void*)256, 64, 0, 20000,
                               reinterpret_cast<const ofx_spmm_options*>(old), buf, sizeof(buf)) ==
             OFX_OK,
         "describe, older options layout");
  std::free(old);
  o.struct_size = 0;
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, m, k, n, nnz, a.rp.data(), a.ci.data(),
                          a.val.data(), b.data(), n, c.data(), n, 0, m, &o) == OFX_EINVAL,
         "unset options");
  ofx_placement pl = OFX_PLACEMENT_INIT;
  pl.device_type = OFX_DEV_CPU;
  pl.parallel_num = 2;
  const int64_t shape[2] = {10, 4};
  EXPECT(ofx_boxing_check_ccl_s2b(&pl, 2, shape, "S(0)", "B") == OFX_OK, "placement");
  pl.struct_size = 4;
  EXPECT(ofx_boxing_check_ccl_s2b(&pl, 2, shape, "S(0)", "B") == OFX_EINVAL, "placement size");
  pl.struct_size = sizeof(pl);
  pl.magic = 0;  // a size that looks right is not trusted without the tag
  EXPECT(ofx_boxing_check_ccl_s2b(&pl, 2, shape, "S(0)", "B") == OFX_EINVAL, "placement tag");
  ofx_tensor_desc untagged = ci;
  untagged.magic = 0;
  EXPECT(ofx_functional_spmm_csr(nullptr, &rp, &untagged, &v, m, k, &bd, &od, nullptr, 0) ==
             OFX_EINVAL,
         "descriptor tag");
  // the unversioned options layout (no struct_size, no tag) in a heap block of exactly its size,
  // with split_threshold = 128: its low half would read as a plausible struct_size; ASan checks
  // that nothing past the 40 bytes is read and the call is refused
  struct options_unversioned {
    int64_t split_threshold, chunk;
    int32_t ordered, variant;
    int64_t heavy_threshold;
    int32_t planned, reserved;
  };
  auto* r4 = static_cast<options_unversioned*>(std::malloc(sizeof(options_unversioned)));
  std::memset(r4, 0, sizeof(*r4));
  r4->split_threshold = 128;
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, m, k, n, nnz, a.rp.data(), a.ci.data(),
                          a.val.data(), b.data(), n, c.data(), n, 0, m,
                          reinterpret_cast<const ofx_spmm_options*>(r4)) == OFX_EINVAL,
         "unversioned options, split_threshold 128");
  std::free(r4);
  EXPECT(ofx_debug_set(99, 0) == OFX_EINVAL, "unknown knob");
}

// ---- the configuration choice of every launch (describe: nothing launched) ---------------------
struct Shape {
  int64_t m, nnz;
};

int64_t ws_of(const char* s) {
  const char* p = std::strstr(s, "ws=");
  return p ? std::atoll(p + 3) : -1;
}

void check_describe() {
  const Shape shapes[] = {{2708, 10556},            // small form
                          {20000, 400000},          // mid form
                          {169343, 1166243},        // prefetching form (arxiv-shaped)
                          {60000, 1500000},         // prefetching form
                          {1000000, 20000000},      // bandwidth configuration
                          {2449029, 123718280},     // products
                          {111059956, 1615685872}}; // papers-scale: B >= 4 GiB at N >= 10 fp32
  const int vals[] = {OFX_DT_FLOAT, OFX_DT_DOUBLE, OFX_DT_BFLOAT16, OFX_DT_FLOAT16};
  const int idxs[] = {OFX_DT_INT32, OFX_DT_INT64};
  int64_t runs = 0;
  char buf[512];
  for (const Shape& sh : shapes)
    for (int vi = 0; vi < 4; ++vi)
      for (int ii = 0; ii < 2; ++ii) {
        const int64_t esz = vals[vi] == OFX_DT_DOUBLE ? 8 : vals[vi] == OFX_DT_FLOAT ? 4 : 2;
        for (int64_t n = 1; n <= 300; n += (n < 72 ? 1 : 13)) {
          size_t whole = 0;
          const int rc0 = ofx_spmm_csr_workspace_size(idxs[ii], vals[vi], sh.m, sh.m, n, sh.nnz,
                                                      nullptr, &whole);
          if (idxs[ii] == OFX_DT_INT32 && sh.nnz > INT32_MAX) continue;
          EXPECT(rc0 == OFX_OK, "ws m=%lld n=%lld", (long long)sh.m, (long long)n);
          // aligned and 4-B / element-aligned views, several row ranges
          for (int64_t addr : {(int64_t)256, 256 + esz}) {  // vector-aligned, element-aligned
            const int64_t ranges[3][2] = {{0, sh.m}, {1, sh.m}, {sh.m / 3, sh.m / 3 + sh.m / 5 + 1}};
            for (const auto& rg : ranges) {
              buf[0] = 0;
              const int rc = ofx_spmm_csr_describe(idxs[ii], vals[vi], sh.m, sh.m, n, sh.nnz,
                                                   (void*)addr, n, (void*)addr, n, rg[0], rg[1],
                                                   nullptr, buf, sizeof(buf));
              ++runs;
              EXPECT(rc == OFX_OK && std::strncmp(buf, "form=", 5) == 0,
                     "describe dt=%d idx=%d m=%lld n=%lld", vals[vi], idxs[ii], (long long)sh.m,
                     (long long)n);
              EXPECT(ws_of(buf) >= 0 && (size_t)ws_of(buf) <= whole,
                     "launch workspace %lld > query %zu (m=%lld n=%lld rows [%lld, %lld))",
                     (long long)ws_of(buf), whole, (long long)sh.m, (long long)n,
                     (long long)rg[0], (long long)rg[1]);
            }
          }
        }
        // forced forms and layouts: applicable or refused with a status, never anything else
        for (int variant : {30000, 30001, 30002, 30003, 30004, 30005, 30006, 104, 108, 116, 132,
                            164, 204, 216, 404, 416, 432, 816}) {
          for (int64_t n : {8, 16, 17, 47, 64, 128}) {
            ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
            o.variant = variant;
            const int rc = ofx_spmm_csr_describe(idxs[ii], vals[vi], sh.m, sh.m, n, sh.nnz,
                                                 (void*)256, n, (void*)256, n, 0, sh.m, &o, buf,
                                                 sizeof(buf));
            ++runs;
            EXPECT(rc == OFX_OK || rc == OFX_EINVAL, "variant %d rc %d", variant, rc);
          }
        }
      }
  // every tuning-table entry (float / 16-bit values, int32 indices)
  for (int vi : {0, 2, 3})
    for (int id = 0; id < 200; ++id)
      for (int64_t n : {8, 16, 17, 20, 32, 47, 64, 128}) {
        ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
        o.variant = 10000 + id;
        const int rc = ofx_spmm_csr_describe(OFX_DT_INT32, vals[vi], 169343, 169343, n, 1166243,
                                             (void*)256, n, (void*)256, n, 0, 169343, &o, buf,
                                             sizeof(buf));
        ++runs;
        EXPECT(rc == OFX_OK || rc == OFX_EINVAL, "tuned %d rc %d", id, rc);
      }
  // the configurations the r03ai patch added (prefetching-form lane layouts)
  auto form = [&](int dt, int64_t n) {
    buf[0] = 0;
    ofx_spmm_csr_describe(OFX_DT_INT32, dt, 60000, 60000, n, 1500000, (void*)256, n, (void*)256, n,
                          0, 60000, nullptr, buf, sizeof(buf));
    return std::string(buf);
  };
  for (int64_t n : {33, 41, 47, 63})
    EXPECT(form(OFX_DT_FLOAT, n).find("VEC=4 LPR=16") != std::string::npos &&
               form(OFX_DT_FLOAT, n).find("SH=1") != std::string::npos,
           "shifted window LPR 16, fp32 N=%lld: %s", (long long)n, form(OFX_DT_FLOAT, n).c_str());
  for (int64_t n : {65, 99, 127})  // round 5: launch_mid_width_pf up to 128 columns
    EXPECT(form(OFX_DT_FLOAT, n).find("VEC=8 LPR=16") != std::string::npos &&
               form(OFX_DT_FLOAT, n).find("HV=4") != std::string::npos,
           "mid-width 8-element windows, fp32 N=%lld: %s", (long long)n, form(OFX_DT_FLOAT, n).c_str());
  for (int64_t n : {131, 301})
    EXPECT(form(OFX_DT_FLOAT, n).find("LPR=64") != std::string::npos &&
               form(OFX_DT_FLOAT, n).find("SH=1") != std::string::npos,
           "shifted window LPR 64, fp32 N=%lld: %s", (long long)n, form(OFX_DT_FLOAT, n).c_str());
  EXPECT(form(OFX_DT_BFLOAT16, 16).find("form=narrow") != std::string::npos, "bf16 N=16: %s",
         form(OFX_DT_BFLOAT16, 16).c_str());
  // round 5: rows of 17-64 columns take launch_mid_width_pf (2-element lanes in the wave items)
  EXPECT(form(OFX_DT_BFLOAT16, 48).find("form=narrow") != std::string::npos &&
             form(OFX_DT_BFLOAT16, 48).find("HV=4 XL=1") != std::string::npos,
         "bf16 N=48: %s", form(OFX_DT_BFLOAT16, 48).c_str());
  EXPECT(form(OFX_DT_FLOAT16, 8).find("form=narrow") != std::string::npos, "f16 N=8: %s",
         form(OFX_DT_FLOAT16, 8).c_str());
  std::printf("describe: %lld configurations\n", (long long)runs);
}

}  // namespace

int main() {
  check_functional_placements();
  check_error_paths();
  check_describe();
  if (g_fail) {
    std::printf("FAILED %d of %lld checks\n", g_fail, (long long)g_checks);
    return 1;
  }
  std::printf("OK %lld checks\n", (long long)g_checks);
  return 0;
}
