/* A plain-C host of the C-ABI (include/ofx_spmm.h), as a non-Python caller (cgo / JNI / a C++
 * framework) would bind it: CPU kernel, fused epilogue, balanced ranges, row slices, error
 * reporting.  Built and run by tests/test_native_abi.py with gcc; no GPU needed. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "ofx_spmm.h"

static int fails = 0;
#define EXPECT(c)                                              \
  do {                                                         \
    if (!(c)) {                                                \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                 \
    }                                                          \
  } while (0)

int main(void) {
  /* A = [[1, 0, 2], [0, 3, 0]] (CSR), B = [[1, 0], [0, 1], [1, 1]] */
  const int32_t rp[3] = {0, 2, 3};
  const int32_t col[3] = {0, 2, 1};
  const float val[3] = {1.f, 2.f, 3.f};
  const float b[6] = {1.f, 0.f, 0.f, 1.f, 1.f, 1.f};
  float c[4];
  memset(c, 0xff, sizeof(c));
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          NULL) == OFX_OK);
  EXPECT(c[0] == 3.f && c[1] == 2.f && c[2] == 0.f && c[3] == 3.f);

  /* fused: relu(A @ B + bias), bias = [-3, -1] -> [[0, 1], [0, 2]]; -0 -> +0 */
  const float bias[2] = {-3.f, -1.f};
  EXPECT(ofx_spmm_csr_fused_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2,
                                0, 2, bias, OFX_ACT_RELU, NULL) == OFX_OK);
  EXPECT(c[0] == 0.f && !signbit(c[0]) && c[1] == 1.f && c[2] == 0.f && c[3] == 2.f);

  /* one row of the global form: row range [1, 2) into a 1-row output */
  float c1[2] = {0, 0};
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c1, 2, 1, 2,
                          NULL) == OFX_OK);
  EXPECT(c1[0] == 0.f && c1[1] == 3.f);

  /* BalancedSplitter(10, 4): 3, 3, 2, 2 */
  int64_t lo, hi;
  EXPECT(ofx_balanced_range(10, 4, 1, &lo, &hi) == OFX_OK && lo == 3 && hi == 6);
  EXPECT(ofx_balanced_range(10, 4, 3, &lo, &hi) == OFX_OK && lo == 8 && hi == 10);

  /* row slice of the CSR: rows [1, 2) -> row_ptr [0, 1], nnz range [2, 3) */
  int32_t out_rp[2];
  int64_t n0, n1;
  EXPECT(ofx_csr_row_slice_host(OFX_DT_INT32, rp, 1, 2, out_rp, &n0, &n1) == OFX_OK);
  EXPECT(out_rp[0] == 0 && out_rp[1] == 1 && n0 == 2 && n1 == 3);

  /* errors: a status code plus a thread-local message, never an abort */
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_FLOAT, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          NULL) == OFX_EUNSUPPORTED);
  EXPECT(strlen(ofx_last_error()) > 0);
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 1, c, 2, 0, 2,
                          NULL) == OFX_EINVAL); /* ldb < n */
  EXPECT(ofx_spmm_default_split(128) == 512);

  /* versioned options (include/ofx_spmm.h): a caller compiled against the first tagged layout
   * (48 bytes, before range_nnz) is read with range_nnz at its default; the unversioned (round-3
   * and round-4) layout, which had no struct_size and no tag (its first 4 bytes are the low half
   * of split_threshold), is refused instead of misread, whatever split_threshold holds */
  struct options_v1 {
    uint32_t struct_size;
    uint32_t magic;
    int64_t split_threshold, chunk;
    int32_t ordered, variant;
    int64_t heavy_threshold;
    int32_t planned, reserved;
  } v1;
  struct options_round3 {
    int64_t split_threshold, chunk;
    int32_t ordered, variant;
    int64_t heavy_threshold;
    int32_t planned, reserved;
  } r3;
  EXPECT(sizeof(v1) == OFX_SPMM_OPTIONS_MIN_SIZE && sizeof(ofx_spmm_options) > sizeof(v1));
  memset(&v1, 0, sizeof(v1));
  v1.struct_size = sizeof(v1);
  v1.magic = OFX_STRUCT_MAGIC;
  v1.split_threshold = 1; /* every row of 2 nonzeros splits: same bits (exact inputs) */
  memset(c, 0xff, sizeof(c));
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          (const ofx_spmm_options*)&v1) == OFX_OK);
  EXPECT(c[0] == 3.f && c[1] == 2.f && c[2] == 0.f && c[3] == 3.f);
  memset(&r3, 0, sizeof(r3));
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          (const ofx_spmm_options*)&r3) == OFX_EINVAL);
  r3.split_threshold = 16;
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          (const ofx_spmm_options*)&r3) == OFX_EINVAL);
  EXPECT(strstr(ofx_last_error(), "OFX_SPMM_OPTIONS_INIT") != NULL);
  /* split_threshold = 128 reads as struct_size 128 (>= the minimum) without the tag */
  r3.split_threshold = 128;
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          (const ofx_spmm_options*)&r3) == OFX_EINVAL);
  EXPECT(strstr(ofx_last_error(), "OFX_STRUCT_MAGIC") != NULL);
  /* a tagged first layout whose tag was overwritten is refused too */
  v1.magic = 0;
  EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0, 2,
                          (const ofx_spmm_options*)&v1) == OFX_EINVAL);
  {
    ofx_spmm_options cur = OFX_SPMM_OPTIONS_INIT;
    EXPECT(cur.struct_size == sizeof(ofx_spmm_options) && cur.magic == OFX_STRUCT_MAGIC);
    EXPECT(ofx_spmm_csr_cpu(1, OFX_DT_INT32, OFX_DT_FLOAT, 2, 3, 2, 3, rp, col, val, b, 2, c, 2, 0,
                            2, &cur) == OFX_OK);
  }

  /* the functional entry with the op's attributes (static_csr is a GPU-kernel state matter: the
   * kCPU kernel ignores it), through tagged tensor descriptors and a tagged attrs struct */
  {
    ofx_tensor_desc d_rp = OFX_TENSOR_DESC_INIT, d_ci = OFX_TENSOR_DESC_INIT,
                    d_v = OFX_TENSOR_DESC_INIT, d_b = OFX_TENSOR_DESC_INIT,
                    d_c = OFX_TENSOR_DESC_INIT;
    d_rp.dtype = OFX_DT_INT32, d_rp.device = -1, d_rp.ndim = 1, d_rp.shape[0] = 3, d_rp.stride[0] = 1;
    d_rp.data = (void*)rp;
    d_ci.dtype = OFX_DT_INT32, d_ci.device = -1, d_ci.ndim = 1, d_ci.shape[0] = 3, d_ci.stride[0] = 1;
    d_ci.data = (void*)col;
    d_v.dtype = OFX_DT_FLOAT, d_v.device = -1, d_v.ndim = 1, d_v.shape[0] = 3, d_v.stride[0] = 1;
    d_v.data = (void*)val;
    d_b.dtype = OFX_DT_FLOAT, d_b.device = -1, d_b.ndim = 2, d_b.shape[0] = 3, d_b.shape[1] = 2;
    d_b.stride[0] = 2, d_b.stride[1] = 1, d_b.data = (void*)b;
    d_c.dtype = OFX_DT_FLOAT, d_c.device = -1, d_c.ndim = 2, d_c.shape[0] = 2, d_c.shape[1] = 2;
    d_c.stride[0] = 2, d_c.stride[1] = 1, d_c.data = c;
    const int64_t hier[1] = {1};
    const int32_t axes[1] = {-1};
    ofx_spmm_attrs at = OFX_SPMM_ATTRS_INIT;
    at.static_csr = 1;
    memset(c, 0xff, sizeof(c));
    EXPECT(ofx_functional_spmm_csr_global_attrs(NULL, &d_rp, &d_ci, &d_v, 2, 3, &d_b, -1, &d_c,
                                                NULL, 0, 1, hier, axes, 0, 1, NULL, &at) == OFX_OK);
    EXPECT(c[0] == 3.f && c[1] == 2.f && c[2] == 0.f && c[3] == 3.f);
    at.magic = 0;
    EXPECT(ofx_functional_spmm_csr_global_attrs(NULL, &d_rp, &d_ci, &d_v, 2, 3, &d_b, -1, &d_c,
                                                NULL, 0, 1, hier, axes, 0, 1, NULL, &at) ==
           OFX_EINVAL);
    int64_t entries = -1, plans = -1, hits = -1;
    EXPECT(ofx_spmm_static_plans(&entries, &plans, &hits, 0) == OFX_OK && entries == 0 &&
           plans == 0 && hits == 0);
  }

  printf("%s %d failures\n", fails ? "FAIL" : "OK", fails);
  return fails ? 1 : 0;
}
