/*
 * ofx_spmm.h — the C-ABI drop-in boundary of the MI355X-native `spmm_csr` operator.
 *
 * Every entry point is `extern "C"`, takes plain pointers/sizes, returns an `int` status
 * (OFX_OK == 0) and, on failure, leaves a human-readable message in the calling thread's
 * `ofx_last_error()` buffer.  No torch / OneFlow types cross this boundary.
 *
 * What each group replaces in the reference (yuang-chen/of-spmm == OneFlow v0.8.1-dev; paths
 * relative to the reference root).  The reference has NO SpMM, so the op-level
 * entries replace the *composition* the reference would run today plus the OneFlow surfaces a
 * new user op plugs into:
 *
 *  - ofx_spmm_csr / ofx_spmm_csr_workspace_size
 *      the device kernel behind `REGISTER_USER_KERNEL("spmm_csr")` for the HIP device.
 *      Semantics restate gather -> multiply -> unsorted_segment_sum:
 *      oneflow/user/kernels/gather_kernel_util.cpp:72-92 (row copy of B[idx]),
 *      oneflow/user/kernels/unsorted_segment_sum_kernel_util.cpp:29-45 (std::plus, index order).
 *      Workspace size mirrors `SetInferTmpSizeFn` (oneflow/core/framework/user_op_kernel_registry.h:90)
 *      and the "tmp_buffer" arg (oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:162).
 *      Launch is async on the given stream, allocates nothing, never synchronises
 *      (kernel contract of oneflow/core/framework/op_kernel.h:287-318).
 *  - ofx_spmm_csr_cpu
 *      the DeviceType::kCPU kernel (row-parallel, idiom of oneflow/core/ep/cpu/cpu_stream.h:104-145).
 *  - ofx_balanced_range / ofx_csr_row_slice
 *      BalancedSplitter::At (oneflow/core/common/balanced_splitter.cpp:20-40) as used by
 *      GetTensorSliceView4ParallelId (oneflow/core/job/nd_sbp_util.cpp:98-104) and the
 *      OpKernelCache row-range pattern (oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:46-78).
 *  - ofx_device_* / ofx_stream_* / ofx_event_* / ofx_memcpy_async / ofx_memset_async / ofx_malloc
 *      the ep device layer reduced to a thin C-ABI: ep::Device (oneflow/core/ep/include/device.h:33-62),
 *      ep::Stream (stream.h:30-49), ep::Event (event.h:26-34), primitive::Memcpy (memcpy.h:33-39),
 *      primitive::Memset (memset.h:26-32); CUDA impl oneflow/core/ep/cuda/cuda_stream.cpp:90-142.
 *  - ofx_comm_* / ofx_allgather
 *      ccl::AllGather (oneflow/user/kernels/collective_communication/include/all_gather.h:24-38),
 *      CudaAllGather::Launch -> ncclAllGather (.../cuda/cuda_all_gather.cpp:25-47), and the comm
 *      bootstrap of EagerNcclCommMgr (oneflow/core/job/eager_nccl_comm_manager.cpp:57-131).
 *  - ofx_functional_spmm_csr
 *      the functional entry `functional::SpmmCsr` (template oneflow/core/functional/impl/nn_functor.cpp:3861-3884)
 *      -> op inference (oneflow/user/ops/spmm_op.cpp, our C++ mirror) -> kernel registry
 *      (REGISTER_USER_KERNEL, oneflow/core/framework/user_op_registry_manager.h:81-84) -> Compute.
 *
 * Data-type codes are OneFlow's `DataType` numbering (oneflow/core/common/data_type.proto:4-26).
 */
#ifndef OFX_SPMM_H_
#define OFX_SPMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define OFX_OK 0
#define OFX_EINVAL 1       /* shape / dtype / argument mismatch (CHECK_*_OR_RETURN analogue) */
#define OFX_EDEVICE 2      /* HIP runtime error (launch, memcpy, ...)                          */
#define OFX_ENOMEM 3       /* allocation failed                                                */
#define OFX_EUNSUPPORTED 4 /* dtype / layout combination not registered (OpKernelNotFound)     */
#define OFX_ECOMM 5        /* RCCL error                                                       */
#define OFX_EWORKSPACE 6   /* workspace smaller than ofx_spmm_csr_workspace_size()             */
#define OFX_EPLAN 7        /* an EARLIER asynchronous launch failed and poisoned its output     *
                            * (NaN): its device-side work-list plan gave up, or it found no     *
                            * valid plan in its workspace                                        *
                            * (reported once, at the next launching call or sync; see            *
                            * ofx_device_error_check)                                            */
#define OFX_EINTERNAL 8    /* an unexpected C++ exception inside the library, caught at the     *
                            * boundary (no exception ever crosses this C-ABI)                    */

/* ---- OneFlow DataType codes (oneflow/core/common/data_type.proto:4-26) ------------------- */
#define OFX_DT_FLOAT 2
#define OFX_DT_DOUBLE 3
#define OFX_DT_INT32 5
#define OFX_DT_INT64 6
#define OFX_DT_FLOAT16 9
#define OFX_DT_BFLOAT16 11

/* Message describing the last failure on the calling thread ("" if none). */
const char* ofx_last_error(void);
/* Library version string, e.g. "ofx-spmm 0.2.0 gfx950". */
const char* ofx_version(void);

/* Device-side loud failures.  A kernel that cannot produce its output (its work-list plan failed
 * or is not valid) fills the whole output with one canonical quiet NaN (f32 0x7fc00000, f64
 * 0x7ff8000000000000, bf16 0x7fc0, f16 0x7e00; the nonzeros of its rows for SDDMM), so no stale
 * or uninitialised value can be read as a result, and raises a device-error word (host-mapped
 * memory).  The library reports it as OFX_EPLAN, once, at the next launching entry
 * (ofx_spmm_csr*, ofx_sddmm_csr, ofx_functional_spmm_csr*), at ofx_stream_sync /
 * ofx_event_sync / ofx_device_synchronize / ofx_graph_launch, or here.  A foreign
 * synchronisation (hipStreamSynchronize, torch.cuda.synchronize()) does not look at the word:
 * call this after it, or read the NaN.  The words are process-wide, not per stream or device:
 * with several threads or streams the report reaches whichever entry comes next, which may not
 * be the caller of the failed launch.  Mirrors the reference's fatal kernel CHECKs
 * (oneflow/user/kernels/matrix_vector_product_kernel.cpp:98-105) as a status code.            */
int ofx_device_error_check(void);

/* Test hooks (no effect unless set).  OFX_DEBUG_PLAN_SPIN_LIMIT: polls of a predecessor's status
 * word before the planner's look-back gives up (default 2^22; 0 = every block but the first gives
 * up at once).  OFX_DEBUG_THROW_IN_COMPUTE: the op kernels' Compute throws (1 std::runtime_error,
 * 2 std::bad_alloc, 3 a non-std exception; 0 off), to test the boundary's exception guard.
 * OFX_DEBUG_EXCHANGE_STALL: the device deadline of ofx_comm_set_timeouts expires (test).
 * value < 0 restores the default.                                                            */
#define OFX_DEBUG_PLAN_SPIN_LIMIT 1
#define OFX_DEBUG_THROW_IN_COMPUTE 2
#define OFX_DEBUG_EXCHANGE_STALL 3 /* != 0: an exchange's device completion is never seen      */
int ofx_debug_set(int knob, int64_t value);

/* ---- SpMM schedule options --------------------------------------------------------------
 * Accumulation-order contract (identical in the CPU kernel, the HIP kernel and the oracle):
 *   acc = 0; for j in row (ascending): acc = acc + (val[j] * B[col[j], :])     (mul, then add;
 *   no FMA contraction; fp32 accumulator for f32/f16/bf16, f64 for f64; one rounding to T at the end)
 * Rows longer than `split_threshold` nonzeros are cut into consecutive chunks of `chunk`
 * nonzeros; each chunk is summed as above from 0, and the chunk partials are then added
 * in chunk order into acc = 0.  split_threshold <= 0 selects the default
 * ofx_spmm_default_split(n); split_threshold == INT64_MAX (or `ordered` != 0) never splits,
 * which is exactly the reference composition's order.                                      */
/* Versioned structs (ofx_spmm_options, ofx_tensor_desc, ofx_placement) open with two tagged
 * words: struct_size = sizeof the struct as the CALLER was compiled, then magic =
 * OFX_STRUCT_MAGIC ("OFX1").  The library checks the tag FIRST and refuses (OFX_EINVAL) a struct
 * without it, before it trusts struct_size: an unversioned caller's first 8 bytes are data (the
 * round-4 options began with int64 split_threshold, whose low half would otherwise read as a
 * size), and no such layout holds the tag.  With the tag present, only the fields inside
 * struct_size are read and the rest take their defaults (a caller built against an older
 * versioned header keeps working); a size below the first tagged layout is refused.  Always
 * initialise with the OFX_*_INIT macros.                                                      */
#define OFX_STRUCT_MAGIC 0x4F465831u /* "OFX1" */

typedef struct ofx_spmm_options {
  uint32_t struct_size;    /* sizeof(ofx_spmm_options) as the CALLER was compiled (above)    */
  uint32_t magic;          /* OFX_STRUCT_MAGIC                                               */
  int64_t split_threshold; /* 0 = default                                                    */
  int64_t chunk;           /* 0 = same as split_threshold                                    */
  int32_t ordered;         /* != 0: never split (reference order, slower on hub rows)       */
  int32_t variant;         /* 0 = auto; >0 forces a kernel variant (tuning / tests)          */
  int64_t heavy_threshold; /* device work order: non-split rows are binned by degree (bins  *
                            * > t first, then the rest in index order;                       *
                            * t = this; 0 = auto (5x mean degree); < 0 = index order.  No    *
                            * numeric effect.                                                */
  int32_t planned;         /* != 0: the workspace already holds the work list that           *
                            * ofx_spmm_csr_plan built for this row_ptr (unchanged since),    *
                            * row range, m, n, nnz and options; the launch skips planning.   *
                            * Only for a static graph (the plan-once / compute-many pattern  *
                            * of a bound CSR).  No numeric effect.                           */
  int32_t reserved;        /* 0                                                              */
  int64_t range_nnz;       /* nonzeros of [row_begin, row_end) when the caller knows them    *
                            * (row_ptr[row_end] - row_ptr[row_begin]); 0 = estimated as      *
                            * nnz * rows / m.  Picks the kernel form only (launches of a few *
                            * rows of a degree-sorted graph); no numeric effect.             */
} ofx_spmm_options;
/* The first tagged layout ended at `reserved` (48 bytes); range_nnz came after it.            */
#define OFX_SPMM_OPTIONS_MIN_SIZE 48u
#define OFX_SPMM_OPTIONS_INIT \
  {(uint32_t)sizeof(ofx_spmm_options), OFX_STRUCT_MAGIC, 0, 0, 0, 0, 0, 0, 0, 0}

/* The default split threshold for dense width n (a fixed function of n; part of the numeric
 * contract).  Written out in DESIGN.md §3 and restated by oracle/oracle.py.                */
int64_t ofx_spmm_default_split(int64_t n);

/* Bytes of device workspace `ofx_spmm_csr` needs for this problem (upper bound, depends
 * only on shapes and options).  May be 0.                                                  */
int ofx_spmm_csr_workspace_size(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                                int64_t nnz, const ofx_spmm_options* opts, size_t* bytes);

/* C[r - row_begin, :] = sum_j values[j] * B[col_idx[j], :]  for r in [row_begin, row_end),
 *   j in [row_ptr[r], row_ptr[r+1]).
 *   row_ptr: idx_dtype[m+1]   col_idx: idx_dtype[nnz]   values: val_dtype[nnz]
 *   b: val_dtype, k rows of stride ldb (>= n)          c: val_dtype, rows of stride ldc (>= n)
 * All pointers are device pointers; `stream` is a hipStream_t (NULL = default stream).
 * Asynchronous; no allocation; no host synchronisation.  0 <= row_begin <= row_end <= m.   */
int ofx_spmm_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                 int64_t nnz, const void* row_ptr, const void* col_idx, const void* values,
                 const void* b, int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                 int64_t row_end, void* workspace, size_t workspace_bytes,
                 const ofx_spmm_options* opts);

/* ofx_spmm_csr with the values read through a permutation: nonzero j's value is
 * values[values_perm[j]] (values_perm: idx_dtype[nnz], device).  The backward's
 * d(b) = A^T @ d(out) runs on A^T's structure (ofx_csr_transpose) with A's values and the
 * transpose's `perm`, so the gathered copy values[perm] (ofx_gather_values) is never written.
 * Same bits as ofx_spmm_csr on the gathered values; same workspace.                        */
int ofx_spmm_csr_gathered(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                          int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                          const void* values, const void* values_perm, const void* b,
                          int64_t ldb, void* c, int64_t ldc, int64_t row_begin, int64_t row_end,
                          void* workspace, size_t workspace_bytes, const ofx_spmm_options* opts);

/* Plans rows [row_begin, row_end) into `workspace` (the hub chunks and degree-binned work list
 * every ofx_spmm_csr launch otherwise builds first: one small kernel over row_ptr), so that
 * launches with opts->planned != 0 on the same row_ptr, range, shapes and options skip it.
 * Asynchronous on `stream`; the same workspace size as ofx_spmm_csr.  A problem that needs no
 * plan (workspace size 0) is a no-op.  No reference counterpart (OneFlow re-plans per call); the
 * pattern is cuSPARSE's SpMM_preprocess.                                                     */
int ofx_spmm_csr_plan(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                      int64_t nnz, const void* row_ptr, int64_t row_begin, int64_t row_end,
                      void* workspace, size_t workspace_bytes, const ofx_spmm_options* opts);

/* The configuration ofx_spmm_csr with these arguments would launch, as text in buf
 * ("form=<small|mid|narrow|prefetch|bandwidth> kernel=... VEC=.. LPR=.. U=.. ..."): the form
 * rules of the launch made observable.  Nothing is launched and no pointer is
 * dereferenced (b and c only enter the width dispatch's alignment checks).  No reference
 * counterpart (OneFlow logs no kernel configuration).                                        */
int ofx_spmm_csr_describe(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                          int64_t nnz, const void* b, int64_t ldb, const void* c, int64_t ldc,
                          int64_t row_begin, int64_t row_end, const ofx_spmm_options* opts,
                          char* buf, size_t buf_bytes);

/* Bounds-checked builds only (OFX_DEBUG_BOUNDS, `make -C of-spmm_amd debug`): every global access
 * of the forward kernels is checked against its launch's allocations before it is made, and an
 * access outside all of them is skipped and recorded.  Synchronises the device and copies the
 * first violation to out[8] = {violations, site (file tag * 100000 + line), address, bytes,
 * block, thread, launch tag, 0}; reset != 0 clears the record.  A release build returns
 * OFX_EUNSUPPORTED.  No reference counterpart (a debugging aid of this port).                  */
int ofx_debug_bounds_read(uint64_t* out, int reset);

/* Fused epilogue: out = act(A @ B + bias), bit-identical to the
 * composition spmm_csr -> bias_add (BroadcastElementwiseBinary kAdd over axis 1,
 * oneflow/user/kernels/bias_add_kernel.cpp:25-53) -> relu (UnaryFunctor<kRelu>,
 * oneflow/core/ep/common/primitive/unary_functor.h:146-156): the row sum is rounded to T,
 * the bias added in the accumulation type and rounded to T again, relu maps x <= 0 to +0.
 * `bias` is T[n] on the device or NULL; `activation` is OFX_ACT_*.  Same workspace as
 * ofx_spmm_csr.                                                                             */
#define OFX_ACT_NONE 0
#define OFX_ACT_RELU 1
int ofx_spmm_csr_fused(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                       int64_t nnz, const void* row_ptr, const void* col_idx, const void* values,
                       const void* b, int64_t ldb, void* c, int64_t ldc, int64_t row_begin,
                       int64_t row_end, const void* bias, int activation, void* workspace,
                       size_t workspace_bytes, const ofx_spmm_options* opts);
int ofx_spmm_csr_fused_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                           int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                           const void* values, const void* b, int64_t ldb, void* c, int64_t ldc,
                           int64_t row_begin, int64_t row_end, const void* bias, int activation,
                           const ofx_spmm_options* opts);

/* Device-side structural check of a CSR (row_ptr monotone, row_ptr[0]==0, row_ptr[m]==nnz,
 * 0 <= col < k).  Writes a 32-bit error code to *flag_dev (0 = ok, 1 = bad row_ptr,
 * 2 = column out of range) asynchronously on `stream`.                                     */
int ofx_csr_validate(void* stream, int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                     const void* row_ptr, const void* col_idx, void* flag_dev);

/* CPU kernel (DeviceType::kCPU).  Same arguments and the same bits as ofx_spmm_csr, host
 * pointers, synchronous; num_threads <= 0 uses OMP_NUM_THREADS / all cores.              */
int ofx_spmm_csr_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                     int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                     const void* values, const void* b, int64_t ldb, void* c, int64_t ldc,
                     int64_t row_begin, int64_t row_end, const ofx_spmm_options* opts);

/* ---- gradient building blocks ---------------------------------------
 * For C = A @ B:  dB = A^T @ dC  (transpose once per graph, gather A's values through `perm`,
 * then ofx_spmm_csr on A^T)  and  dvalues = SDDMM(dC, B) on A's sparsity pattern.
 * Transpose: out_row_ptr I[k+1], out_col_idx I[nnz] (= row ids of A), out_perm I[nnz] (A^T's
 * t-th nonzero is A's nonzero perm[t]); entries of each A^T row in ascending A-row order
 * (stable), so dB follows the forward accumulation contract.  Device version needs a workspace
 * (nnz <= 2^31-1).                                                                          */
int ofx_csr_transpose_workspace_size(int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                                     size_t* bytes);
int ofx_csr_transpose(void* stream, int idx_dtype, int64_t m, int64_t k, int64_t nnz,
                      const void* row_ptr, const void* col_idx, void* out_row_ptr,
                      void* out_col_idx, void* out_perm, void* workspace, size_t workspace_bytes);
int ofx_csr_transpose_cpu(int idx_dtype, int64_t m, int64_t k, int64_t nnz, const void* row_ptr,
                          const void* col_idx, void* out_row_ptr, void* out_col_idx,
                          void* out_perm);
/* dst[t] = src[perm[t]] for t < nnz (any 2/4/8-byte value dtype). */
int ofx_gather_values(void* stream, int idx_dtype, int val_dtype, int64_t nnz, const void* perm,
                      const void* src, void* dst);
/* Host version (CPU kernel of spmm_csr_gathered). */
int ofx_gather_values_host(int idx_dtype, int val_dtype, int64_t nnz, const void* perm,
                           const void* src, void* dst);
/* out[j] = sum_n a[r - row_begin, n] * b[col_idx[j], n] for the nonzeros j of rows
 * r in [row_begin, row_end).  Order: products rounded, 8-element leaves summed sequentially from
 * +0, leaves (zero-padded to a power of two) added pairwise; fp32 accumulation for 16-bit types.
 * n <= 131072 (beyond 2048 the leaves are processed in 256-leaf tiles whose pairwise trees are
 * added pairwise: the same order).  Asynchronous, workspace from ofx_sddmm_csr_workspace_size. */
int ofx_sddmm_csr_workspace_size(int idx_dtype, int val_dtype, int64_t m, int64_t n, int64_t nnz,
                                 size_t* bytes);
int ofx_sddmm_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                  int64_t nnz, const void* row_ptr, const void* col_idx, const void* a,
                  int64_t lda, const void* b, int64_t ldb, void* out, int64_t row_begin,
                  int64_t row_end, void* workspace, size_t workspace_bytes);
/* ofx_sddmm_csr with options (NULL: defaults); only `planned` is read: the workspace already
 * holds the plan ofx_sddmm_csr_plan built for this row_ptr (contents unchanged), row range and
 * n, so the launch skips the planner kernel (the static-CSR path of op "sddmm_csr").          */
int ofx_sddmm_csr_ex(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t n,
                     int64_t nnz, const void* row_ptr, const void* col_idx, const void* a,
                     int64_t lda, const void* b, int64_t ldb, void* out, int64_t row_begin,
                     int64_t row_end, void* workspace, size_t workspace_bytes,
                     const ofx_spmm_options* opts);
int ofx_sddmm_csr_plan(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t n,
                       int64_t nnz, const void* row_ptr, int64_t row_begin, int64_t row_end,
                       void* workspace, size_t workspace_bytes);
int ofx_sddmm_csr_cpu(int num_threads, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                      int64_t n, int64_t nnz, const void* row_ptr, const void* col_idx,
                      const void* a, int64_t lda, const void* b, int64_t ldb, void* out,
                      int64_t row_begin, int64_t row_end);

/* ---- COO (edge_index) -> CSR -----------------------------------------
 * Canonical CSR from COO pairs: rows ascending, columns ascending; with merge_duplicates != 0,
 * equal (row, col) entries become one whose value is their sum in input order (fp32 accumulation
 * for 16-bit types), else duplicates are kept in input order.  values/out_values may both be
 * NULL (structure only).  out_nnz: device int64 scalar (host int64* for the CPU version);
 * bad_flag (device uint32, may be NULL) is set non-zero if an entry lies outside m x k.
 * Outputs must hold nnz entries (the upper bound).  Device version: nnz < 2^31.            */
int ofx_coo_to_csr_workspace_size(int idx_dtype, int64_t m, int64_t k, int64_t nnz, size_t* bytes);
int ofx_coo_to_csr(void* stream, int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t nnz,
                   const void* row, const void* col, const void* values, int merge_duplicates,
                   void* out_row_ptr, void* out_col_idx, void* out_values, void* out_nnz,
                   void* bad_flag, void* workspace, size_t workspace_bytes);
int ofx_coo_to_csr_cpu(int idx_dtype, int val_dtype, int64_t m, int64_t k, int64_t nnz,
                       const void* row, const void* col, const void* values, int merge_duplicates,
                       void* out_row_ptr, void* out_col_idx, void* out_values, int64_t* out_nnz);

/* ---- fused-epilogue backward ------------------------------------------
 * For y = relu?(A @ b + bias?):  dx = relu ? (y > 0 ? dy : 0) : dy   (ReluGrad from the output,
 * oneflow/core/autograd/gradient_funcs/activation.cpp:195-205) and d_bias[j] = sum_i dx[i, j]
 * (bias_add grad, gradient_funcs/bias_add.cpp:62), in one pass.  dx may be NULL (only d_bias),
 * d_bias may be NULL (only dx).  Column-sum order (identical on CPU and GPU): chunks of 2048 rows
 * summed in row order from +0 in the accumulation type; chunk partials in 8 interleaved lanes
 * (lane l: chunks l, l+8, ...), lanes combined ((l0+l4)+(l2+l6))+((l1+l5)+(l3+l7)); one rounding. */
int ofx_relu_bias_grad_workspace_size(int val_dtype, int64_t m, int64_t n, size_t* bytes);
int ofx_relu_bias_grad(void* stream, int val_dtype, int64_t m, int64_t n, const void* y,
                       int64_t ldy, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                       void* d_bias, int relu, void* workspace, size_t workspace_bytes);
int ofx_relu_bias_grad_cpu(int num_threads, int val_dtype, int64_t m, int64_t n, const void* y,
                           int64_t ldy, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                           void* d_bias, int relu);

/* ---- row partition (BalancedSplitter) ---------------------------------------------------- */
int ofx_balanced_range(int64_t total, int64_t parts, int64_t idx, int64_t* begin, int64_t* end);
/* Rebase a row slice of a CSR: out_row_ptr[i] = row_ptr[row_begin + i] - row_ptr[row_begin],
 * i in [0, row_end-row_begin]; returns nnz offset/count.  Device version (async).          */
int ofx_csr_row_slice(void* stream, int idx_dtype, const void* row_ptr, int64_t row_begin,
                      int64_t row_end, void* out_row_ptr);
int ofx_csr_row_slice_host(int idx_dtype, const void* row_ptr, int64_t row_begin,
                           int64_t row_end, void* out_row_ptr, int64_t* nnz_begin,
                           int64_t* nnz_end);

/* ---- thin device layer (ep::Device / ep::Stream / ep::Event / primitives) --------------- */
int ofx_device_count(int* count);
int ofx_set_device(int device);
int ofx_get_device(int* device);
int ofx_device_synchronize(void);
int ofx_malloc(void** ptr, size_t bytes);       /* 512-B aligned (ep::kMaxAlignmentRequirement) */
int ofx_free(void* ptr);
int ofx_host_malloc(void** ptr, size_t bytes);  /* pinned */
int ofx_host_free(void* ptr);
int ofx_stream_create(void** stream);
int ofx_stream_destroy(void* stream);
int ofx_stream_sync(void* stream);
#define OFX_MEMCPY_H2D 1
#define OFX_MEMCPY_D2H 2
#define OFX_MEMCPY_D2D 3
#define OFX_MEMCPY_DEFAULT 4
int ofx_memcpy_async(void* stream, void* dst, const void* src, size_t bytes, int kind);
int ofx_memset_async(void* stream, void* dst, int value, size_t bytes);
int ofx_event_create(void** event, int timing);
int ofx_event_destroy(void* event);
int ofx_event_record(void* event, void* stream);
int ofx_event_sync(void* event);
int ofx_event_elapsed_ms(void* start, void* end, float* ms);
int ofx_stream_wait_event(void* stream, void* event);
/* hipGraph executable and stream capture: ep::CudaGraphExecutable (ep/cuda/cuda_stream.h:41-56,
 * cuda_stream.cpp:49-80) and CudaStream::BeginGraphCapture / EndGraphCapture / IsGraphCapturing /
 * LaunchGraph (cuda_stream.cpp:178-196).  end_capture updates a live executable in place
 * (hipGraphExecUpdate) and re-instantiates only when the update is refused; exec == NULL
 * discards the capture.  Capture mode is thread-local, as the reference's.                   */
int ofx_graph_exec_create(void** exec);
int ofx_graph_exec_destroy(void* exec);
int ofx_graph_exec_stats(void* exec, int* instantiated, int64_t* instantiations, int64_t* updates,
                         int64_t* launches);
int ofx_stream_begin_capture(void* stream);
int ofx_stream_is_capturing(void* stream, int* capturing);
int ofx_stream_end_capture(void* stream, void* exec);
int ofx_graph_launch(void* exec, void* stream);

/* ---- RCCL all-gather (ccl::AllGather) ---------------------------------------------------- */
#define OFX_UNIQUE_ID_BYTES 128
int ofx_comm_get_unique_id(void* uid_out /* OFX_UNIQUE_ID_BYTES */);
int ofx_comm_init_rank(void** comm, int nranks, const void* uid, int rank);
/* ofx_comm_init_rank with a deadline: a non-blocking communicator (ncclCommInitRankConfig with
 * config.blocking = 0) whose set-up is polled (ncclCommGetAsyncError); if a peer has not joined
 * within timeout_s seconds the communicator is aborted (ncclCommAbort) and OFX_ECOMM returned
 * with the wait named.  Every later call on it (all-gathers, send/recv groups, finalize) is
 * bounded by the same timeout and aborts the communicator when it expires.  Replaces the
 * unbounded EagerNcclCommMgr::CreateNcclComm (eager_nccl_comm_manager.cpp:57-80).           */
int ofx_comm_init_rank_deadline(void** comm, int nranks, const void* uid, int rank,
                                double timeout_s);
/* This communicator's deadlines: call_timeout_s bounds a call left in progress (<= 0 keeps it);
 * device_timeout_s > 0 makes every exchange on it (all-gathers, send/recv groups) wait for its
 * completion on the device for at most that long, then abort the communicator and return
 * OFX_ECOMM naming the exchange (a peer that never joins otherwise leaves the stream stuck with
 * no host call to time out); 0 keeps exchanges asynchronous.  Not waited for during a capture.  */
int ofx_comm_set_timeouts(void* comm, double call_timeout_s, double device_timeout_s);
/* ncclCommAbort: drops the communicator's pending operations so that peers waiting on this rank
 * fail too (a rank's watchdog calls it before exiting).  The handle stays valid: every later call
 * on it returns OFX_ECOMM; ofx_comm_destroy frees it. */
int ofx_comm_abort(void* comm);
/* ncclCommFinalize (waited for) + ncclCommDestroy; an aborted communicator's handle is only freed,
 * and one whose finalize fails is aborted rather than leaked. */
int ofx_comm_destroy(void* comm);
/* ncclCommCount / ncclCommUserRank of a communicator. */
int ofx_comm_count(void* comm, int* nranks, int* rank);
/* out[r*count .. (r+1)*count) = in of rank r; count in elements of dtype. */
int ofx_allgather(void* stream, const void* in, void* out, size_t count, int dtype, void* comm);
/* The same all-gather as grouped point-to-point send/recv with every peer (in place: this
 * rank's slot of `buf` is the send buffer).  Same result bytes as ofx_allgather.           */
int ofx_allgather_p2p(void* stream, void* buf, size_t count, int dtype, void* comm);
/* ---- the pull form of the same all-gather (peer reads over xGMI) ------------
 * Every rank's gathered buffer has one layout, so a rank can read each peer's slot straight out
 * of the peer's buffer (IPC-mapped) into its own.  Replaces ncclAllGather's ring
 * (cuda_all_gather.cpp:25-47) as a tune() candidate; same result bytes.
 * ofx_peer_export: IPC handle (OFX_PEER_HANDLE_BYTES) of the allocation holding `ptr`, with the
 *   offset of ptr in it.  ofx_peer_open maps a peer's handle (a handle opened twice maps once,
 *   reference-counted); ofx_peer_close unmaps a pointer ofx_peer_open returned.
 * ofx_peer_publish: system-scope release on every XCD, stream-ordered: this rank's earlier
 *   stores reach HBM, where peers' reads find them.
 * ofx_peer_pull: for every peer p != rank, bytes [p*slot_bytes, (p+1)*slot_bytes) of
 *   peer_bufs[p] (peer p's buffer, mapped) into the same bytes of buf; peer_bufs[rank] unused.
 *   The caller orders it: every peer's slot written and published before (a barrier), no peer
 *   rewrites its slot until every rank's pull is done (a second barrier).
 * ofx_peer_pull_host: the same tile plan over host memory (tests).
 * ofx_allgather_pull: the composed exchange on a communicator: publish, a stream-ordered RCCL
 *   barrier (1-element all-reduce), pull, barrier; count elements per slot as ofx_allgather_p2p
 *   (in place: this rank's slot of buf is already written).                                   */
#define OFX_PEER_HANDLE_BYTES 96
#define OFX_PEER_MAX_RANKS 16
int ofx_peer_export(const void* ptr, void* handle_out);
int ofx_peer_open(const void* handle, void** ptr_out);
int ofx_peer_close(void* ptr);
int ofx_peer_publish(void* stream);
int ofx_peer_pull(void* stream, int nranks, int rank, const void* const* peer_bufs, void* buf,
                  uint64_t slot_bytes);
int ofx_peer_pull_host(int nranks, int rank, const void* const* peer_bufs, void* buf,
                       uint64_t slot_bytes);
int ofx_allgather_pull(void* stream, void* comm, const void* const* peer_bufs, void* buf,
                       size_t count, int dtype);
/* One row-split step on this rank: in-place all-gather of the padded B shards
 * in b_gathered [k_padded, n] (k_padded = ranks * P; this rank's rows already at
 * [rank * P, rank * P + K_r)), then the local SpMM of this rank's m_local rows (row_ptr rebased
 * to 0, columns remapped by ofx_padded_owner_remap).  `workspace` as ofx_spmm_csr for
 * (m_local, k_padded, n, nnz_local).                                                         */
int ofx_spmm_rowsplit(void* stream, void* comm, int idx_dtype, int val_dtype, int64_t m_local,
                      int64_t k_padded, int64_t n, int64_t nnz_local, const void* row_ptr,
                      const void* col_idx, const void* values, void* b_gathered, void* c,
                      int64_t ldc, void* workspace, size_t workspace_bytes,
                      const ofx_spmm_options* opts);
/* Column c of B -> its row in the padded gathered buffer: c + max(owner(c) - k % world, 0)
 * when k % world > 0, c otherwise; owner from BalancedSplitter(k, world)
 * (oneflow/core/common/balanced_splitter.cpp:20-40).                                         */
int ofx_padded_owner_remap(void* stream, int idx_dtype, int64_t nnz, int64_t k, int64_t world,
                           const void* col_in, void* col_out);
/* Halo exchange: grouped send/recv of B rows with per-peer counts, the
 * ShuffleData pattern of oneflow/user/kernels/data_shuffle_kernel.cu:119-135.  Counts and
 * offsets are in rows of n elements (host arrays, one entry per rank); this rank's entry and
 * zero counts are skipped.                                                                  */
int ofx_exchange_rows(void* stream, void* comm, int dtype, int64_t n, const void* send_buf,
                      const int64_t* send_counts, const int64_t* send_offsets, void* recv_buf,
                      const int64_t* recv_counts, const int64_t* recv_offsets);
/* Row gather on the device: dst[i, :] = src[idx[i], :] for i < count, rows of row_bytes bytes,
 * strides in bytes (packs the halo rows a peer requested into one send buffer).  idx == NULL
 * is the identity: a strided 2-D copy (column-block packing of the N-split exchange).        */
/* 3-level strided block copy on the device, strides in bytes: for o < nouter, i < ninner,
 * r < rows, row_bytes from src + o*src_outer + i*src_inner + r*src_row to the same position in
 * dst's strides.  One launch packs a B shard into the grid exchange's column blocks (and
 * unpacks the returned C blocks); replaces per-block ofx_gather_rows calls.                  */
int ofx_copy_blocks(void* stream, int64_t nouter, int64_t ninner, int64_t rows, int64_t row_bytes,
                    const void* src, int64_t src_outer, int64_t src_inner, int64_t src_row,
                    void* dst, int64_t dst_outer, int64_t dst_inner, int64_t dst_row);
int ofx_gather_rows(void* stream, int idx_dtype, int64_t count, int64_t row_bytes,
                    const void* idx, const void* src, int64_t src_stride_bytes, void* dst,
                    int64_t dst_stride_bytes);

/* ---- synthetic power-law CSR (deterministic, counter-based) ---------------- */
/* row_ptr_out: int64[m+1].  Degrees of a Chung–Lu power law (exponent gamma), rows permuted. */
int ofx_synth_row_ptr(int64_t m, int64_t k, int64_t nnz, double gamma, uint64_t seed,
                      int64_t* row_ptr_out);
/* Columns for rows [row_begin,row_end) written at col_out[row_ptr[r]-row_ptr[row_begin] ...],
 * sorted ascending and unique per row.  idx_dtype int32/int64.  Host, OpenMP.              */
int ofx_synth_columns(int64_t m, int64_t k, double gamma, uint64_t seed, const int64_t* row_ptr,
                      int64_t row_begin, int64_t row_end, int idx_dtype, void* col_out,
                      int num_threads);
/* values[j - j_begin] for global nonzero ids j in [j_begin, j_end): U[-1,1) or exact-mode. */
int ofx_synth_values_host(int val_dtype, int64_t j_begin, int64_t j_end, uint64_t seed, int exact,
                          void* out);
/* Dense rows [r_begin, r_end) of a k x n matrix with leading dim ld, on the device. */
int ofx_synth_dense(void* stream, int val_dtype, int64_t r_begin, int64_t r_end, int64_t n,
                    int64_t ld, uint64_t seed, int exact, void* out);
int ofx_synth_dense_host(int val_dtype, int64_t r_begin, int64_t r_end, int64_t n, int64_t ld,
                         uint64_t seed, int exact, void* out);

/* ---- functional entry (Python binding -> C++ op/kernel registry -> device kernel) ------- */
/* A tensor as the functional layer sees it: dtype code, device (-1 = CPU, >=0 HIP ordinal),
 * rank-1/2 shape, row stride (elements) for rank-2, data pointer.                          */
typedef struct ofx_tensor_desc {
  uint32_t struct_size; /* sizeof(ofx_tensor_desc) as the caller was compiled (checked, as in   *
                         * ofx_spmm_options; OFX_TENSOR_DESC_INIT)                              */
  uint32_t magic;       /* OFX_STRUCT_MAGIC                                                     */
  int32_t dtype;
  int32_t device;
  int32_t ndim;
  int32_t reserved;     /* 0                                                                    */
  int64_t shape[2];
  int64_t stride[2];
  void* data;
} ofx_tensor_desc;
#define OFX_TENSOR_DESC_MIN_SIZE 64u
#define OFX_TENSOR_DESC_INIT \
  {(uint32_t)sizeof(ofx_tensor_desc), OFX_STRUCT_MAGIC, 0, 0, 0, 0, {0, 0}, {0, 0}, 0}
/* Shape/dtype inference of op "spmm_csr" (oneflow/user/ops/spmm_op.cpp mirror). Fills
 * out->dtype/ndim/shape; returns OFX_EINVAL with the op's error message on mismatch.      */
int ofx_functional_spmm_csr_infer(const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
                                  const ofx_tensor_desc* values, int64_t a_num_rows,
                                  int64_t a_num_cols, const ofx_tensor_desc* b,
                                  ofx_tensor_desc* out);
/* Runs the registered kernel for (op "spmm_csr", out->device's device type, dtype) on
 * `stream` with a caller-provided tmp buffer (size: ofx_functional_spmm_csr_tmp_size).     */
int ofx_functional_spmm_csr_tmp_size(const ofx_tensor_desc* row_ptr,
                                     const ofx_tensor_desc* col_idx,
                                     const ofx_tensor_desc* values, int64_t a_num_rows,
                                     int64_t a_num_cols, const ofx_tensor_desc* b,
                                     size_t* bytes);
int ofx_functional_spmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                            const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                            int64_t a_num_rows, int64_t a_num_cols, const ofx_tensor_desc* b,
                            ofx_tensor_desc* out, void* tmp, size_t tmp_bytes);
/* Global form on one rank of a placement: the op's physical inference gives this rank's out
 * shape and the kernel's OpKernelCache its row range, both from the hierarchy and out's NdSbp
 * (GetPhysicalShape, oneflow/core/operator/operator.cpp:1551-1626; GetTensorSliceView4ParallelId,
 * oneflow/core/job/nd_sbp_util.cpp:58-104, as oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:
 * 59-78 uses it).  hierarchy: hierarchy_ndim dims (e.g. {8} or {2, 4}); out_split_axes: per
 * hierarchy axis, out's split axis (0 = rows, 1 = columns, -1 = broadcast); b's NdSbp follows (B
 * for a row split, S(1) for a column split).  `b` and `out` are this rank's physical tensors;
 * b_logical_cols is the logical N (-1: b's own width).  The hub-row schedule is that of the
 * logical N, so every rank's bits equal the matching slice of the single-device result.
 * tmp_size_out != NULL: only the tmp size is computed.  num_threads: CPU kernel only.       */
int ofx_functional_spmm_csr_global(void* stream, const ofx_tensor_desc* row_ptr,
                                   const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                                   int64_t a_num_rows, int64_t a_num_cols, const ofx_tensor_desc* b,
                                   int64_t b_logical_cols, ofx_tensor_desc* out, void* tmp,
                                   size_t tmp_bytes, int hierarchy_ndim, const int64_t* hierarchy,
                                   const int32_t* out_split_axes, int64_t parallel_id,
                                   int num_threads, size_t* tmp_size_out);
/* Op attributes of "spmm_csr" beyond a_num_rows / a_num_cols (a tagged, versioned struct as
 * ofx_spmm_options; OFX_SPMM_ATTRS_INIT).
 *   static_csr: attr `static_csr` (SI64, default 0).  Non-zero promises that the CSR at these
 *     addresses (row_ptr above all) is not rewritten while the op instance lives; the value is
 *     part of the plan's key, so a caller that frees a static CSR and builds another one at the
 *     same addresses gives it a new value.  The HIP kernel's OpKernelState
 *     (OpKernel::CreateOpKernelState, oneflow/core/framework/op_kernel.h:292) then keeps the
 *     work-list plan in a device workspace of its own, keyed on (static_csr, row_ptr's address,
 *     m, k, n, nnz, row range, dtypes, schedule, stream), and later calls launch with
 *     options.planned = 1: the planner kernel runs once per static CSR instead of once per call.
 *     The first call of a key allocates and plans (not while the stream is capturing a graph:
 *     such a call takes the ordinary path through the tmp buffer); at most 8 plans per state,
 *     least recently used evicted.  No numeric effect; the kCPU kernel has no plan and ignores
 *     it.  The eager entries below hold one state per (kernel registration, device), as
 *     OneFlow's functor keeps one StatefulOpKernel per op expression and device.            */
typedef struct ofx_spmm_attrs {
  uint32_t struct_size; /* sizeof(ofx_spmm_attrs) as the caller was compiled                     */
  uint32_t magic;       /* OFX_STRUCT_MAGIC                                                      */
  int64_t static_csr;   /* 0 = plan every call (default)                                         */
} ofx_spmm_attrs;
#define OFX_SPMM_ATTRS_MIN_SIZE 16u
#define OFX_SPMM_ATTRS_INIT {(uint32_t)sizeof(ofx_spmm_attrs), OFX_STRUCT_MAGIC, 0}
/* ofx_functional_spmm_csr_global with the op's attributes (attrs == NULL: every default).  */
int ofx_functional_spmm_csr_global_attrs(
    void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
    const ofx_tensor_desc* values, int64_t a_num_rows, int64_t a_num_cols,
    const ofx_tensor_desc* b, int64_t b_logical_cols, ofx_tensor_desc* out, void* tmp,
    size_t tmp_bytes, int hierarchy_ndim, const int64_t* hierarchy, const int32_t* out_split_axes,
    int64_t parallel_id, int num_threads, size_t* tmp_size_out, const ofx_spmm_attrs* attrs);
/* The static-CSR plans the eager op states hold, summed over devices: live entries, plans built
 * (planner launches) and calls that reused a plan.  A state keeps at most 8 plans, evicting the
 * least recently used, except plans a graph capture used: a captured graph holds their pointer,
 * so they stay until released.  release != 0 first frees every entry's workspace (after a device
 * synchronisation), captured ones included: destroy those graphs first.                        */
int ofx_spmm_static_plans(int64_t* entries, int64_t* plans, int64_t* hits, int release);

/* 1-D shorthand of ofx_functional_spmm_csr_global: hierarchy {parallel_num}, out split on
 * out_split_axis (0 or -1; a column split needs the logical width, so it takes the _global form).
 * 2-D tensors must have unit column stride (refused with OFX_EINVAL otherwise).            */
int ofx_functional_spmm_csr_ex(void* stream, const ofx_tensor_desc* row_ptr,
                               const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                               int64_t a_num_rows, int64_t a_num_cols, const ofx_tensor_desc* b,
                               ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                               int64_t parallel_id, int64_t parallel_num, int out_split_axis,
                               int num_threads);
/* Op "fused_spmm_csr" (relu?(A @ b + bias?), oneflow/user/ops/fused_spmm_op.cpp mirror) through
 * the op-registry dispatch; bias may be NULL (optional input absent).  With tmp_size_out !=
 * NULL only the tmp-buffer size is computed (nothing runs).                                  */
int ofx_functional_fused_spmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                                  const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                                  const ofx_tensor_desc* b, const ofx_tensor_desc* bias,
                                  int64_t a_num_rows, int64_t a_num_cols, int relu,
                                  ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                                  size_t* tmp_size_out);
/* ofx_functional_fused_spmm_csr with the op's other attributes (attrs == NULL: every default);
 * static_csr keeps the work-list plan in the eager op's kernel state, as for spmm_csr.          */
int ofx_functional_fused_spmm_csr_attrs(void* stream, const ofx_tensor_desc* row_ptr,
                                        const ofx_tensor_desc* col_idx,
                                        const ofx_tensor_desc* values, const ofx_tensor_desc* b,
                                        const ofx_tensor_desc* bias, int64_t a_num_rows,
                                        int64_t a_num_cols, int relu, ofx_tensor_desc* out,
                                        void* tmp, size_t tmp_bytes, size_t* tmp_size_out,
                                        const ofx_spmm_attrs* attrs);
/* Gradient functors (ops "sddmm_csr", "csr_transpose"; oneflow/user/ops/sddmm_op.cpp) through
 * the same op-registry dispatch.  With tmp_size_out != NULL only the tmp-buffer size is
 * computed (nothing runs).  Outputs: sddmm out [nnz] in b's dtype; transpose out_row_ptr [k+1],
 * out_col_idx [nnz], out_perm [nnz] in the index dtype.                                      */
int ofx_functional_sddmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                             const ofx_tensor_desc* col_idx, const ofx_tensor_desc* a,
                             const ofx_tensor_desc* b, int64_t a_num_rows, int64_t a_num_cols,
                             ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                             size_t* tmp_size_out);
/* ofx_functional_sddmm_csr with the op's other attributes (attrs == NULL: defaults): static_csr
 * keeps the SDDMM's plan of an unchanged CSR in the eager op's kernel state.                  */
int ofx_functional_sddmm_csr_attrs(void* stream, const ofx_tensor_desc* row_ptr,
                                   const ofx_tensor_desc* col_idx, const ofx_tensor_desc* a,
                                   const ofx_tensor_desc* b, int64_t a_num_rows,
                                   int64_t a_num_cols, ofx_tensor_desc* out, void* tmp,
                                   size_t tmp_bytes, size_t* tmp_size_out,
                                   const ofx_spmm_attrs* attrs);
int ofx_functional_csr_transpose(void* stream, const ofx_tensor_desc* row_ptr,
                                 const ofx_tensor_desc* col_idx, int64_t a_num_rows,
                                 int64_t a_num_cols, ofx_tensor_desc* out_row_ptr,
                                 ofx_tensor_desc* out_col_idx, ofx_tensor_desc* out_perm,
                                 void* tmp, size_t tmp_bytes, size_t* tmp_size_out);
/* functional::SpmmCsrGathered: op "spmm_csr_gathered" (out = A @ b with values read through
 * values_perm; the d(b) gradient with learnable values). */
int ofx_functional_spmm_csr_gathered(void* stream, const ofx_tensor_desc* row_ptr,
                                     const ofx_tensor_desc* col_idx,
                                     const ofx_tensor_desc* values,
                                     const ofx_tensor_desc* values_perm, const ofx_tensor_desc* b,
                                     int64_t a_num_rows, int64_t a_num_cols, ofx_tensor_desc* out,
                                     void* tmp, size_t tmp_bytes, size_t* tmp_size_out);
/* ofx_functional_spmm_csr_gathered with the op's other attributes (attrs == NULL: defaults):
 * static_csr keeps the plan of an unchanged A^T in the eager op's kernel state.               */
int ofx_functional_spmm_csr_gathered_attrs(void* stream, const ofx_tensor_desc* row_ptr,
                                           const ofx_tensor_desc* col_idx,
                                           const ofx_tensor_desc* values,
                                           const ofx_tensor_desc* values_perm,
                                           const ofx_tensor_desc* b, int64_t a_num_rows,
                                           int64_t a_num_cols, ofx_tensor_desc* out, void* tmp,
                                           size_t tmp_bytes, size_t* tmp_size_out,
                                           const ofx_spmm_attrs* attrs);
/* The op's registered SBP signatures and no-grad inputs, as text (tests / introspection). */
int ofx_op_spmm_csr_sbp_signatures(char* buf, size_t len);
/* Same for any registered op; optional_inputs = comma-separated optional inputs present.   */
int ofx_op_sbp_signatures(const char* op_name, const char* optional_inputs, char* buf, size_t len);

/* ---- collectives of the OneFlow mirror and the lazy path ------------------------------------
 * The control plane a host passes in (OneFlow's CtrlClient KV store and ring transport, which
 * this library does not reimplement): push/pull of the RCCL unique id under a key
 * (EagerNcclCommMgr, oneflow/core/job/eager_nccl_comm_manager.cpp:57-131) and one ring step of
 * the kCPU all-gather (collective_communication/cpu/cpu_all_gather.cpp:27-80).  Callbacks return
 * 0 on success; pull blocks until the key exists and stores the value's length in *len.        */
typedef int (*ofx_kv_push_fn)(void* user, const char* key, const void* val, size_t len);
typedef int (*ofx_kv_pull_fn)(void* user, const char* key, void* val, size_t cap, size_t* len);
typedef int (*ofx_sendrecv_fn)(void* user, const void* send, size_t send_bytes, int64_t to,
                               void* recv, size_t recv_bytes, int64_t from);
int ofx_process_ctx_init(int64_t rank, int64_t world, ofx_kv_push_fn push, ofx_kv_pull_fn pull,
                         ofx_sendrecv_fn sendrecv, void* user);

/* A placement (oneflow/core/job/parallel_desc.h): device type (OFX_DEV_*), parallel_num devices,
 * this process's parallel_id, and per parallel id its machine (= process rank) and local device
 * (NULL arrays: parallel id p is machine p, device p).                                          */
#define OFX_DEV_CPU 1
#define OFX_DEV_HIP 4
typedef struct ofx_placement {
  uint32_t struct_size; /* sizeof(ofx_placement) as the caller was compiled (checked, as in     *
                         * ofx_spmm_options; OFX_PLACEMENT_INIT)                                */
  uint32_t magic;       /* OFX_STRUCT_MAGIC                                                     */
  int32_t device_type;
  int32_t reserved;     /* 0                                                                    */
  int64_t parallel_num;
  int64_t parallel_id;
  const int64_t* machine_ids;
  const int64_t* device_ids;
} ofx_placement;
#define OFX_PLACEMENT_MIN_SIZE 48u
#define OFX_PLACEMENT_INIT {(uint32_t)sizeof(ofx_placement), OFX_STRUCT_MAGIC, 0, 0, 0, 0, 0, 0}
/* Whether ccl::AllGather and a ccl::CommunicationContext are registered for a device type
 * (REGISTER_COLLECTIVE_COMMUNICATION, collective_communication/include/all_gather.h:24-38). */
int ofx_ccl_registered(int device_type, int* all_gather, int* communication_context);
/* Eager boxing "ccl-s-to-b" (oneflow/core/boxing/ccl_boxing_function.cpp:104-122,185-215): the
 * check alone (OFX_OK or OFX_EINVAL with the failed condition; e.g. logical dim 0 % ranks != 0),
 * and the boxing of this rank's S(0) slice `in` into the full B tensor `out` through op
 * eager_ccl_all_gather and its registered kernel (RCCL on kHIP, host ring on kCPU).           */
int ofx_boxing_check_ccl_s2b(const ofx_placement* pl, int ndim, const int64_t* logical_shape,
                             const char* in_sbp, const char* out_sbp);
int ofx_boxing_ccl_s2b(void* stream, const ofx_placement* pl, const ofx_tensor_desc* in,
                       ofx_tensor_desc* out, int64_t logical_dim0);
/* Op "_nccl_logical_all_gather" (the lazy compiler's S(0) -> B) through its kHIP kernel
 * (reference kernel: oneflow/user/kernels/nccl_logical_kernels.cpp:175-205, kCUDA only).      */
int ofx_nccl_logical_all_gather(void* stream, const ofx_placement* pl, const ofx_tensor_desc* in,
                                ofx_tensor_desc* out, const char* stream_name);
/* InsertNcclLogicalOpPass's choice for one edge of a 1-D placement
 * (insert_nccl_logical_op_pass.cpp:150-240): the op type, or "" when none applies.            */
int ofx_insert_nccl_logical_op(const char* src_sbp, const char* dst_sbp, int ndim,
                               const int64_t* logical_shape, int64_t parallel_num, char* op_type,
                               size_t len);
/* The key EagerRcclCommMgr publishes a placement's unique id under, and the RCCL rank of
 * (machine, device) in it (-1 if absent).                                                      */
int ofx_rccl_comm_key(const ofx_placement* pl, const char* stream_name, int64_t machine,
                      int64_t device, char* key, size_t len, int* rank);
/* A compiled row-split spmm_csr job (the nn.Graph form of the layer): b (S(0), this rank's K/P
 * rows) -> _nccl_logical_all_gather -> b (B) -> spmm_csr (a_csr_*: B) -> out (S(0), this rank's
 * BalancedSplitter rows).  Create compiles once (every rank of the placement must call it: the
 * logical collective's RCCL communicator is created collectively on the first run); run is
 * stream-ordered launches only (hipGraph-capturable) with a caller tmp of the described size. */
int ofx_spmm_job_create(const ofx_placement* pl, int idx_dtype, int val_dtype, int64_t m, int64_t k,
                        int64_t n, int64_t nnz, const char* stream_name, void** job);
int ofx_spmm_job_describe(void* job, char* buf, size_t len, size_t* tmp_bytes);
int ofx_spmm_job_run(void* job, void* stream, const void* row_ptr, const void* col_idx,
                     const void* values, const void* b_shard, void* out, void* tmp,
                     size_t tmp_bytes);
int ofx_spmm_job_destroy(void* job);
/* Graph mode of a compiled job (UserKernel::ForwardUserKernel, core/kernel/user_kernel.cpp:
 * 676-707, with ONEFLOW_KERNEL_ENABLE_CUDA_GRAPH): the first run on a HIP placement is eager
 * (the logical all-gather creates its communicator then); the next is captured (on the job's
 * own stream) into a hipGraph that is launched on the caller's stream; a later run with the same
 * tensor addresses launches the graph, one with different ones re-captures (an in-place
 * executable update).  Host placements
 * ignore graph mode.  Stats: captures, launches of a captured graph without re-capture, and
 * captures that updated the executable in place.                                            */
int ofx_spmm_job_set_graph(void* job, int enable);
/* The compiled job's spmm_csr with attr static_csr (see ofx_spmm_attrs): the job's own kernel
 * state (as a lazy UserKernel owns its OpKernelState) keeps the plan of its row_ptr, so eager
 * runs and graph replays after the first launch no planner kernel.  0 turns it off (the
 * default).  Stats: plans built and runs that reused one.                                   */
int ofx_spmm_job_set_static(void* job, int64_t static_csr);
int ofx_spmm_job_static_stats(void* job, int64_t* plans, int64_t* hits);
int ofx_spmm_job_graph_stats(void* job, int64_t* captures, int64_t* replays, int64_t* updates);

#ifdef __cplusplus
}
#endif

#endif /* OFX_SPMM_H_ */
