/*
 * ccl_functor.cpp — C-ABI of the collective layer of the OneFlow mirror (include/ofx_spmm.h,
 * "collectives and the lazy path"): the host control plane, the eager S(0) -> B boxing through the
 * op/kernel registries (ccl_boxing_function.cpp), the lazy graph's logical all-gather, the
 * InsertNcclLogicalOpPass decision, and SpmmJob — a compiled row-split spmm_csr graph:
 *
 *     b (S(0), this rank's K/P rows) --_nccl_logical_all_gather--> b (B) --spmm_csr--> out (S(0))
 *
 * the job the lazy compiler builds for a row-split layer (spmm_csr's signature a_csr_*: B, b: B,
 * out: S(0); the pass inserts the logical collective on b's S(0) -> B edge,
 * insert_nccl_logical_op_pass.cpp:189-198).  Compile once (inference, kernel choice, kernel state
 * with the RCCL communicator, tmp layout), run many; every run is stream-ordered launches only,
 * so it captures into a hipGraph (the CUDA-graph mode of nn.Graph, user_kernel.cpp:676-707).
 */
#include <hip/hip_runtime.h>

#include <cstring>
#include <sstream>

#include "oneflow/core/boxing/ccl_boxing_function.h"
#include "oneflow/core/control/ctrl_client.h"
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/functional/spmm_functor.h"
#include "oneflow/core/job/eager_rccl_comm_manager.h"
#include "oneflow/core/job_rewriter/insert_nccl_logical_op_pass.h"
#include "oneflow/user/kernels/collective_communication/include/all_gather.h"
#include "ofx_internal.h"
#include "ofx_spmm.h"
#include "spmm_common.h"

namespace oneflow {
namespace {

int ToStatus(const Maybe<void>& m, int code = OFX_EINVAL) {
  if (m.IsOk()) return OFX_OK;
  return ofx::fail(m.kind() == "OpKernelNotFoundError" ? OFX_EUNSUPPORTED : code, "%s: %s",
                   m.kind().c_str(), m.message().c_str());
}

DeviceType DeviceOf(int32_t code) {
  switch (code) {
    case 1: return DeviceType::kCPU;
    case 4: return DeviceType::kHIP;
    default: return DeviceType::kInvalidDevice;
  }
}

Maybe<void> MakeParallelDesc(const ofx_placement* pl, ParallelDesc* pd) {
  CHECK_OR_RETURN(pl != nullptr) << Error::RuntimeError() << "NULL placement";
  const char* why = ofx::versioned_struct_problem(pl, OFX_PLACEMENT_MIN_SIZE);
  CHECK_OR_RETURN(why == nullptr)
      << Error::RuntimeError() << "ofx_placement " << why << " (" << OFX_PLACEMENT_MIN_SIZE
      << " bytes): initialise it with OFX_PLACEMENT_INIT";
  CHECK_OR_RETURN(pl->parallel_num >= 1 && pl->parallel_id >= 0 &&
                  pl->parallel_id < pl->parallel_num)
      << Error::RuntimeError() << "placement: parallel_id " << pl->parallel_id << " of "
      << pl->parallel_num;
  const DeviceType dt = DeviceOf(pl->device_type);
  CHECK_OR_RETURN(dt != DeviceType::kInvalidDevice)
      << Error::RuntimeError() << "placement: unknown device type " << pl->device_type;
  std::vector<std::pair<int64_t, int64_t>> md;
  for (int64_t p = 0; p < pl->parallel_num; ++p)
    md.emplace_back(pl->machine_ids ? pl->machine_ids[p] : p, pl->device_ids ? pl->device_ids[p] : p);
  *pd = ParallelDesc(dt, md);
  return Maybe<void>::Ok();
}

Shape ShapeOf(const ofx_tensor_desc* d) {
  std::vector<int64_t> dims;
  for (int i = 0; i < d->ndim; ++i) dims.push_back(d->shape[i]);
  return Shape(dims);
}

Maybe<void> CheckContiguous(const ofx_tensor_desc* t, const char* name) {
  CHECK_OR_RETURN(t != nullptr) << Error::RuntimeError() << "NULL " << name;
  const char* why = ofx::versioned_struct_problem(t, OFX_TENSOR_DESC_MIN_SIZE);
  CHECK_OR_RETURN(why == nullptr)
      << Error::RuntimeError() << name << ": ofx_tensor_desc " << why << " ("
      << OFX_TENSOR_DESC_MIN_SIZE << " bytes): initialise it with OFX_TENSOR_DESC_INIT";
  CHECK_OR_RETURN(t->ndim >= 1 && t->ndim <= 2) << Error::RuntimeError() << name << " must be 1-D or 2-D";
  if (t->ndim == 2 && t->shape[0] > 1)
    CHECK_OR_RETURN(t->stride[0] == t->shape[1] && (t->shape[1] <= 1 || t->stride[1] == 1))
        << Error::RuntimeError() << name << " must be contiguous";
  return Maybe<void>::Ok();
}

// Streams of the kernels: a HIP stream handle for kHIP, the host for kCPU.
// Makes `device` current for its scope and restores the caller's device (a negative device, a
// host placement, changes nothing).
struct DeviceGuard {
  int prev = -1, rc = OFX_OK;
  explicit DeviceGuard(int device) {
    if (device < 0) return;
    if (hipGetDevice(&prev) != hipSuccess) {
      rc = ofx::fail(OFX_EDEVICE, "spmm job: hipGetDevice failed");
      prev = -1;
      return;
    }
    if (prev == device) {
      prev = -1;
      return;
    }
    if (hipSetDevice(device) != hipSuccess) {
      rc = ofx::fail(OFX_EDEVICE, "spmm job: hipSetDevice(%d) failed", device);
      prev = -1;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct StreamPair {
  ep::CpuStream cpu{0};
  ep::HipStream hip;
  StreamPair(void* s, int dev) : hip(s, dev) {}
  ep::Stream* of(DeviceType dt) { return dt == DeviceType::kCPU ? static_cast<ep::Stream*>(&cpu) : &hip; }
};

// ---- SpmmJob -----------------------------------------------------------------------------
class SpmmJob {
 public:
  Maybe<void> Compile(const ParallelDesc& pd, int64_t parallel_id, int idx_dtype, int val_dtype,
                      int64_t m, int64_t k, int64_t n, int64_t nnz, const std::string& stream_name) {
    pd_ = pd;
    pc_ = ParallelContext(parallel_id, pd.parallel_num());
    idx_dtype_ = idx_dtype;
    val_dtype_ = val_dtype;
    m_ = m;
    k_ = k;
    n_ = n;
    nnz_ = nnz;
    // the functional layer's device code: -1 = host, else the HIP ordinal
    device_ = pd.device_type() == DeviceType::kCPU ? -1 : (int)pd.DeviceId4ParallelId(parallel_id);
    const int64_t P = pd.parallel_num();
    const Shape b_logical({k, n});
    std::ostringstream plan;
    // 1. the pass on b's edge: S(0) (producer) -> B (spmm_csr's row-split signature)
    if (P > 1) {
      CHECK_OR_RETURN(pd.device_type() == DeviceType::kHIP)
          << Error::RuntimeError() << "lazy spmm job: InsertNcclLogicalOpPass rewrites edges of "
          << "device placements only; a " << DeviceTypeName(pd.device_type())
          << " placement keeps ordinary boxing";
      gather_op_ = NcclLogicalOpType1D("S(0)", "B", b_logical, P);
      CHECK_OR_RETURN(gather_op_ == "_nccl_logical_all_gather")
          << Error::RuntimeError() << "lazy spmm job: b's S(0) -> B edge with K = " << k << " on "
          << P << " ranks is not a logical collective (K % P != 0); the row-split wrapper "
          << "pads the shards (RowSplitSpmm)";
      JUST(CompileGather(b_logical, stream_name));
      plan << "b[" << k << "," << n << "] S(0) (" << b_shard_.ToString() << " on this rank) -> "
           << gather_op_ << "(src S(0), dst B, stream " << stream_name << ") -> b B "
           << b_full_.ToString() << "; ";
    } else {
      b_full_ = b_logical;
      b_shard_ = b_logical;
      plan << "b[" << k << "," << n << "]: one device, S(0) == B, no boxing; ";
    }
    // 2. spmm_csr(a_csr_*: B, b: B) -> out S(0): physical out rows of this rank and its tmp
    const auto rows = BalancedSplitter(m, P).At(parallel_id);
    out_rows_ = rows.second - rows.first;
    esz_ = GetSizeOfDataType((DataType)val_dtype);
    gathered_bytes_ = P > 1 ? (size_t)(k * n) * esz_ : 0;
    gathered_bytes_ = (gathered_bytes_ + 511) / 512 * 512;
    ofx_tensor_desc rp, ci, v, b, out;
    Descs(nullptr, nullptr, nullptr, nullptr, nullptr, &rp, &ci, &v, &b, &out);
    const int64_t h = P;
    const int32_t ax = 0;
    const int rc = ofx_functional_spmm_csr_global(nullptr, &rp, &ci, &v, m, k, &b, -1, &out, nullptr,
                                                  0, 1, &h, &ax, parallel_id, 0, &spmm_tmp_bytes_);
    CHECK_EQ_OR_RETURN(rc, OFX_OK) << Error::RuntimeError() << ofx_last_error();
    plan << "spmm_csr(a_csr_row_ptr/col_idx/values B, b B) -> out S(0) rows [" << rows.first << ","
         << rows.second << ") of " << m << "; tmp " << gathered_bytes_ << " + " << spmm_tmp_bytes_
         << " bytes";
    plan_ = plan.str();
    return Maybe<void>::Ok();
  }

  const std::string& plan() const { return plan_; }
  size_t tmp_bytes() const { return gathered_bytes_ + spmm_tmp_bytes_; }

  // Graph mode is validated at one rank only (tests/test_ccl_gpu.py): a multi-rank capture
  // records ncclAllGather into the graph, and that capture/replay has not run on hardware yet
  // (the driver's 8-GPU node is the first place it could), so P > 1 is refused until it has.
  int set_graph(bool enable) {
    OFX_REQUIRE(!enable || pd_.parallel_num() == 1, OFX_EUNSUPPORTED,
                "spmm job: graph mode with %lld ranks (a captured RCCL all-gather) is not "
                "validated on hardware; run the %lld-rank job eagerly",
                (long long)pd_.parallel_num(), (long long)pd_.parallel_num());
    graph_enabled_ = enable && pd_.device_type() == DeviceType::kHIP;
    if (!graph_enabled_) graph_.reset();
    return OFX_OK;
  }
  // attr static_csr of the job's spmm_csr (include/ofx_spmm.h ofx_spmm_attrs): the job's own
  // kernel state keeps the plan of the row_ptr it runs on, so the eager first run plans and
  // every later run (or graph replay) launches planned.
  void set_static(int64_t static_csr) { static_csr_ = static_csr; }
  void static_stats(int64_t* plans, int64_t* hits) const {
    int64_t e = 0, p = 0, h = 0;
    if (spmm_state_) SpmmCsrPlanStateStats(spmm_state_.get(), &e, &p, &h, false);
    if (plans) *plans = p;
    if (hits) *hits = h;
  }
  void graph_stats(int64_t* captures, int64_t* replays, int64_t* updates) const {
    if (captures) *captures = captures_;
    if (replays) *replays = replays_;
    if (updates) *updates = graph_ ? graph_->updates() : 0;
  }

  // UserKernel::ForwardUserKernel's graph branch (core/kernel/user_kernel.cpp:676-707): launch
  // the captured graph while the tensors are unchanged; otherwise capture this run's launches
  // on the stream (updating the executable in place), then launch it.
  int Run(void* stream, const void* row_ptr, const void* col_idx, const void* values,
          const void* b_shard, void* out, void* tmp, size_t tmp_bytes) {
    OFX_REQUIRE(tmp_bytes >= this->tmp_bytes() && (tmp || this->tmp_bytes() == 0), OFX_EWORKSPACE,
                "spmm job: tmp of %zu bytes < %zu", tmp_bytes, this->tmp_bytes());
    // CudaGraphSupport::IsReadyForCapture: the logical all-gather creates its RCCL communicator
    // on its first run (not capturable), so the first run of a job is always eager.
    if (!graph_enabled_ || !ready_) {
      const int rc = Launches(stream, row_ptr, col_idx, values, b_shard, out, tmp);
      if (rc == OFX_OK) ready_ = true;
      return rc;
    }
    ep::HipStream caller(stream, device_);
    OFX_REQUIRE(stream == nullptr || !caller.IsGraphCapturing(), OFX_EINVAL,
                "spmm job: graph mode inside an outer capture; disable one of them");
    const std::vector<const void*> key = {row_ptr, col_idx, values, b_shard, out, tmp};
    if (graph_ && graph_->IsInstantiated() && key == graph_key_) {
      ++replays_;
      return caller.LaunchGraph(graph_.get());
    }
    // The launches are recorded on the job's own capture stream (a graph does not remember the
    // stream it was captured on, and the caller's may be the null stream, which cannot be
    // captured); the graph is then launched on the caller's stream, in its order.  The capture
    // stream, the capture and the instantiation belong to the job's device, whatever device
    // the caller has current (restored on return).
    DeviceGuard guard(device_);
    if (guard.rc) return guard.rc;
    if (!capture_stream_) {
      const int rc = ofx_stream_create(&capture_stream_);
      if (rc) return rc;
    }
    if (!graph_) graph_.reset(new ep::HipGraphExecutable());
    ep::HipStream cap(capture_stream_, device_);
    int rc = cap.BeginGraphCapture();
    if (rc) return rc;
    rc = Launches(capture_stream_, row_ptr, col_idx, values, b_shard, out, tmp);
    if (rc) {
      const std::string why = ofx_last_error();
      cap.EndGraphCapture(nullptr);  // discard the partial capture
      graph_key_.clear();
      return ofx::fail(rc, "%s", why.c_str());
    }
    rc = cap.EndGraphCapture(graph_.get());
    if (rc) {
      graph_key_.clear();
      return rc;
    }
    graph_key_ = key;
    ++captures_;
    return caller.LaunchGraph(graph_.get());
  }

  ~SpmmJob() {
    graph_.reset();
    if (capture_stream_) ofx_stream_destroy(capture_stream_);
  }

 private:
  int Launches(void* stream, const void* row_ptr, const void* col_idx, const void* values,
               const void* b_shard, void* out, void* tmp) {
    const void* b_full = b_shard;
    if (gather_kernel_) {
      user_op::Tensor t_in(b_shard_, (DataType)val_dtype_, const_cast<void*>(b_shard));
      user_op::Tensor t_out(b_full_, (DataType)val_dtype_, tmp);
      std::map<std::pair<std::string, int32_t>, user_op::Tensor*> tensors = {{{"in", 0}, &t_in},
                                                                             {{"out", 0}, &t_out}};
      StreamPair sp(stream, device_);
      user_op::KernelComputeContext ctx(sp.of(pd_.device_type()), tensors, {}, pd_.device_type());
      ctx.set_parallel_ctx(pc_);
      try {
        gather_kernel_->Compute(&ctx, gather_state_.get(), nullptr);
      } catch (const KernelCheckError& e) {
        return ofx::fail(OFX_ECOMM, "%s", e.msg.c_str());
      }
      b_full = tmp;
    }
    ofx_tensor_desc rp, ci, v, b, o;
    Descs(row_ptr, col_idx, values, b_full, out, &rp, &ci, &v, &b, &o);
    const int64_t h = pd_.parallel_num();
    const int32_t ax = 0;
    char* spmm_tmp = spmm_tmp_bytes_ ? static_cast<char*>(tmp) + gathered_bytes_ : nullptr;
    return SpmmCsrGlobalWithState(stream, &rp, &ci, &v, m_, k_, &b, -1, &o, spmm_tmp,
                                  spmm_tmp_bytes_, 1, &h, &ax, pc_.parallel_id(), static_csr_,
                                  &spmm_state_);
  }

  Maybe<void> CompileGather(const Shape& b_logical, const std::string& stream_name) {
    const user_op::OpRegistryResult* op =
        user_op::UserOpRegistryMgr::Get().GetOpRegistryResult(gather_op_);
    CHECK_OR_RETURN(op != nullptr) << Error::RuntimeError() << gather_op_ << " is not registered";
    const DataType dt = (DataType)val_dtype_;
    user_op::InferContext lctx({{{"in", 0}, user_op::TensorDesc(b_logical, dt)}}, {});
    JUST(op->logical_infer(&lctx));
    JUST(op->dtype_infer(&lctx));
    user_op::InferNdSbpFnContext sctx(*pd_.hierarchy(), {},
                                      {{"src_reduced_nd_sbp", {"S(0)"}}, {"dst_reduced_nd_sbp", {"B"}}});
    JUST(op->nd_sbp_infer(&sctx));
    JUST(GetPhysicalShape(b_logical, sctx.NdSbp4ArgName("in"), pd_, pc_, &b_shard_));
    JUST(GetPhysicalShape(lctx.OutputTensorDesc("out", 0).shape(), sctx.NdSbp4ArgName("out"), pd_,
                          pc_, &b_full_));
    user_op::KernelRegContext rc;
    rc.device_type_ = pd_.device_type();
    rc.dtypes[{"in", 0}] = rc.dtypes[{"out", 0}] = dt;
    const user_op::OpKernelRegistryResult* reg = nullptr;
    JUST(user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult(gather_op_, rc, &reg));
    gather_kernel_.reset(reg->create_fn());
    user_op::KernelInitContext ictx(pc_, pd_, pd_.device_type(), stream_name);
    try {
      gather_state_ = gather_kernel_->CreateOpKernelState(&ictx);
    } catch (const KernelCheckError& e) {
      return Maybe<void>("KernelCheckError", e.msg);
    }
    return Maybe<void>::Ok();
  }

  void Descs(const void* rp, const void* ci, const void* v, const void* b, void* out,
             ofx_tensor_desc* d_rp, ofx_tensor_desc* d_ci, ofx_tensor_desc* d_v,
             ofx_tensor_desc* d_b, ofx_tensor_desc* d_o) const {
    auto vec = [&](ofx_tensor_desc* d, int dt, int64_t len, const void* p) {
      *d = ofx_tensor_desc OFX_TENSOR_DESC_INIT;
      d->dtype = dt;
      d->device = device_;
      d->ndim = 1;
      d->shape[0] = len;
      d->stride[0] = 1;
      d->data = const_cast<void*>(p);
    };
    auto mat = [&](ofx_tensor_desc* d, int64_t r, const void* p) {
      *d = ofx_tensor_desc OFX_TENSOR_DESC_INIT;
      d->dtype = val_dtype_;
      d->device = device_;
      d->ndim = 2;
      d->shape[0] = r;
      d->shape[1] = n_;
      d->stride[0] = n_;
      d->stride[1] = 1;
      d->data = const_cast<void*>(p);
    };
    vec(d_rp, idx_dtype_, m_ + 1, rp);
    vec(d_ci, idx_dtype_, nnz_, ci);
    vec(d_v, val_dtype_, nnz_, v);
    mat(d_b, k_, b);
    mat(d_o, out_rows_, out);
  }

  ParallelDesc pd_;
  ParallelContext pc_;
  int idx_dtype_ = 0, val_dtype_ = 0, device_ = 0;
  int64_t m_ = 0, k_ = 0, n_ = 0, nnz_ = 0, out_rows_ = 0;
  size_t esz_ = 0, gathered_bytes_ = 0, spmm_tmp_bytes_ = 0;
  std::string gather_op_, plan_;
  Shape b_shard_, b_full_;
  std::unique_ptr<user_op::OpKernel> gather_kernel_;
  std::shared_ptr<user_op::OpKernelState> gather_state_;
  std::shared_ptr<user_op::OpKernelState> spmm_state_;  // spmm_csr's state (static_csr plans)
  int64_t static_csr_ = 0;
  bool graph_enabled_ = false, ready_ = false;
  void* capture_stream_ = nullptr;
  std::unique_ptr<ep::HipGraphExecutable> graph_;
  std::vector<const void*> graph_key_;
  int64_t captures_ = 0, replays_ = 0;
};

}  // namespace
}  // namespace oneflow

using namespace oneflow;

extern "C" int ofx_process_ctx_init(int64_t rank, int64_t world, ofx_kv_push_fn push,
                                    ofx_kv_pull_fn pull, ofx_sendrecv_fn sendrecv, void* user) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(world >= 1 && rank >= 0 && rank < world, OFX_EINVAL,
                "process_ctx_init: rank %lld of %lld", (long long)rank, (long long)world);
    ctrl::Install(rank, world, push, pull, sendrecv, user);
    return OFX_OK;
  });
}

extern "C" int ofx_ccl_registered(int device_type, int* all_gather, int* communication_context) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(all_gather && communication_context, OFX_EINVAL, "ccl_registered: NULL argument");
    *all_gather = ccl::IsAllGatherRegistered(DeviceOf(device_type)) ? 1 : 0;
    *communication_context = ccl::IsCommunicationContextRegistered(DeviceOf(device_type)) ? 1 : 0;
    return OFX_OK;
  });
}

extern "C" int ofx_boxing_check_ccl_s2b(const ofx_placement* pl, int ndim,
                                        const int64_t* logical_shape, const char* in_sbp,
                                        const char* out_sbp) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(ndim >= 0 && ndim <= 8 && (ndim == 0 || logical_shape) && in_sbp && out_sbp,
                OFX_EINVAL, "boxing_check_ccl_s2b: bad arguments");
    ParallelDesc pd;
    int rc = ToStatus(MakeParallelDesc(pl, &pd));
    if (rc) return rc;
    const Shape logical(std::vector<int64_t>(logical_shape, logical_shape + ndim));
    return ToStatus(CheckCclS2B({{in_sbp}, pd}, {{out_sbp}, pd}, logical));
  });
}

extern "C" int ofx_boxing_ccl_s2b(void* stream, const ofx_placement* pl, const ofx_tensor_desc* in,
                                  ofx_tensor_desc* out, int64_t logical_dim0) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ParallelDesc pd;
    int rc = ToStatus(MakeParallelDesc(pl, &pd));
    if (rc) return rc;
    rc = ToStatus(CheckContiguous(in, "in"));
    if (rc) return rc;
    rc = ToStatus(CheckContiguous(out, "out"));
    if (rc) return rc;
    Shape logical = ShapeOf(in);
    logical.Set(0, logical_dim0);
    user_op::Tensor t_in(ShapeOf(in), (DataType)in->dtype, in->data);
    user_op::Tensor t_out(ShapeOf(out), (DataType)out->dtype, out->data);
    StreamPair sp(stream, in->device);
    return ToStatus(CclS2B(sp.of(pd.device_type()), t_in, &t_out, {{"S(0)"}, pd}, {{"B"}, pd}, logical,
                           pl->parallel_id),
                    OFX_ECOMM);
  });
}

extern "C" int ofx_nccl_logical_all_gather(void* stream, const ofx_placement* pl,
                                           const ofx_tensor_desc* in, ofx_tensor_desc* out,
                                           const char* stream_name) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ParallelDesc pd;
    int rc = ToStatus(MakeParallelDesc(pl, &pd));
    if (rc) return rc;
    rc = ToStatus(CheckContiguous(in, "in"));
    if (rc) return rc;
    rc = ToStatus(CheckContiguous(out, "out"));
    if (rc) return rc;
    const std::string op_name = "_nccl_logical_all_gather";
    const user_op::OpRegistryResult* op = user_op::UserOpRegistryMgr::Get().GetOpRegistryResult(op_name);
    OFX_REQUIRE(op, OFX_EINVAL, "%s is not registered", op_name.c_str());
    Shape logical = ShapeOf(in);
    logical.Set(0, ShapeOf(out).At(0));
    user_op::InferNdSbpFnContext sctx(*pd.hierarchy(), {},
                                      {{"src_reduced_nd_sbp", {"S(0)"}}, {"dst_reduced_nd_sbp", {"B"}}});
    rc = ToStatus(op->nd_sbp_infer(&sctx));
    if (rc) return rc;
    user_op::KernelRegContext reg_ctx;
    reg_ctx.device_type_ = pd.device_type();
    reg_ctx.dtypes[{"in", 0}] = reg_ctx.dtypes[{"out", 0}] = (DataType)in->dtype;
    const user_op::OpKernelRegistryResult* reg = nullptr;
    rc = ToStatus(user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult(op_name, reg_ctx, &reg));
    if (rc) return rc;
    std::unique_ptr<user_op::OpKernel> kernel(reg->create_fn());
    const ParallelContext pc(pl->parallel_id, pd.parallel_num());
    user_op::KernelInitContext ictx(pc, pd, pd.device_type(), stream_name ? stream_name : "");
    user_op::Tensor t_in(ShapeOf(in), (DataType)in->dtype, in->data);
    user_op::Tensor t_out(ShapeOf(out), (DataType)out->dtype, out->data);
    std::map<std::pair<std::string, int32_t>, user_op::Tensor*> tensors = {{{"in", 0}, &t_in},
                                                                           {{"out", 0}, &t_out}};
    StreamPair sp(stream, in->device);
    user_op::KernelComputeContext ctx(sp.of(pd.device_type()), tensors, {}, pd.device_type());
    ctx.set_parallel_ctx(pc);
    try {
      std::shared_ptr<user_op::OpKernelState> state = kernel->CreateOpKernelState(&ictx);
      kernel->Compute(&ctx, state.get(), nullptr);
    } catch (const KernelCheckError& e) {
      return ofx::fail(OFX_ECOMM, "%s", e.msg.c_str());
    }
    return OFX_OK;
  });
}

extern "C" int ofx_insert_nccl_logical_op(const char* src_sbp, const char* dst_sbp, int ndim,
                                          const int64_t* logical_shape, int64_t parallel_num,
                                          char* op_type, size_t len) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(src_sbp && dst_sbp && op_type && len > 0 && ndim >= 0 && ndim <= 8 &&
                    (ndim == 0 || logical_shape) && parallel_num >= 1,
                OFX_EINVAL, "insert_nccl_logical_op: bad arguments");
    const Shape logical(std::vector<int64_t>(logical_shape, logical_shape + ndim));
    snprintf(op_type, len, "%s", NcclLogicalOpType1D(src_sbp, dst_sbp, logical, parallel_num).c_str());
    return OFX_OK;
  });
}

extern "C" int ofx_rccl_comm_key(const ofx_placement* pl, const char* stream_name, int64_t machine,
                                 int64_t device, char* key, size_t len, int* rank) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ParallelDesc pd;
    int rc = ToStatus(MakeParallelDesc(pl, &pd));
    if (rc) return rc;
    OFX_REQUIRE(key && len > 0 && rank, OFX_EINVAL, "rccl_comm_key: NULL argument");
    DeviceSet set;
    for (int64_t p = 0; p < pd.parallel_num(); ++p)
      set.emplace(pd.MachineId4ParallelId(p), pd.DeviceId4ParallelId(p));
    const std::vector<std::pair<int64_t, int64_t>> vec(set.begin(), set.end());
    snprintf(key, len, "%s",
             EagerRcclCommMgr::UniqueIdKey(vec, stream_name ? stream_name
                                                            : EagerRcclCommMgr::kDefaultStreamName)
                 .c_str());
    *rank = EagerRcclCommMgr::RankInSet(vec, machine, device);
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_create(const ofx_placement* pl, int idx_dtype, int val_dtype, int64_t m,
                                   int64_t k, int64_t n, int64_t nnz, const char* stream_name,
                                   void** job) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_create: NULL job");
    OFX_REQUIRE(ofx::is_index_dtype(idx_dtype) && ofx::is_value_dtype(val_dtype), OFX_EUNSUPPORTED,
                "spmm_job_create: dtypes %d / %d", idx_dtype, val_dtype);
    OFX_REQUIRE(m >= 0 && k >= 0 && n >= 0 && nnz >= 0, OFX_EINVAL, "spmm_job_create: bad shape");
    ParallelDesc pd;
    int rc = ToStatus(MakeParallelDesc(pl, &pd));
    if (rc) return rc;
    std::unique_ptr<SpmmJob> j(new SpmmJob());
    rc = ToStatus(j->Compile(pd, pl->parallel_id, idx_dtype, val_dtype, m, k, n, nnz,
                             stream_name && *stream_name ? stream_name
                                                         : EagerRcclCommMgr::kDefaultStreamName));
    if (rc) return rc;
    *job = j.release();
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_describe(void* job, char* buf, size_t len, size_t* tmp_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job && buf && len > 0, OFX_EINVAL, "spmm_job_describe: NULL argument");
    const SpmmJob* j = static_cast<SpmmJob*>(job);
    snprintf(buf, len, "%s", j->plan().c_str());
    if (tmp_bytes) *tmp_bytes = j->tmp_bytes();
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_run(void* job, void* stream, const void* row_ptr, const void* col_idx,
                                const void* values, const void* b_shard, void* out, void* tmp,
                                size_t tmp_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_run: NULL job");
    return static_cast<SpmmJob*>(job)->Run(stream, row_ptr, col_idx, values, b_shard, out, tmp,
                                           tmp_bytes);
  });
}

extern "C" int ofx_spmm_job_destroy(void* job) {
  return ::ofx::guarded(__func__, [&]() -> int {
    delete static_cast<SpmmJob*>(job);
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_set_graph(void* job, int enable) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_set_graph: NULL job");
    return static_cast<SpmmJob*>(job)->set_graph(enable != 0);
  });
}

extern "C" int ofx_spmm_job_set_static(void* job, int64_t static_csr) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_set_static: NULL job");
    static_cast<SpmmJob*>(job)->set_static(static_csr);
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_static_stats(void* job, int64_t* plans, int64_t* hits) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_static_stats: NULL job");
    static_cast<const SpmmJob*>(job)->static_stats(plans, hits);
    return OFX_OK;
  });
}

extern "C" int ofx_spmm_job_graph_stats(void* job, int64_t* captures, int64_t* replays,
                                        int64_t* updates) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(job, OFX_EINVAL, "spmm_job_graph_stats: NULL job");
    static_cast<const SpmmJob*>(job)->graph_stats(captures, replays, updates);
    return OFX_OK;
  });
}
