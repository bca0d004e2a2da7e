/*
 * spmm_functor.cpp — functional::SpmmCsr and its C-ABI entry (the Python binding calls this).
 *
 * Mirrors the functional layer of the reference: YAML signature
 *   "Tensor (Tensor a_csr_row_ptr, Tensor a_csr_col_idx, Tensor a_csr_values, Int64 a_num_rows,
 *            Int64 a_num_cols, Tensor b) => SpmmCsr"      (template functional_api.yaml:1062-1065)
 * and the functor pattern of oneflow/core/functional/impl/nn_functor.cpp:3861-3884 (argument
 * checks as RuntimeError, then OpInterpUtil::Dispatch).  "Dispatch" here is the eager-local
 * interpreter reduced to what one op needs (oneflow/core/framework/op_interpreter/
 * eager_local_op_interpreter.cpp:74-160): run the op's logical/dtype inference, choose the one
 * matching kernel (StatefulOpKernel::ChooseOpKernel, oneflow/user/kernels/stateful_opkernel.cpp:873-910),
 * init its cache (:912-935) and Compute on the device stream.  Output/tmp memory is owned by the
 * caller, as the VM owns it in the reference (oneflow/core/vm/op_call_instruction_policy.cpp:28-36).
 */
#include <mutex>

#include "oneflow/core/framework/framework.h"
#include "oneflow/core/functional/spmm_functor.h"
#include "ofx_internal.h"
#include "ofx_spmm.h"

namespace oneflow {
namespace {

using DescMap = std::map<std::pair<std::string, int32_t>, user_op::TensorDesc>;

Shape ShapeOf(const ofx_tensor_desc* d) {
  std::vector<int64_t> dims;
  for (int i = 0; i < d->ndim; ++i) dims.push_back(d->shape[i]);
  return Shape(dims);
}

int ToStatus(const Maybe<void>& m) {
  if (m.IsOk()) return OFX_OK;
  return ofx::fail(OFX_EINVAL, "%s: %s", m.kind().c_str(), m.message().c_str());
}

// A versioned descriptor (include/ofx_spmm.h): the tag, then struct_size at least the first
// tagged layout's.
Maybe<void> CheckDesc(const ofx_tensor_desc* d, const char* name) {
  const char* why = ofx::versioned_struct_problem(d, OFX_TENSOR_DESC_MIN_SIZE);
  CHECK_OR_RETURN(why == nullptr)
      << Error::RuntimeError() << name << ": ofx_tensor_desc " << why << " ("
      << OFX_TENSOR_DESC_MIN_SIZE << " bytes): initialise it with OFX_TENSOR_DESC_INIT";
  return Maybe<void>::Ok();
}

Maybe<void> CheckArgs(const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
                      const ofx_tensor_desc* values, const ofx_tensor_desc* b) {
  CHECK_OR_RETURN(row_ptr && col_idx && values && b)
      << Error::RuntimeError() << "spmm_csr: NULL tensor argument";
  JUST(CheckDesc(row_ptr, "a_csr_row_ptr"));
  JUST(CheckDesc(col_idx, "a_csr_col_idx"));
  JUST(CheckDesc(values, "a_csr_values"));
  JUST(CheckDesc(b, "b"));
  CHECK_OR_RETURN(row_ptr->ndim >= 1 && row_ptr->ndim <= 2 && col_idx->ndim >= 1 &&
                  col_idx->ndim <= 2 && values->ndim >= 1 && values->ndim <= 2 && b->ndim >= 1 &&
                  b->ndim <= 2)
      << Error::RuntimeError() << "spmm_csr: tensors must be 1-D or 2-D";
  CHECK_OR_RETURN(row_ptr->device == col_idx->device && row_ptr->device == values->device &&
                  row_ptr->device == b->device)
      << Error::RuntimeError() << "spmm_csr: expected all tensors on the same device, got "
      << row_ptr->device << ", " << col_idx->device << ", " << values->device << ", "
      << b->device;
  return Maybe<void>::Ok();
}

// Stride contract of the kernels: a 2-D tensor is rows of unit-stride elements at row_stride
// >= shape[1] (b may be a row-strided view; out too).  A column stride != 1 (e.g. out[:, ::2])
// cannot be expressed to the kernel, which takes only the row stride, and is refused.
Maybe<void> CheckUnitColumnStride(const ofx_tensor_desc* t, const char* name) {
  if (t->ndim == 2 && t->shape[0] > 0 && t->shape[1] > 1) {
    CHECK_OR_RETURN(t->stride[1] == 1 && t->stride[0] >= t->shape[1])
        << Error::RuntimeError() << "spmm_csr: " << name << " must have unit column stride and "
        << "row stride >= its columns, got strides (" << t->stride[0] << ", " << t->stride[1]
        << ")";
  }
  return Maybe<void>::Ok();
}

// Placement of a (possibly global) call: the hierarchy, out's NdSbp and b's NdSbp (out S(0) ->
// b B, out S(1) -> b S(1), out B -> b B), and this rank.  A local call is the 1-device placement.
struct Placement {
  Shape hierarchy{1};
  NdSbp out_sbp{"B"}, b_sbp{"B"};
  int64_t parallel_id = 0;
  int64_t parallel_num() const { return hierarchy.elem_cnt(); }
};

Maybe<void> MakePlacement(int hierarchy_ndim, const int64_t* hierarchy, const int32_t* out_split,
                          int64_t parallel_id, Placement* p) {
  CHECK_OR_RETURN(hierarchy_ndim >= 1 && hierarchy_ndim <= 4 && hierarchy && out_split)
      << Error::RuntimeError() << "spmm_csr: placement needs a 1-D..4-D hierarchy";
  std::vector<int64_t> dims;
  p->out_sbp.clear();
  p->b_sbp.clear();
  for (int i = 0; i < hierarchy_ndim; ++i) {
    CHECK_GE_OR_RETURN(hierarchy[i], 1) << Error::RuntimeError() << "bad hierarchy dim";
    CHECK_OR_RETURN(out_split[i] >= -1 && out_split[i] <= 1)
        << Error::RuntimeError() << "out can be split on axis 0 or 1 only";
    dims.push_back(hierarchy[i]);
    p->out_sbp.push_back(out_split[i] < 0 ? "B" : "S(" + std::to_string(out_split[i]) + ")");
    p->b_sbp.push_back(out_split[i] == 1 ? "S(1)" : "B");
  }
  p->hierarchy = Shape(dims);
  CHECK_OR_RETURN(parallel_id >= 0 && parallel_id < p->parallel_num())
      << Error::RuntimeError() << "spmm_csr: parallel_id " << parallel_id << " outside "
      << p->hierarchy.ToString();
  p->parallel_id = parallel_id;
  return Maybe<void>::Ok();
}

// Logical inference (the op's logical rule on the logical b: K x b_logical_cols), then the
// physical out of this rank (the op's physical rule on the physical inputs + placement).
Maybe<void> Infer(const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
                  const ofx_tensor_desc* values, int64_t m, int64_t k, const ofx_tensor_desc* b,
                  int64_t b_logical_cols, const Placement& pl, user_op::TensorDesc* logical_out,
                  user_op::TensorDesc* physical_out) {
  JUST(CheckArgs(row_ptr, col_idx, values, b));
  JUST(CheckUnitColumnStride(b, "b"));
  const user_op::OpRegistryResult* op = user_op::UserOpRegistryMgr::Get().GetOpRegistryResult("spmm_csr");
  CHECK_OR_RETURN(op != nullptr) << Error::RuntimeError() << "op spmm_csr is not registered";
  DescMap in;
  in[{"a_csr_row_ptr", 0}] = user_op::TensorDesc(ShapeOf(row_ptr), (DataType)row_ptr->dtype);
  in[{"a_csr_col_idx", 0}] = user_op::TensorDesc(ShapeOf(col_idx), (DataType)col_idx->dtype);
  in[{"a_csr_values", 0}] = user_op::TensorDesc(ShapeOf(values), (DataType)values->dtype);
  DescMap logical_in = in;
  Shape b_logical = ShapeOf(b);
  if (b_logical.NumAxes() == 2 && b_logical_cols >= 0) b_logical.Set(1, b_logical_cols);
  logical_in[{"b", 0}] = user_op::TensorDesc(b_logical, (DataType)b->dtype);
  const user_op::AttrMap attrs = {{"a_num_rows", m}, {"a_num_cols", k}};
  user_op::InferContext lctx(logical_in, attrs);
  JUST(op->logical_infer(&lctx));
  JUST(op->dtype_infer(&lctx));
  *logical_out = lctx.OutputTensorDesc("out", 0);
  in[{"b", 0}] = user_op::TensorDesc(ShapeOf(b), (DataType)b->dtype);
  user_op::InferContext pctx(in, attrs);
  pctx.SetParallel(ParallelContext(pl.parallel_id, pl.parallel_num()), ParallelDesc(pl.hierarchy),
                   {{"out", pl.out_sbp}, {"b", pl.b_sbp}}, {{"out", *logical_out}});
  JUST(op->physical_infer(&pctx));
  JUST(op->dtype_infer(&pctx));
  *physical_out = pctx.OutputTensorDesc("out", 0);
  return Maybe<void>::Ok();
}

struct KernelEntry {
  const user_op::OpKernelRegistryResult* reg;
  std::unique_ptr<user_op::OpKernel> kernel;
};

// Kernel objects are shared and const, cached per registration (stateful_opkernel.cpp:887-908).
const user_op::OpKernel* GetKernel(const user_op::OpKernelRegistryResult* reg) {
  static std::mutex mu;
  static std::map<const void*, std::unique_ptr<user_op::OpKernel>> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto& slot = cache[reg];
  if (!slot) slot.reset(reg->create_fn());
  return slot.get();
}

Maybe<void> Choose(const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* b, int device,
                   const user_op::OpKernelRegistryResult** reg) {
  user_op::KernelRegContext rc;
  rc.device_type_ = device < 0 ? DeviceType::kCPU : DeviceType::kHIP;
  rc.dtypes[{"out", 0}] = (DataType)b->dtype;
  rc.dtypes[{"a_csr_row_ptr", 0}] = (DataType)row_ptr->dtype;
  return user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult("spmm_csr", rc, reg);
}

// The eager op's kernel states: one per (kernel registration, device), as OneFlow's functor
// holds one op expression whose StatefulOpKernel keeps a state per device
// (stateful_opkernel.cpp:887-908).  Created on first use through CreateOpKernelState.
// Never destroyed: a state frees device memory, which must not happen from a static destructor
// after the HIP runtime has gone at process exit.
std::mutex g_eager_states_mu;
auto& g_eager_states =
    *new std::map<std::pair<const void*, int>, std::shared_ptr<user_op::OpKernelState>>();

user_op::OpKernelState* EagerKernelState(const user_op::OpKernelRegistryResult* reg,
                                         const user_op::OpKernel* kernel, int device,
                                         DeviceType dev) {
  std::lock_guard<std::mutex> lock(g_eager_states_mu);
  auto key = std::make_pair(static_cast<const void*>(reg), device);
  auto it = g_eager_states.find(key);
  if (it != g_eager_states.end()) return it->second.get();
  user_op::KernelInitContext ictx(ParallelContext(0, 1), ParallelDesc(Shape({1})), dev);
  auto st = kernel->CreateOpKernelState(&ictx);
  user_op::OpKernelState* raw = st.get();
  g_eager_states[key] = std::move(st);
  return raw;
}

// functional::SpmmCsr on a local or global tensor set: inference, kernel choice, then either the
// tmp size (tmp_size_out != NULL) or the kernel's cache init + Compute on the stream.  `state`:
// the compiled job's own kernel state (NULL: the eager op's, per registration and device).
int RunSpmmCsr(void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
               const ofx_tensor_desc* values, int64_t m, int64_t k, const ofx_tensor_desc* b,
               int64_t b_logical_cols, ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
               const Placement& pl, int num_threads, size_t* tmp_size_out, int64_t static_csr = 0,
               std::shared_ptr<user_op::OpKernelState>* state = nullptr) {
  user_op::TensorDesc logical_od, od;
  int rc = ToStatus(Infer(row_ptr, col_idx, values, m, k, b, b_logical_cols, pl, &logical_od, &od));
  if (rc) return rc;
  const user_op::OpKernelRegistryResult* reg = nullptr;
  rc = ToStatus(Choose(row_ptr, b, b->device, &reg));
  if (rc) return rc;
  if (tmp_size_out) {
    user_op::InferSizeContext sc;
    sc.descs[{"a_csr_row_ptr", 0}] = user_op::TensorDesc(ShapeOf(row_ptr), (DataType)row_ptr->dtype);
    sc.descs[{"a_csr_col_idx", 0}] = user_op::TensorDesc(ShapeOf(col_idx), (DataType)col_idx->dtype);
    sc.descs[{"b", 0}] = user_op::TensorDesc(ShapeOf(b), (DataType)b->dtype);
    sc.attrs = {{"a_num_rows", m}, {"a_num_cols", k}};
    sc.logical["out"] = logical_od;
    *tmp_size_out = reg->infer_tmp_size ? reg->infer_tmp_size(&sc) : 0;
    return OFX_OK;
  }
  OFX_REQUIRE(out, OFX_EINVAL, "spmm_csr: out is NULL");
  // an earlier launch's loud failure comes back here as OFX_EPLAN, before this call launches
  // (the functional call is a library entry like ofx_spmm_csr)
  OFX_TAKE_DEVICE_ERROR("spmm_csr");
  rc = ToStatus(CheckDesc(out, "out"));
  if (rc) return rc;
  const int64_t phys_rows = od.shape().At(0);
  OFX_REQUIRE(out->ndim == 2 && out->shape[0] == phys_rows && out->shape[1] == od.shape().At(1) &&
                  out->dtype == (int32_t)od.data_type() && out->device == b->device,
              OFX_EINVAL,
              "spmm_csr: out must be a (%lld, %lld) tensor of dtype %d on device %d",
              (long long)phys_rows, (long long)od.shape().At(1), (int)od.data_type(), b->device);
  rc = ToStatus(CheckUnitColumnStride(out, "out"));
  if (rc) return rc;
  const user_op::OpKernel* kernel = GetKernel(reg);

  user_op::Tensor t_rp(ShapeOf(row_ptr), (DataType)row_ptr->dtype, row_ptr->data);
  user_op::Tensor t_ci(ShapeOf(col_idx), (DataType)col_idx->dtype, col_idx->data);
  user_op::Tensor t_v(ShapeOf(values), (DataType)values->dtype, values->data);
  user_op::Tensor t_b(ShapeOf(b), (DataType)b->dtype, b->data, b->ndim == 2 ? b->stride[0] : -1);
  user_op::Tensor t_o(ShapeOf(out), (DataType)out->dtype, out->data, out->stride[0]);
  user_op::Tensor t_tmp(Shape({(int64_t)tmp_bytes}), kChar, tmp);
  std::map<std::pair<std::string, int32_t>, user_op::Tensor*> tensors = {
      {{"a_csr_row_ptr", 0}, &t_rp}, {{"a_csr_col_idx", 0}, &t_ci}, {{"a_csr_values", 0}, &t_v},
      {{"b", 0}, &t_b},              {{"out", 0}, &t_o}};
  if (tmp) tensors[{"tmp_buffer", 0}] = &t_tmp;
  const DeviceType dev = b->device < 0 ? DeviceType::kCPU : DeviceType::kHIP;
  ep::CpuStream cpu_stream(num_threads);
  ep::HipStream hip_stream(stream, b->device);
  ep::Stream* s = dev == DeviceType::kCPU ? static_cast<ep::Stream*>(&cpu_stream)
                                          : static_cast<ep::Stream*>(&hip_stream);
  // the op's attributes: the registered defaults, then this call's values
  user_op::AttrMap attrs;
  if (const user_op::OpRegistryResult* op =
          user_op::UserOpRegistryMgr::Get().GetOpRegistryResult("spmm_csr"))
    for (const auto& a : op->attrs) attrs[a.first] = a.second;
  attrs["a_num_rows"] = m;
  attrs["a_num_cols"] = k;
  attrs["static_csr"] = static_csr;
  user_op::OpKernelState* kstate = nullptr;
  if (state != nullptr) {
    if (!*state) {
      // a compiled op's launches are ordered on its one (named) stream
      user_op::KernelInitContext ictx(ParallelContext(pl.parallel_id, pl.parallel_num()),
                                      ParallelDesc(pl.hierarchy), dev, "compiled_job");
      *state = kernel->CreateOpKernelState(&ictx);
    }
    kstate = state->get();
  } else if (static_csr != 0) {
    kstate = EagerKernelState(reg, kernel, b->device, dev);
  }
  user_op::KernelCacheContext cache_ctx(ParallelContext(pl.parallel_id, pl.parallel_num()),
                                        ParallelDesc(pl.hierarchy),
                                        {{"out", pl.out_sbp}, {"b", pl.b_sbp}},
                                        {{"out", logical_od}}, dev);
  user_op::KernelComputeContext ctx(s, tensors, attrs, dev);
  try {
    std::shared_ptr<user_op::OpKernelCache> cache = kernel->InitOpKernelCache(&cache_ctx);
    if (phys_rows == 0 || od.shape().At(1) == 0) {
      if (!kernel->AlwaysComputeWhenAllOutputsEmpty()) return OFX_OK;
    }
    kernel->Compute(&ctx, kstate, cache.get());
  } catch (const KernelCheckError& e) {
    return ofx::fail(OFX_EINVAL, "%s", e.msg.c_str());
  }
  return OFX_OK;
}

}  // namespace

int SpmmCsrGlobalWithState(void* stream, const ofx_tensor_desc* row_ptr,
                           const ofx_tensor_desc* col_idx, const ofx_tensor_desc* values,
                           int64_t m, int64_t k, const ofx_tensor_desc* b, int64_t b_logical_cols,
                           ofx_tensor_desc* out, void* tmp, size_t tmp_bytes, int hierarchy_ndim,
                           const int64_t* hierarchy, const int32_t* out_split_axes,
                           int64_t parallel_id, int64_t static_csr,
                           std::shared_ptr<user_op::OpKernelState>* state) {
  Placement pl;
  int rc = ToStatus(MakePlacement(hierarchy_ndim, hierarchy, out_split_axes, parallel_id, &pl));
  if (rc) return rc;
  return RunSpmmCsr(stream, row_ptr, col_idx, values, m, k, b, b_logical_cols, out, tmp,
                    tmp_bytes, pl, 0, nullptr, static_csr, state);
}

}  // namespace oneflow

using namespace oneflow;

extern "C" int ofx_functional_spmm_csr_infer(const ofx_tensor_desc* row_ptr,
                                             const ofx_tensor_desc* col_idx,
                                             const ofx_tensor_desc* values, int64_t a_num_rows,
                                             int64_t a_num_cols, const ofx_tensor_desc* b,
                                             ofx_tensor_desc* out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    user_op::TensorDesc lod, od;
    int rc = ToStatus(Infer(row_ptr, col_idx, values, a_num_rows, a_num_cols, b, -1, Placement(),
                            &lod, &od));
    if (rc) return rc;
    rc = ToStatus(CheckDesc(out, "out"));
    if (rc) return rc;
    if (out) {
      out->dtype = od.data_type();
      out->ndim = (int32_t)od.shape().NumAxes();
      for (int i = 0; i < out->ndim; ++i) out->shape[i] = od.shape().At(i);
      out->device = b->device;
    }
    return OFX_OK;
  });
}

extern "C" int ofx_functional_spmm_csr_tmp_size(const ofx_tensor_desc* row_ptr,
                                                const ofx_tensor_desc* col_idx,
                                                const ofx_tensor_desc* values, int64_t a_num_rows,
                                                int64_t a_num_cols, const ofx_tensor_desc* b,
                                                size_t* bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(bytes, OFX_EINVAL, "spmm_csr_tmp_size: bytes is NULL");
    return RunSpmmCsr(nullptr, row_ptr, col_idx, values, a_num_rows, a_num_cols, b, -1, nullptr,
                      nullptr, 0, Placement(), 0, bytes);
  });
}

extern "C" int ofx_functional_spmm_csr_global(
    void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
    const ofx_tensor_desc* values, int64_t a_num_rows, int64_t a_num_cols,
    const ofx_tensor_desc* b, int64_t b_logical_cols, ofx_tensor_desc* out, void* tmp,
    size_t tmp_bytes, int hierarchy_ndim, const int64_t* hierarchy, const int32_t* out_split_axes,
    int64_t parallel_id, int num_threads, size_t* tmp_size_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    Placement pl;
    int rc = ToStatus(MakePlacement(hierarchy_ndim, hierarchy, out_split_axes, parallel_id, &pl));
    if (rc) return rc;
    return RunSpmmCsr(stream, row_ptr, col_idx, values, a_num_rows, a_num_cols, b, b_logical_cols,
                      out, tmp, tmp_bytes, pl, num_threads, tmp_size_out);
  });
}

extern "C" int ofx_functional_spmm_csr_global_attrs(
    void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
    const ofx_tensor_desc* values, int64_t a_num_rows, int64_t a_num_cols,
    const ofx_tensor_desc* b, int64_t b_logical_cols, ofx_tensor_desc* out, void* tmp,
    size_t tmp_bytes, int hierarchy_ndim, const int64_t* hierarchy, const int32_t* out_split_axes,
    int64_t parallel_id, int num_threads, size_t* tmp_size_out, const ofx_spmm_attrs* attrs) {
  return ::ofx::guarded(__func__, [&]() -> int {
    int64_t static_csr = 0;
    if (attrs != nullptr) {
      const char* why = ofx::versioned_struct_problem(attrs, OFX_SPMM_ATTRS_MIN_SIZE);
      OFX_REQUIRE(why == nullptr, OFX_EINVAL,
                  "spmm_csr: ofx_spmm_attrs %s (%u bytes): initialise it with OFX_SPMM_ATTRS_INIT",
                  why ? why : "", OFX_SPMM_ATTRS_MIN_SIZE);
      static_csr = attrs->static_csr;
    }
    Placement pl;
    int rc = ToStatus(MakePlacement(hierarchy_ndim, hierarchy, out_split_axes, parallel_id, &pl));
    if (rc) return rc;
    return RunSpmmCsr(stream, row_ptr, col_idx, values, a_num_rows, a_num_cols, b, b_logical_cols,
                      out, tmp, tmp_bytes, pl, num_threads, tmp_size_out, static_csr);
  });
}

extern "C" int ofx_spmm_static_plans(int64_t* entries, int64_t* plans, int64_t* hits,
                                     int release) {
  return ::ofx::guarded(__func__, [&]() -> int {
    int64_t e = 0, p = 0, h = 0;
    std::lock_guard<std::mutex> lock(g_eager_states_mu);
    for (auto& kv : g_eager_states)
      if (kv.second) SpmmCsrPlanStateStats(kv.second.get(), &e, &p, &h, release != 0);
    if (entries) *entries = e;
    if (plans) *plans = p;
    if (hits) *hits = h;
    return OFX_OK;
  });
}

extern "C" int ofx_functional_spmm_csr_ex(void* stream, const ofx_tensor_desc* row_ptr,
                                          const ofx_tensor_desc* col_idx,
                                          const ofx_tensor_desc* values, int64_t a_num_rows,
                                          int64_t a_num_cols, const ofx_tensor_desc* b,
                                          ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                                          int64_t parallel_id, int64_t parallel_num,
                                          int out_split_axis, int num_threads) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(out_split_axis != 1 || parallel_num == 1, OFX_EINVAL,
                "spmm_csr_ex: a column split needs the logical width: use "
                "ofx_functional_spmm_csr_global");
    const int64_t h = parallel_num;
    const int32_t ax = out_split_axis;
    return ofx_functional_spmm_csr_global(stream, row_ptr, col_idx, values, a_num_rows, a_num_cols,
                                          b, -1, out, tmp, tmp_bytes, 1, &h, &ax, parallel_id,
                                          num_threads, nullptr);
  });
}

extern "C" int ofx_functional_spmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                                       const ofx_tensor_desc* col_idx,
                                       const ofx_tensor_desc* values, int64_t a_num_rows,
                                       int64_t a_num_cols, const ofx_tensor_desc* b,
                                       ofx_tensor_desc* out, void* tmp, size_t tmp_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return RunSpmmCsr(stream, row_ptr, col_idx, values, a_num_rows, a_num_cols, b, -1, out, tmp,
                      tmp_bytes, Placement(), 0, nullptr);
  });
}

// SBP signatures of a registered op, for the tests: "arg:sbp,arg:sbp;...|no_grad:..." into buf.
// `optional_inputs`: comma-separated optional inputs the op instance has (e.g. "bias").
extern "C" int ofx_op_sbp_signatures(const char* op_name, const char* optional_inputs, char* buf,
                                     size_t len) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(op_name && buf && len > 0, OFX_EINVAL, "op_sbp_signatures: NULL argument");
    const user_op::OpRegistryResult* op = user_op::UserOpRegistryMgr::Get().GetOpRegistryResult(op_name);
    OFX_REQUIRE(op, OFX_EINVAL, "op %s is not registered", op_name);
    std::vector<std::string> present;
    if (optional_inputs) {
      std::string all(optional_inputs), cur;
      for (char ch : all + ",") {
        if (ch == ',') {
          if (!cur.empty()) present.push_back(cur);
          cur.clear();
        } else {
          cur += ch;
        }
      }
    }
    user_op::SbpContext ctx{user_op::UserOpConfView(present)};
    int rc = ToStatus(op->get_sbp(&ctx));
    if (rc) return rc;
    std::string s;
    for (const auto& sig : ctx.signatures()) {
      if (!s.empty()) s += ";";
      for (size_t i = 0; i < sig.size(); ++i) s += (i ? "," : "") + sig[i].first + ":" + sig[i].second;
    }
    // input-arg modifiers: which inputs have requires_grad disabled
    std::map<std::string, user_op::InputArgModifier> mods;
    user_op::GetInputArgModifier get = [&](const std::string& n, int32_t) { return &mods[n]; };
    if (op->input_modify) {
      rc = ToStatus(op->input_modify(get, user_op::UserOpConfWrapper()));
      if (rc) return rc;
    }
    s += "|no_grad:";
    bool first = true;
    for (const auto& kv : mods)
      if (!kv.second.requires_grad) {
        s += (first ? "" : ",") + kv.first;
        first = false;
      }
    snprintf(buf, len, "%s", s.c_str());
    return OFX_OK;
  });
}

extern "C" int ofx_op_spmm_csr_sbp_signatures(char* buf, size_t len) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return ofx_op_sbp_signatures("spmm_csr", nullptr, buf, len);
  });
}

// ---- gradient functors: functional::SddmmCsr / functional::CsrTranspose ----------------------
// The grad function of spmm_csr calls these; the Python autograd binding
// (oneflow_spmm/autograd.py) goes through the same entries.  Generic eager-local dispatch of a
// registered user op: inference -> output check -> kernel choice (HOB on every arg's dtype) ->
// tmp size or Compute.
namespace oneflow {
namespace {

struct Arg {
  const char* name;
  const ofx_tensor_desc* d;
};

Maybe<void> RunUserOp(const std::string& op_name, const std::vector<Arg>& ins,
                      const std::vector<Arg>& outs, const user_op::AttrMap& call_attrs, void* stream,
                      void* tmp, size_t tmp_bytes, size_t* tmp_size_out) {
  const user_op::OpRegistryResult* op = user_op::UserOpRegistryMgr::Get().GetOpRegistryResult(op_name);
  CHECK_OR_RETURN(op != nullptr) << Error::RuntimeError() << "op " << op_name << " is not registered";
  // the op's attributes: the registered defaults, then this call's values
  user_op::AttrMap attrs;
  for (const auto& a : op->attrs) attrs[a.first] = a.second;
  for (const auto& a : call_attrs) attrs[a.first] = a.second;
  const int device = ins.front().d->device;
  DescMap in;
  for (const Arg& a : ins) {
    CHECK_OR_RETURN(a.d != nullptr) << Error::RuntimeError() << op_name << ": NULL input " << a.name;
    JUST(CheckDesc(a.d, a.name));
    CHECK_OR_RETURN(a.d->ndim >= 1 && a.d->ndim <= 2)
        << Error::RuntimeError() << op_name << ": " << a.name << " must be 1-D or 2-D";
    CHECK_EQ_OR_RETURN(a.d->device, device)
        << Error::RuntimeError() << op_name << ": expected all tensors on the same device";
    JUST(CheckUnitColumnStride(a.d, a.name));
    in[{a.name, 0}] = user_op::TensorDesc(ShapeOf(a.d), (DataType)a.d->dtype);
  }
  user_op::InferContext ictx(in, attrs);
  JUST(op->logical_infer(&ictx));
  JUST(op->dtype_infer(&ictx));
  user_op::KernelRegContext rc;
  rc.device_type_ = device < 0 ? DeviceType::kCPU : DeviceType::kHIP;
  for (const Arg& a : ins) rc.dtypes[{a.name, 0}] = (DataType)a.d->dtype;
  for (const std::string& o : op->outputs) rc.dtypes[{o, 0}] = ictx.OutputTensorDesc(o, 0).data_type();
  const user_op::OpKernelRegistryResult* reg = nullptr;
  JUST(user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult(op_name, rc, &reg));
  if (tmp_size_out) {
    user_op::InferSizeContext sc;
    sc.descs = in;
    sc.attrs = attrs;
    *tmp_size_out = reg->infer_tmp_size ? reg->infer_tmp_size(&sc) : 0;
    return Maybe<void>::Ok();
  }
  std::vector<std::unique_ptr<user_op::Tensor>> hold;
  std::map<std::pair<std::string, int32_t>, user_op::Tensor*> tensors;
  auto add = [&](const Arg& a) {
    hold.emplace_back(new user_op::Tensor(ShapeOf(a.d), (DataType)a.d->dtype, a.d->data,
                                          a.d->ndim == 2 ? a.d->stride[0] : -1));
    tensors[{a.name, 0}] = hold.back().get();
  };
  for (const Arg& a : ins) add(a);
  for (const Arg& o : outs) {
    CHECK_OR_RETURN(o.d != nullptr) << Error::RuntimeError() << op_name << ": NULL output " << o.name;
    JUST(CheckDesc(o.d, o.name));
    const user_op::TensorDesc& want = ictx.OutputTensorDesc(o.name, 0);
    CHECK_OR_RETURN(ShapeOf(o.d) == want.shape() && (DataType)o.d->dtype == want.data_type() &&
                    o.d->device == device)
        << Error::RuntimeError() << op_name << ": output " << o.name << " must be "
        << want.shape().ToString() << " of dtype " << DataType_Name(want.data_type());
    JUST(CheckUnitColumnStride(o.d, o.name));
    add(o);
  }
  user_op::Tensor t_tmp(Shape({(int64_t)tmp_bytes}), kChar, tmp);
  if (tmp) tensors[{"tmp_buffer", 0}] = &t_tmp;
  ep::CpuStream cpu_stream(0);
  ep::HipStream hip_stream(stream, device);
  ep::Stream* s = device < 0 ? static_cast<ep::Stream*>(&cpu_stream) : static_cast<ep::Stream*>(&hip_stream);
  user_op::KernelComputeContext ctx(s, tensors, attrs, rc.device_type());
  const user_op::OpKernel* kernel = GetKernel(reg);
  // a static CSR's plan lives in the eager op's kernel state (per registration and device)
  auto sc = attrs.find("static_csr");
  user_op::OpKernelState* kstate = nullptr;
  if (sc != attrs.end() && static_cast<int64_t>(sc->second) != 0)
    kstate = EagerKernelState(reg, kernel, device, rc.device_type());
  try {
    kernel->Compute(&ctx, kstate, nullptr);
  } catch (const KernelCheckError& e) {
    return Maybe<void>("KernelCheckError", e.msg);
  }
  return Maybe<void>::Ok();
}

}  // namespace
}  // namespace oneflow

extern "C" int ofx_functional_sddmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                                        const ofx_tensor_desc* col_idx, const ofx_tensor_desc* a,
                                        const ofx_tensor_desc* b, int64_t a_num_rows,
                                        int64_t a_num_cols, ofx_tensor_desc* out, void* tmp,
                                        size_t tmp_bytes, size_t* tmp_size_out) {
  return ofx_functional_sddmm_csr_attrs(stream, row_ptr, col_idx, a, b, a_num_rows, a_num_cols,
                                        out, tmp, tmp_bytes, tmp_size_out, nullptr);
}

// The same with the op's other attributes (static_csr: the SDDMM's plan of an unchanged CSR is
// kept in the eager op's kernel state -- the values-gradient of a static graph).
extern "C" int ofx_functional_sddmm_csr_attrs(void* stream, const ofx_tensor_desc* row_ptr,
                                              const ofx_tensor_desc* col_idx,
                                              const ofx_tensor_desc* a, const ofx_tensor_desc* b,
                                              int64_t a_num_rows, int64_t a_num_cols,
                                              ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                                              size_t* tmp_size_out, const ofx_spmm_attrs* attrs) {
  return ::ofx::guarded(__func__, [&]() -> int {
    int64_t static_csr = 0;
    if (attrs != nullptr) {
      const char* why = ofx::versioned_struct_problem(attrs, OFX_SPMM_ATTRS_MIN_SIZE);
      OFX_REQUIRE(why == nullptr, OFX_EINVAL,
                  "sddmm_csr: ofx_spmm_attrs %s (%u bytes): initialise it with "
                  "OFX_SPMM_ATTRS_INIT", why ? why : "", OFX_SPMM_ATTRS_MIN_SIZE);
      static_csr = attrs->static_csr;
    }
    return ToStatus(RunUserOp("sddmm_csr",
                              {{"a_csr_row_ptr", row_ptr}, {"a_csr_col_idx", col_idx}, {"a", a}, {"b", b}},
                              {{"out", out}},
                              {{"a_num_rows", a_num_rows}, {"a_num_cols", a_num_cols},
                               {"static_csr", static_csr}},
                              stream, tmp, tmp_bytes, tmp_size_out));
  });
}

extern "C" int ofx_functional_csr_transpose(void* stream, const ofx_tensor_desc* row_ptr,
                                            const ofx_tensor_desc* col_idx, int64_t a_num_rows,
                                            int64_t a_num_cols, ofx_tensor_desc* out_row_ptr,
                                            ofx_tensor_desc* out_col_idx, ofx_tensor_desc* out_perm,
                                            void* tmp, size_t tmp_bytes, size_t* tmp_size_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    return ToStatus(RunUserOp("csr_transpose", {{"a_csr_row_ptr", row_ptr}, {"a_csr_col_idx", col_idx}},
                              {{"out_row_ptr", out_row_ptr}, {"out_col_idx", out_col_idx}, {"out_perm", out_perm}},
                              {{"a_num_rows", a_num_rows}, {"a_num_cols", a_num_cols}}, stream, tmp,
                              tmp_bytes, tmp_size_out));
  });
}

// functional::SpmmCsrGathered: the d(b) gradient of spmm_csr with learnable values, A^T's
// structure with A's values read through A^T's perm.
extern "C" int ofx_functional_spmm_csr_gathered(void* stream, const ofx_tensor_desc* row_ptr,
                                                const ofx_tensor_desc* col_idx,
                                                const ofx_tensor_desc* values,
                                                const ofx_tensor_desc* values_perm,
                                                const ofx_tensor_desc* b, int64_t a_num_rows,
                                                int64_t a_num_cols, ofx_tensor_desc* out,
                                                void* tmp, size_t tmp_bytes,
                                                size_t* tmp_size_out) {
  return ofx_functional_spmm_csr_gathered_attrs(stream, row_ptr, col_idx, values, values_perm, b,
                                                a_num_rows, a_num_cols, out, tmp, tmp_bytes,
                                                tmp_size_out, nullptr);
}

// The same with the op's other attributes (static_csr: autograd's cached A^T keeps its plan).
extern "C" int ofx_functional_spmm_csr_gathered_attrs(
    void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
    const ofx_tensor_desc* values, const ofx_tensor_desc* values_perm, const ofx_tensor_desc* b,
    int64_t a_num_rows, int64_t a_num_cols, ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
    size_t* tmp_size_out, const ofx_spmm_attrs* attrs) {
  return ::ofx::guarded(__func__, [&]() -> int {
    int64_t static_csr = 0;
    if (attrs != nullptr) {
      const char* why = ofx::versioned_struct_problem(attrs, OFX_SPMM_ATTRS_MIN_SIZE);
      OFX_REQUIRE(why == nullptr, OFX_EINVAL,
                  "spmm_csr_gathered: ofx_spmm_attrs %s (%u bytes): initialise it with "
                  "OFX_SPMM_ATTRS_INIT", why ? why : "", OFX_SPMM_ATTRS_MIN_SIZE);
      static_csr = attrs->static_csr;
    }
    return ToStatus(RunUserOp("spmm_csr_gathered",
                              {{"a_csr_row_ptr", row_ptr}, {"a_csr_col_idx", col_idx},
                               {"a_csr_values", values}, {"values_perm", values_perm}, {"b", b}},
                              {{"out", out}},
                              {{"a_num_rows", a_num_rows}, {"a_num_cols", a_num_cols},
                               {"static_csr", static_csr}},
                              stream, tmp, tmp_bytes, tmp_size_out));
  });
}

// functional::FusedSpmmCsr: relu?(A @ b + bias?) through op
// "fused_spmm_csr"; `bias` may be NULL (the optional input is then absent).
extern "C" int ofx_functional_fused_spmm_csr(void* stream, const ofx_tensor_desc* row_ptr,
                                             const ofx_tensor_desc* col_idx,
                                             const ofx_tensor_desc* values,
                                             const ofx_tensor_desc* b, const ofx_tensor_desc* bias,
                                             int64_t a_num_rows, int64_t a_num_cols, int relu,
                                             ofx_tensor_desc* out, void* tmp, size_t tmp_bytes,
                                             size_t* tmp_size_out) {
  return ofx_functional_fused_spmm_csr_attrs(stream, row_ptr, col_idx, values, b, bias,
                                             a_num_rows, a_num_cols, relu, out, tmp, tmp_bytes,
                                             tmp_size_out, nullptr);
}

// The same with the op's other attributes (static_csr: the plan kept in the eager op's kernel
// state, as for spmm_csr).
extern "C" int ofx_functional_fused_spmm_csr_attrs(
    void* stream, const ofx_tensor_desc* row_ptr, const ofx_tensor_desc* col_idx,
    const ofx_tensor_desc* values, const ofx_tensor_desc* b, const ofx_tensor_desc* bias,
    int64_t a_num_rows, int64_t a_num_cols, int relu, ofx_tensor_desc* out, void* tmp,
    size_t tmp_bytes, size_t* tmp_size_out, const ofx_spmm_attrs* attrs) {
  return ::ofx::guarded(__func__, [&]() -> int {
    int64_t static_csr = 0;
    if (attrs != nullptr) {
      const char* why = ofx::versioned_struct_problem(attrs, OFX_SPMM_ATTRS_MIN_SIZE);
      OFX_REQUIRE(why == nullptr, OFX_EINVAL,
                  "fused_spmm_csr: ofx_spmm_attrs %s (%u bytes): initialise it with "
                  "OFX_SPMM_ATTRS_INIT", why ? why : "", OFX_SPMM_ATTRS_MIN_SIZE);
      static_csr = attrs->static_csr;
    }
    // an earlier launch's loud failure comes back here as OFX_EPLAN (as for spmm_csr)
    if (tmp_size_out == nullptr) OFX_TAKE_DEVICE_ERROR("fused_spmm_csr");
    std::vector<Arg> ins = {{"a_csr_row_ptr", row_ptr}, {"a_csr_col_idx", col_idx},
                            {"a_csr_values", values}, {"b", b}};
    if (bias != nullptr) ins.push_back({"bias", bias});
    return ToStatus(RunUserOp("fused_spmm_csr", ins, {{"out", out}},
                              {{"a_num_rows", a_num_rows}, {"a_num_cols", a_num_cols},
                               {"relu", relu ? 1 : 0}, {"static_csr", static_csr}},
                              stream, tmp, tmp_bytes, tmp_size_out));
  });
}
