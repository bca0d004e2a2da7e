// ccl_boxing_function.cpp — see the header.
#include "oneflow/core/boxing/ccl_boxing_function.h"

namespace oneflow {

namespace {

bool NdSbpIsAllSplit(const NdSbp& nd_sbp, int64_t axis) {
  for (const auto& s : nd_sbp)
    if (SplitAxisOf(s) != axis) return false;
  return !nd_sbp.empty();
}
bool NdSbpIsAllBroadcast(const NdSbp& nd_sbp) {
  for (const auto& s : nd_sbp)
    if (s != "B") return false;
  return !nd_sbp.empty();
}

// CheckCclKernelRegistered (ccl_boxing_function.cpp:29-38): a kernel of `op` for the device type.
Maybe<void> CheckCclKernelRegistered(const std::string& op, DeviceType device_type) {
  user_op::KernelRegContext rc;
  rc.device_type_ = device_type;
  const user_op::OpKernelRegistryResult* reg = nullptr;
  return user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult(op, rc, &reg);
}

}  // namespace

Maybe<void> CheckCclS2B(const PlacedNdSbp& in, const PlacedNdSbp& out, const Shape& logical_shape) {
  CHECK_EQ_OR_RETURN(in.nd_sbp.size(), 1u);
  CHECK_EQ_OR_RETURN(out.nd_sbp.size(), 1u);
  CHECK_OR_RETURN(NdSbpIsAllSplit(in.nd_sbp, 0));
  CHECK_OR_RETURN(NdSbpIsAllBroadcast(out.nd_sbp));
  CHECK_GT_OR_RETURN(logical_shape.NumAxes(), 0);
  CHECK_OR_RETURN(logical_shape.At(0) % in.placement.parallel_num() == 0)
      << "logical dim 0 (" << logical_shape.At(0) << ") is not divisible by the "
      << in.placement.parallel_num() << " ranks";
  CHECK_OR_RETURN(in.placement == out.placement);
  JUST(CheckCclKernelRegistered("eager_ccl_all_gather", in.placement.device_type()));
  return Maybe<void>::Ok();
}

Maybe<void> CclS2B(ep::Stream* stream, const user_op::Tensor& in, user_op::Tensor* out,
                   const PlacedNdSbp& in_p, const PlacedNdSbp& out_p, const Shape& logical_shape,
                   int64_t parallel_id) {
  JUST(CheckCclS2B(in_p, out_p, logical_shape));
  // functional::GlobalAllGather -> OpInterpUtil::Dispatch of eager_ccl_all_gather
  const user_op::OpRegistryResult* op =
      user_op::UserOpRegistryMgr::Get().GetOpRegistryResult("eager_ccl_all_gather");
  CHECK_OR_RETURN(op != nullptr) << Error::RuntimeError() << "eager_ccl_all_gather not registered";
  const ParallelDesc& pd = in_p.placement;
  user_op::InferContext lctx({{{"in", 0}, user_op::TensorDesc(logical_shape, in.data_type())}}, {});
  JUST(op->logical_infer(&lctx));
  JUST(op->dtype_infer(&lctx));
  user_op::InferNdSbpFnContext sctx(*pd.hierarchy(), {{"in", in_p.nd_sbp}});
  JUST(op->nd_sbp_infer(&sctx));
  const ParallelContext pc(parallel_id, pd.parallel_num());
  Shape in_phys, out_phys;
  JUST(GetPhysicalShape(logical_shape, sctx.NdSbp4ArgName("in"), pd, pc, &in_phys));
  JUST(GetPhysicalShape(lctx.OutputTensorDesc("out", 0).shape(), sctx.NdSbp4ArgName("out"), pd, pc,
                        &out_phys));
  CHECK_OR_RETURN(in.shape_view() == in_phys)
      << Error::RuntimeError() << "ccl-s-to-b: input is " << in.shape_view().ToString()
      << ", this rank's S(0) slice is " << in_phys.ToString();
  CHECK_OR_RETURN(out->shape_view() == out_phys && out->data_type() == in.data_type())
      << Error::RuntimeError() << "ccl-s-to-b: output must be " << out_phys.ToString();
  user_op::KernelRegContext rc;
  rc.device_type_ = pd.device_type();
  rc.dtypes[{"in", 0}] = rc.dtypes[{"out", 0}] = in.data_type();
  const user_op::OpKernelRegistryResult* reg = nullptr;
  JUST(user_op::UserOpRegistryMgr::Get().GetOpKernelRegistryResult("eager_ccl_all_gather", rc, &reg));
  std::unique_ptr<user_op::OpKernel> kernel(reg->create_fn());
  user_op::Tensor t_in = in;
  std::map<std::pair<std::string, int32_t>, user_op::Tensor*> tensors = {{{"in", 0}, &t_in},
                                                                         {{"out", 0}, out}};
  user_op::KernelCacheContext cache_ctx(pc, pd, {{"in", sctx.NdSbp4ArgName("in")},
                                                 {"out", sctx.NdSbp4ArgName("out")}},
                                        {{"out", lctx.OutputTensorDesc("out", 0)}}, pd.device_type());
  user_op::KernelComputeContext ctx(stream, tensors, {}, pd.device_type());
  ctx.set_parallel_ctx(pc);
  try {
    std::shared_ptr<user_op::OpKernelCache> cache = kernel->InitOpKernelCache(&cache_ctx);
    if (out->shape_view().elem_cnt() == 0 && !kernel->AlwaysComputeWhenAllOutputsEmpty())
      return Maybe<void>::Ok();
    kernel->Compute(&ctx, nullptr, cache.get());
  } catch (const KernelCheckError& e) {
    return Maybe<void>("KernelCheckError", e.msg);
  }
  return Maybe<void>::Ok();
}

}  // namespace oneflow
