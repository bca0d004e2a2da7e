/*
 * ccl_ops.cpp — the two S(0) -> B all-gather ops the row-split spmm_csr's dense operand goes
 * through (SBP signature a_csr_*: B, b: B, out: S(0); the producer of b is S(0)):
 *   eager_ccl_all_gather      eager boxing "ccl-s-to-b" (oneflow/core/boxing/ccl_boxing_function.cpp:
 *                             185-215 -> functional::GlobalAllGather -> this op); semantics as
 *                             oneflow/user/ops/eager_nccl_ops.cpp:188-233
 *   _nccl_logical_all_gather  what the lazy compiler inserts for S(0) -> B
 *                             (oneflow/core/job_rewriter/insert_nccl_logical_op_pass.cpp:189-198);
 *                             semantics as oneflow/user/ops/nccl_logical_ops.cpp:104-142
 * Both: out's logical shape is in's; in is S(0), out is B on every hierarchy axis.
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/framework/op_generated.h"

namespace oneflow {

/* static */ Maybe<void> EagerCclAllGatherOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  ctx->SetOutputShape("out", 0, ctx->InputShape("in", 0));
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> EagerCclAllGatherOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  return InferLogicalTensorDesc(ctx);
}

/* static */ Maybe<void> EagerCclAllGatherOp::GetSbp(user_op::SbpContext* ctx) {
  // GetSbpFnUtil::DefaultBroadcastToBroadcast
  ctx->NewBuilder().Broadcast(user_op::OpArg("in", 0)).Broadcast(user_op::OpArg("out", 0)).Build();
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> EagerCclAllGatherOp::InferNdSbp(user_op::InferNdSbpFnContext* ctx) {
  const NdSbp& in_dis_hint = ctx->NdSbpHint4InputArgNameAndIndex("in", 0);
  CHECK_GE_OR_RETURN(in_dis_hint.size(), 1u);
  for (const std::string& sbp_hint : in_dis_hint) {
    CHECK_EQ_OR_RETURN(SplitAxisOf(sbp_hint), 0) << Error::RuntimeError()
                                                 << "eager_ccl_all_gather needs S(0) input, got "
                                                 << sbp_hint;
  }
  NdSbp* in_nd_sbp = ctx->NdSbp4ArgNameAndIndex("in", 0);
  NdSbp* out_nd_sbp = ctx->NdSbp4ArgNameAndIndex("out", 0);
  in_nd_sbp->clear();
  out_nd_sbp->clear();
  const Shape& parallel_hierarchy = ctx->parallel_hierarchy();
  CHECK_GE_OR_RETURN(parallel_hierarchy.NumAxes(), 1);
  for (int64_t i = 0; i < parallel_hierarchy.NumAxes(); ++i) {  // S(0) -> B
    in_nd_sbp->push_back("S(0)");
    out_nd_sbp->push_back("B");
  }
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> EagerCclAllGatherOp::InferDataType(user_op::InferContext* ctx) {
  ctx->SetOutputDType("out", 0, ctx->InputDType("in", 0));
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> _ncclLogicalAllGatherOp::InferLogicalTensorDesc(
    user_op::InferContext* ctx) {
  ctx->SetOutputShape("out", 0, ctx->InputShape("in", 0));
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> _ncclLogicalAllGatherOp::GetSbp(user_op::SbpContext* ctx) {
  ctx->NewBuilder().Broadcast(user_op::OpArg("in", 0)).Broadcast(user_op::OpArg("out", 0)).Build();
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> _ncclLogicalAllGatherOp::InferNdSbp(user_op::InferNdSbpFnContext* ctx) {
  NdSbp* input_nd_sbp = ctx->NdSbp4ArgNameAndIndex("in", 0);
  NdSbp* output_nd_sbp = ctx->NdSbp4ArgNameAndIndex("out", 0);
  *input_nd_sbp = ctx->Attr<std::vector<std::string>>("src_reduced_nd_sbp");
  *output_nd_sbp = ctx->Attr<std::vector<std::string>>("dst_reduced_nd_sbp");
  // S(0)->B on a 1-D hierarchy
  CHECK_EQ_OR_RETURN(input_nd_sbp->size(), 1u);
  CHECK_EQ_OR_RETURN(output_nd_sbp->size(), 1u);
  CHECK_EQ_OR_RETURN(SplitAxisOf(input_nd_sbp->at(0)), 0)
      << Error::RuntimeError() << "_nccl_logical_all_gather: src must be S(0)";
  CHECK_OR_RETURN(output_nd_sbp->at(0) == "B")
      << Error::RuntimeError() << "_nccl_logical_all_gather: dst must be B";
  CHECK_EQ_OR_RETURN(ctx->parallel_hierarchy().NumAxes(), 1);
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> _ncclLogicalAllGatherOp::InferDataType(user_op::InferContext* ctx) {
  ctx->SetOutputDType("out", 0, ctx->InputDType("in", 0));
  return Maybe<void>::Ok();
}

}  // namespace oneflow
