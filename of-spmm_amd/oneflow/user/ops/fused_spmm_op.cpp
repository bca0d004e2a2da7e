/*
 * fused_spmm_op.cpp — op "fused_spmm_csr": out[M, N] = relu?(A_csr[M, K] @ b[K, N] + bias?[N]).
 *
 * The epilogue row of SURVEY.md §8f (rank 4): a GCN layer's spmm_csr -> bias_add -> relu in one
 * kernel, bit-identical to the three ops run separately (bias_add:
 * oneflow/user/kernels/bias_add_kernel.cpp:25-53; relu:
 * oneflow/core/ep/common/primitive/unary_functor.h:146-156).  Shape/dtype inference is that of
 * spmm_csr plus the bias checks of bias_add (bias 1-D, length = out dim 1, same dtype;
 * oneflow/user/ops/bias_add_op.cpp).  Optional input handled as fused ops in the reference do
 * (ctx->has_input, oneflow/core/framework/infer_util.h:71).
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/framework/op_generated.h"

namespace oneflow {

Maybe<void> SpmmCsrInferPhysicalOut(user_op::InferContext* ctx);  // spmm_op.cpp

namespace {
// The spmm_csr half of the checks reuses the spmm_csr schema functions (same input names).
Maybe<void> InferBias(user_op::InferContext* ctx) {
  if (!ctx->has_input("bias", 0)) return Maybe<void>::Ok();
  const user_op::TensorDesc& bias = ctx->InputTensorDesc("bias", 0);
  const int64_t n = ctx->InputTensorDesc("b", 0).shape().At(1);
  CHECK_EQ_OR_RETURN(bias.shape().NumAxes(), 1)
      << Error::RuntimeError() << "bias should be 1-D, got shape " << bias.shape().ToString();
  CHECK_EQ_OR_RETURN(bias.shape().At(0), n)
      << Error::RuntimeError() << "bias length " << bias.shape().At(0)
      << " should be equal to b's dim1 (" << n << "). ";
  return Maybe<void>::Ok();
}
}  // namespace

/* static */ Maybe<void> FusedSpmmCsrOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  JUST(SpmmCsrOp::InferLogicalTensorDesc(ctx));
  return InferBias(ctx);
}

/* static */ Maybe<void> FusedSpmmCsrOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  JUST(InferLogicalTensorDesc(ctx));  // bias checked against the physical b (S(0) with S(1) b)
  return SpmmCsrInferPhysicalOut(ctx);
}

/* static */ Maybe<void> FusedSpmmCsrOp::GetSbp(user_op::SbpContext* ctx) {
  const bool has_bias = ctx->user_op_conf().has_input("bias", 0);
  // Row split: bias is needed whole by every rank.
  auto row = ctx->NewBuilder();
  row.Broadcast(user_op::OpArg("a_csr_row_ptr", 0))
      .Broadcast(user_op::OpArg("a_csr_col_idx", 0))
      .Broadcast(user_op::OpArg("a_csr_values", 0))
      .Broadcast(user_op::OpArg("b", 0));
  if (has_bias) row.Broadcast(user_op::OpArg("bias", 0));
  row.Split(user_op::OpArg("out", 0), 0).Build();
  // Column split of the dense operand: bias splits with it.
  auto colsplit = ctx->NewBuilder();
  colsplit.Broadcast(user_op::OpArg("a_csr_row_ptr", 0))
      .Broadcast(user_op::OpArg("a_csr_col_idx", 0))
      .Broadcast(user_op::OpArg("a_csr_values", 0))
      .Split(user_op::OpArg("b", 0), 1);
  if (has_bias) colsplit.Split(user_op::OpArg("bias", 0), 0);
  colsplit.Split(user_op::OpArg("out", 0), 1).Build();
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> FusedSpmmCsrOp::InferDataType(user_op::InferContext* ctx) {
  JUST(SpmmCsrOp::InferDataType(ctx));
  if (ctx->has_input("bias", 0)) {
    CHECK_EQ_OR_RETURN(ctx->InputDType("bias", 0), ctx->InputDType("b", 0))
        << Error::TypeError() << "bias datatype should be equal to b. ";
  }
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> FusedSpmmCsrOp::ModifyInputArg(
    const user_op::GetInputArgModifier& GetInputArgModifierFn,
    const user_op::UserOpConfWrapper& conf) {
  return SpmmCsrOp::ModifyInputArg(GetInputArgModifierFn, conf);
}

}  // namespace oneflow
