/*
 * spmm_op.cpp — op "spmm_csr": out[M, N] = A_csr[M, K] @ b[K, N].
 *
 * Written for OneFlow's user-op surface exactly as a new op in oneflow/user/ops would be
 * (templates: oneflow/user/ops/matrix_vector_product_op.cpp:73-107 for infer/SBP structure,
 * oneflow/user/ops/unsorted_segment_sum_op.cpp:21-80 for index-dtype checks and the
 * requires_grad=false input modifier).  Errors are CHECK_*_OR_RETURN -> Maybe -> Python
 * exception, as in the reference.
 *
 * SBP signatures:
 *   A parts B, b B,    out S(0)   row split: each rank computes its BalancedSplitter row range
 *                                 (the framework all-gathers b from S(0) -> B first).
 *   A parts B, b S(1), out S(1)   column split of the dense operand, no communication.
 *
 * Op "spmm_csr_gathered" (the d(b) gradient with learnable values) takes one more input,
 * values_perm [nnz] (A^T's perm from csr_transpose): nonzero j's value is
 * a_csr_values[values_perm[j]].  Same shapes, dtypes and SBP signatures otherwise.
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/framework/op_generated.h"

namespace oneflow {

namespace {

constexpr const char* kRowPtr = "a_csr_row_ptr";
constexpr const char* kColIdx = "a_csr_col_idx";
constexpr const char* kValues = "a_csr_values";

Maybe<void> InferTensorDesc4SpmmCsr(user_op::InferContext* ctx) {
  const user_op::TensorDesc& row_ptr = ctx->InputTensorDesc(kRowPtr, 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc(kColIdx, 0);
  const user_op::TensorDesc& values = ctx->InputTensorDesc(kValues, 0);
  const user_op::TensorDesc& b = ctx->InputTensorDesc("b", 0);
  const int64_t m = ctx->Attr<int64_t>("a_num_rows");
  const int64_t k = ctx->Attr<int64_t>("a_num_cols");
  CHECK_GE_OR_RETURN(m, 0) << Error::RuntimeError() << "a_num_rows must be non-negative. ";
  CHECK_GE_OR_RETURN(k, 0) << Error::RuntimeError() << "a_num_cols must be non-negative. ";
  CHECK_EQ_OR_RETURN(row_ptr.shape().NumAxes(), 1)
      << Error::RuntimeError() << "a_csr_row_ptr should be 1-D, got shape "
      << row_ptr.shape().ToString();
  CHECK_EQ_OR_RETURN(col_idx.shape().NumAxes(), 1)
      << Error::RuntimeError() << "a_csr_col_idx should be 1-D, got shape "
      << col_idx.shape().ToString();
  CHECK_EQ_OR_RETURN(values.shape().NumAxes(), 1)
      << Error::RuntimeError() << "a_csr_values should be 1-D, got shape "
      << values.shape().ToString();
  CHECK_EQ_OR_RETURN(b.shape().NumAxes(), 2)
      << Error::RuntimeError() << "b should be 2-D, got shape " << b.shape().ToString();
  CHECK_EQ_OR_RETURN(row_ptr.shape().At(0), m + 1)
      << Error::RuntimeError() << "a_csr_row_ptr should have a_num_rows + 1 elements. ";
  CHECK_EQ_OR_RETURN(col_idx.shape().At(0), values.shape().At(0))
      << Error::RuntimeError() << "a_csr_col_idx and a_csr_values should have nnz elements each. ";
  CHECK_EQ_OR_RETURN(b.shape().At(0), k)
      << Error::RuntimeError() << "Dim K should be equal to b's dim0 (a_num_cols). ";
  ctx->SetOutputShape("out", 0, Shape({m, b.shape().At(1)}));
  return Maybe<void>::Ok();
}

Maybe<void> InferDataType4SpmmCsr(user_op::InferContext* ctx) {
  const DataType index_dtype = ctx->InputDType(kRowPtr, 0);
  CHECK_OR_RETURN(IsIndexDataType(index_dtype))
      << Error::TypeError() << "a_csr_row_ptr should be int32 or int64, got "
      << DataType_Name(index_dtype);
  CHECK_EQ_OR_RETURN(ctx->InputDType(kColIdx, 0), index_dtype)
      << Error::TypeError() << "a_csr_col_idx should have the dtype of a_csr_row_ptr. ";
  const DataType dtype = ctx->InputDType("b", 0);
  CHECK_EQ_OR_RETURN(ctx->InputDType(kValues, 0), dtype)
      << Error::TypeError() << "a_csr_values datatype should be equal to b. ";
  CHECK_OR_RETURN(dtype == kFloat || dtype == kDouble || dtype == kFloat16 || dtype == kBFloat16)
      << Error::TypeError() << "spmm_csr supports float, double, float16, bfloat16; got "
      << DataType_Name(dtype);
  ctx->SetOutputDType("out", 0, dtype);
  return Maybe<void>::Ok();
}

Maybe<void> CheckValuesPerm(user_op::InferContext* ctx) {
  const user_op::TensorDesc& perm = ctx->InputTensorDesc("values_perm", 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc(kColIdx, 0);
  CHECK_EQ_OR_RETURN(perm.shape().NumAxes(), 1)
      << Error::RuntimeError() << "values_perm should be 1-D, got shape " << perm.shape().ToString();
  CHECK_EQ_OR_RETURN(perm.shape().At(0), col_idx.shape().At(0))
      << Error::RuntimeError() << "values_perm should have nnz elements. ";
  return Maybe<void>::Ok();
}

// Physical out of a global spmm_csr.  Every signature keeps the CSR broadcast, so the logical
// rule applied to the physical inputs gives [a_num_rows, N_phys]: right for a broadcast out and
// for the column split (b is then its S(1) slice).  A row split (out S(0)) holds only this rank's
// rows, which no input shows: they come from out's nd_sbp and the placement as GetPhysicalShape
// computes them (oneflow/core/operator/operator.cpp:1551-1626; the same pattern as
// oneflow/user/ops/affine_grid_op.cpp:113-120), so OneFlow's check of each physical blob against
// GetPhysicalShape (oneflow/core/graph/exec_graph.cpp:84-123) holds under S(0) and (S(0), S(1)).
Maybe<void> InferPhysicalOut4SpmmCsr(user_op::InferContext* ctx) {
  if (ctx->parallel_ctx().parallel_num() == 1) return Maybe<void>::Ok();
  const user_op::TensorDesc* logical_out = ctx->LogicalTensorDesc4ArgNameAndIndex("out", 0);
  CHECK_NOTNULL_OR_RETURN(logical_out) << Error::RuntimeError() << "no logical desc for out";
  Shape physical;
  JUST(GetPhysicalShape(logical_out->shape(), ctx->NdSbp4ArgNameAndIndex("out", 0),
                        ctx->parallel_desc(), ctx->parallel_ctx(), &physical));
  CHECK_EQ_OR_RETURN(physical.At(1), ctx->InputTensorDesc("b", 0).shape().At(1))
      << Error::RuntimeError() << "physical b has " << ctx->InputTensorDesc("b", 0).shape().At(1)
      << " columns but out's slice has " << physical.At(1);
  ctx->SetOutputShape("out", 0, physical);
  return Maybe<void>::Ok();
}

Maybe<void> GetSbp4SpmmCsr(user_op::SbpContext* ctx, bool with_perm) {
  // Row split: the CSR is broadcast, b is gathered to broadcast, out rows are split.
  auto row = ctx->NewBuilder();
  row.Broadcast(user_op::OpArg(kRowPtr, 0))
      .Broadcast(user_op::OpArg(kColIdx, 0))
      .Broadcast(user_op::OpArg(kValues, 0));
  if (with_perm) row.Broadcast(user_op::OpArg("values_perm", 0));
  row.Broadcast(user_op::OpArg("b", 0)).Split(user_op::OpArg("out", 0), 0).Build();
  // Column split of the dense operand: no exchange at all.
  auto col = ctx->NewBuilder();
  col.Broadcast(user_op::OpArg(kRowPtr, 0))
      .Broadcast(user_op::OpArg(kColIdx, 0))
      .Broadcast(user_op::OpArg(kValues, 0));
  if (with_perm) col.Broadcast(user_op::OpArg("values_perm", 0));
  col.Split(user_op::OpArg("b", 0), 1).Split(user_op::OpArg("out", 0), 1).Build();
  return Maybe<void>::Ok();
}

}  // namespace

// Shared with fused_spmm_csr (fused_spmm_op.cpp).
Maybe<void> SpmmCsrInferPhysicalOut(user_op::InferContext* ctx) {
  return InferPhysicalOut4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  return InferTensorDesc4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  JUST(InferLogicalTensorDesc(ctx));
  return InferPhysicalOut4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrOp::GetSbp(user_op::SbpContext* ctx) {
  return GetSbp4SpmmCsr(ctx, false);
}

/* static */ Maybe<void> SpmmCsrOp::InferDataType(user_op::InferContext* ctx) {
  return InferDataType4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrOp::ModifyInputArg(
    const user_op::GetInputArgModifier& GetInputArgModifierFn, const user_op::UserOpConfWrapper&) {
  user_op::InputArgModifier* row_ptr_modifier = GetInputArgModifierFn(kRowPtr, 0);
  CHECK_NOTNULL_OR_RETURN(row_ptr_modifier);
  row_ptr_modifier->set_requires_grad(false);
  user_op::InputArgModifier* col_idx_modifier = GetInputArgModifierFn(kColIdx, 0);
  CHECK_NOTNULL_OR_RETURN(col_idx_modifier);
  col_idx_modifier->set_requires_grad(false);
  return Maybe<void>::Ok();
}

// ---- spmm_csr_gathered ----------------------------------------------------------------------
/* static */ Maybe<void> SpmmCsrGatheredOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  JUST(CheckValuesPerm(ctx));
  return InferTensorDesc4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrGatheredOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  JUST(InferLogicalTensorDesc(ctx));
  return InferPhysicalOut4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrGatheredOp::GetSbp(user_op::SbpContext* ctx) {
  return GetSbp4SpmmCsr(ctx, true);
}

/* static */ Maybe<void> SpmmCsrGatheredOp::InferDataType(user_op::InferContext* ctx) {
  CHECK_EQ_OR_RETURN(ctx->InputDType("values_perm", 0), ctx->InputDType(kRowPtr, 0))
      << Error::TypeError() << "values_perm should have the dtype of a_csr_row_ptr. ";
  return InferDataType4SpmmCsr(ctx);
}

/* static */ Maybe<void> SpmmCsrGatheredOp::ModifyInputArg(
    const user_op::GetInputArgModifier& GetInputArgModifierFn, const user_op::UserOpConfWrapper& c) {
  JUST(SpmmCsrOp::ModifyInputArg(GetInputArgModifierFn, c));
  user_op::InputArgModifier* perm_modifier = GetInputArgModifierFn("values_perm", 0);
  CHECK_NOTNULL_OR_RETURN(perm_modifier);
  perm_modifier->set_requires_grad(false);
  return Maybe<void>::Ok();
}

}  // namespace oneflow
