/*
 * sddmm_op.cpp / csr_transpose — the gradient ops of "spmm_csr" (SURVEY.md §8f row 1).
 *
 *   sddmm_csr(a_csr_row_ptr, a_csr_col_idx, a[M,N], b[K,N]) -> out[nnz]
 *       out[j] = <a[row(j), :], b[col(j), :]>        (d values of spmm_csr: a = d out)
 *   csr_transpose(a_csr_row_ptr, a_csr_col_idx) -> out_row_ptr[K+1], out_col_idx[nnz], out_perm[nnz]
 *       structure of A^T; A^T's values are values[out_perm] (d b of spmm_csr = A^T @ d out)
 * Same conventions as spmm_op.cpp (templates oneflow/user/ops/matrix_vector_product_op.cpp:73-107,
 * unsorted_segment_sum_op.cpp:21-80).
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/framework/op_generated.h"

namespace oneflow {

namespace {

Maybe<void> CheckCsrStructure(user_op::InferContext* ctx, int64_t* nnz) {
  const user_op::TensorDesc& row_ptr = ctx->InputTensorDesc("a_csr_row_ptr", 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc("a_csr_col_idx", 0);
  const int64_t m = ctx->Attr<int64_t>("a_num_rows");
  CHECK_GE_OR_RETURN(m, 0) << Error::RuntimeError() << "a_num_rows must be non-negative. ";
  CHECK_GE_OR_RETURN(ctx->Attr<int64_t>("a_num_cols"), 0)
      << Error::RuntimeError() << "a_num_cols must be non-negative. ";
  CHECK_EQ_OR_RETURN(row_ptr.shape().NumAxes(), 1)
      << Error::RuntimeError() << "a_csr_row_ptr should be 1-D. ";
  CHECK_EQ_OR_RETURN(col_idx.shape().NumAxes(), 1)
      << Error::RuntimeError() << "a_csr_col_idx should be 1-D. ";
  CHECK_EQ_OR_RETURN(row_ptr.shape().At(0), m + 1)
      << Error::RuntimeError() << "a_csr_row_ptr should have a_num_rows + 1 elements. ";
  *nnz = col_idx.shape().At(0);
  return Maybe<void>::Ok();
}

Maybe<void> CheckIndexTypes(user_op::InferContext* ctx) {
  const DataType index_dtype = ctx->InputDType("a_csr_row_ptr", 0);
  CHECK_OR_RETURN(IsIndexDataType(index_dtype))
      << Error::TypeError() << "a_csr_row_ptr should be int32 or int64, got "
      << DataType_Name(index_dtype);
  CHECK_EQ_OR_RETURN(ctx->InputDType("a_csr_col_idx", 0), index_dtype)
      << Error::TypeError() << "a_csr_col_idx should have the dtype of a_csr_row_ptr. ";
  return Maybe<void>::Ok();
}

}  // namespace

/* static */ Maybe<void> SddmmCsrOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  int64_t nnz = 0;
  JUST(CheckCsrStructure(ctx, &nnz));
  const user_op::TensorDesc& a = ctx->InputTensorDesc("a", 0);
  const user_op::TensorDesc& b = ctx->InputTensorDesc("b", 0);
  CHECK_EQ_OR_RETURN(a.shape().NumAxes(), 2) << Error::RuntimeError() << "a should be 2-D. ";
  CHECK_EQ_OR_RETURN(b.shape().NumAxes(), 2) << Error::RuntimeError() << "b should be 2-D. ";
  CHECK_EQ_OR_RETURN(a.shape().At(0), ctx->Attr<int64_t>("a_num_rows"))
      << Error::RuntimeError() << "a should have a_num_rows rows. ";
  CHECK_EQ_OR_RETURN(b.shape().At(0), ctx->Attr<int64_t>("a_num_cols"))
      << Error::RuntimeError() << "b should have a_num_cols rows. ";
  CHECK_EQ_OR_RETURN(a.shape().At(1), b.shape().At(1))
      << Error::RuntimeError() << "a and b should have the same number of columns. ";
  ctx->SetOutputShape("out", 0, Shape({nnz}));
  return Maybe<void>::Ok();
}
/* static */ Maybe<void> SddmmCsrOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  return InferLogicalTensorDesc(ctx);
}
/* static */ Maybe<void> SddmmCsrOp::GetSbp(user_op::SbpContext* ctx) {
  // Split N: each rank holds a column slice of a and b; partial dot products sum to the whole.
  ctx->NewBuilder()
      .Broadcast(user_op::OpArg("a_csr_row_ptr", 0))
      .Broadcast(user_op::OpArg("a_csr_col_idx", 0))
      .Split(user_op::OpArg("a", 0), 1)
      .Split(user_op::OpArg("b", 0), 1)
      .PartialSum(user_op::OpArg("out", 0))
      .Build();
  return Maybe<void>::Ok();
}
/* static */ Maybe<void> SddmmCsrOp::InferDataType(user_op::InferContext* ctx) {
  JUST(CheckIndexTypes(ctx));
  const DataType dtype = ctx->InputDType("b", 0);
  CHECK_EQ_OR_RETURN(ctx->InputDType("a", 0), dtype)
      << Error::TypeError() << "a datatype should be equal to b. ";
  CHECK_OR_RETURN(dtype == kFloat || dtype == kDouble || dtype == kFloat16 || dtype == kBFloat16)
      << Error::TypeError() << "sddmm_csr supports float, double, float16, bfloat16; got "
      << DataType_Name(dtype);
  ctx->SetOutputDType("out", 0, dtype);
  return Maybe<void>::Ok();
}

/* static */ Maybe<void> CsrTransposeOp::InferLogicalTensorDesc(user_op::InferContext* ctx) {
  int64_t nnz = 0;
  JUST(CheckCsrStructure(ctx, &nnz));
  ctx->SetOutputShape("out_row_ptr", 0, Shape({ctx->Attr<int64_t>("a_num_cols") + 1}));
  ctx->SetOutputShape("out_col_idx", 0, Shape({nnz}));
  ctx->SetOutputShape("out_perm", 0, Shape({nnz}));
  return Maybe<void>::Ok();
}
/* static */ Maybe<void> CsrTransposeOp::InferPhysicalTensorDesc(user_op::InferContext* ctx) {
  return InferLogicalTensorDesc(ctx);
}
/* static */ Maybe<void> CsrTransposeOp::GetSbp(user_op::SbpContext* ctx) {
  ctx->NewBuilder()
      .Broadcast(user_op::OpArg("a_csr_row_ptr", 0))
      .Broadcast(user_op::OpArg("a_csr_col_idx", 0))
      .Broadcast(user_op::OpArg("out_row_ptr", 0))
      .Broadcast(user_op::OpArg("out_col_idx", 0))
      .Broadcast(user_op::OpArg("out_perm", 0))
      .Build();
  return Maybe<void>::Ok();
}
/* static */ Maybe<void> CsrTransposeOp::InferDataType(user_op::InferContext* ctx) {
  JUST(CheckIndexTypes(ctx));
  const DataType index_dtype = ctx->InputDType("a_csr_row_ptr", 0);
  ctx->SetOutputDType("out_row_ptr", 0, index_dtype);
  ctx->SetOutputDType("out_col_idx", 0, index_dtype);
  ctx->SetOutputDType("out_perm", 0, index_dtype);
  return Maybe<void>::Ok();
}

}  // namespace oneflow
