// framework.cpp — implementation of the minimal OneFlow framework shim (framework.h).
#include "oneflow/core/framework/framework.h"

#include "ofx_spmm.h"

namespace oneflow {

const char* DataType_Name(DataType dt) {
  switch (dt) {
    case kChar: return "kChar";
    case kFloat: return "kFloat";
    case kDouble: return "kDouble";
    case kInt8: return "kInt8";
    case kInt32: return "kInt32";
    case kInt64: return "kInt64";
    case kUInt8: return "kUInt8";
    case kFloat16: return "kFloat16";
    case kBFloat16: return "kBFloat16";
    case kBool: return "kBool";
    default: return "kInvalidDataType";
  }
}

const char* DeviceTypeName(DeviceType t) {
  switch (t) {
    case DeviceType::kCPU: return "cpu";
    case DeviceType::kCUDA: return "cuda";
    case DeviceType::kHIP: return "hip";
    case DeviceType::kMockDevice: return "mock";
    default: return "invalid";
  }
}

std::string Shape::ToString() const {
  std::ostringstream os;
  os << "(";
  for (size_t i = 0; i < dims_.size(); ++i) os << (i ? "," : "") << dims_[i];
  if (dims_.size() == 1) os << ",";
  os << ")";
  return os.str();
}

BalancedSplitter::BalancedSplitter(int64_t total_num, int64_t split_num)
    : total_(total_num), parts_(split_num) {}

std::pair<int64_t, int64_t> BalancedSplitter::At(int64_t idx) const {
  int64_t b = 0, e = 0;
  ofx_balanced_range(total_, parts_, idx, &b, &e);
  return {b, e};
}

namespace user_op {

UserOpRegistryMgr& UserOpRegistryMgr::Get() {
  static UserOpRegistryMgr mgr;
  return mgr;
}

Maybe<void> UserOpRegistryMgr::GetOpKernelRegistryResult(const std::string& op,
                                                         const KernelRegContext& ctx,
                                                         const OpKernelRegistryResult** out) const {
  const OpKernelRegistryResult* found = nullptr;
  int matched = 0;
  std::string tried;
  for (const auto& k : kernels_) {
    if (k.op_type_name != op) continue;
    tried += "\n  " + k.is_matched.debug;
    if (k.is_matched(ctx)) {
      found = &k;
      ++matched;
    }
  }
  if (matched == 0)
    return Maybe<void>("OpKernelNotFoundError",
                       "cannot find the kernel matching the current context: op " + op +
                           " on device " + DeviceTypeName(ctx.device_type) +
                           " with dtype " + DataType_Name(ctx.dtype("out", 0)) +
                           "; registered kernels:" + tried);
  if (matched > 1)
    return Maybe<void>("MultipleOpKernelsMatchedError",
                       "there are more than one kernels matching the current context: op " + op);
  *out = found;
  return Maybe<void>::Ok();
}

}  // namespace user_op
}  // namespace oneflow
