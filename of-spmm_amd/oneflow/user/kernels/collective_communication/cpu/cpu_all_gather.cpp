// cpu_all_gather.cpp — ccl::AllGather for DeviceType::kCPU: the ring of the reference's
// CpuAllGather (oneflow/user/kernels/collective_communication/cpu/cpu_all_gather.cpp:27-80).
// This rank's chunk goes to its slot of `out` (skipped when `in` already is that slot); then
// P-1 steps, each sending the part received last to the next rank of the ring while receiving
// the previous rank's part, parts walked downwards from this rank's own.  Ranks of the ring are
// the placement's machines in parallel-id order.
#include <cstring>

#include "oneflow/core/control/ctrl_client.h"
#include "oneflow/user/kernels/collective_communication/cpu/cpu_communication_context.h"
#include "oneflow/user/kernels/collective_communication/include/all_gather.h"

namespace oneflow {
namespace ccl {

REGISTER_COLLECTIVE_COMMUNICATION_COMMUNICATOR(DeviceType::kCPU, CpuCommunicationContext);

namespace {

int64_t RingDecrease(int64_t i, int64_t n) { return (i - 1 + n) % n; }

Maybe<void> AllGatherImpl(const void* in, void* out, size_t elem_cnt, DataType dtype,
                          const ParallelDesc& parallel_desc) {
  const int64_t parallel_num = parallel_desc.parallel_num();
  const size_t chunk = elem_cnt * GetSizeOfDataType(dtype);
  if (parallel_num == 1) {
    if (in != out && chunk) std::memcpy(out, in, chunk);
    return Maybe<void>::Ok();
  }
  // this process's parallel id in the placement
  int64_t parallel_id = -1;
  for (int64_t p = 0; p < parallel_num; ++p)
    if (parallel_desc.MachineId4ParallelId(p) == GlobalProcessCtx::Rank()) parallel_id = p;
  CHECK_OR_RETURN(parallel_id >= 0) << Error::RuntimeError() << "process rank "
                                    << GlobalProcessCtx::Rank() << " is not in the placement";
  char* o = static_cast<char*>(out);
  const BalancedSplitter bs((int64_t)chunk * parallel_num, parallel_num);
  if (in != o + parallel_id * chunk && chunk) std::memcpy(o + parallel_id * chunk, in, chunk);
  const int64_t next = parallel_desc.MachineId4ParallelId((parallel_id + 1) % parallel_num);
  const int64_t prev = parallel_desc.MachineId4ParallelId(RingDecrease(parallel_id, parallel_num));
  for (int64_t i = 0, part = parallel_id; i < parallel_num - 1;
       ++i, part = RingDecrease(part, parallel_num)) {
    const auto s = bs.At(part);
    const auto r = bs.At(RingDecrease(part, parallel_num));
    JUST(TransportSendRecv(o + s.first, (size_t)(s.second - s.first), next, o + r.first,
                           (size_t)(r.second - r.first), prev));
  }
  return Maybe<void>::Ok();
}

}  // namespace

class CpuAllGather final : public AllGather {
 public:
  void Init(DataType datatype) override { datatype_ = datatype; }
  void Launch(ep::Stream*, const void* in, void* out, size_t elem_cnt,
              const std::shared_ptr<CommunicationContext>& communication_ctx) const override {
    const auto cpu_ctx = std::dynamic_pointer_cast<CpuCommunicationContext>(communication_ctx);
    OFX_KERNEL_CHECK(cpu_ctx != nullptr, "CpuAllGather needs a CpuCommunicationContext");
    const Maybe<void> m = AllGatherImpl(in, out, elem_cnt, datatype_, cpu_ctx->parallel_desc());
    OFX_KERNEL_CHECK(m.IsOk(), m.message());
  }

 private:
  DataType datatype_ = kInvalidDataType;
};

REGISTER_COLLECTIVE_COMMUNICATION(DeviceType::kCPU, AllGather, CpuAllGather);

}  // namespace ccl
}  // namespace oneflow
