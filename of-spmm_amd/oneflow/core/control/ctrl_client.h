// ctrl_client.h — the control plane the collective layer needs, reduced to what OneFlow's
// collectives use from it and supplied by the host through the C-ABI (ofx_process_ctx_init):
//   GlobalProcessCtx::Rank()        oneflow/core/rpc/include/global_process_ctx.h
//   CtrlClient::PushKV / PullKV     oneflow/core/control/ctrl_client.h (the RCCL unique id
//                                   exchange of EagerNcclCommMgr, eager_nccl_comm_manager.cpp:68-74)
//   TransportUtil ring send / recv  oneflow/core/framework/transport_util.h (the CPU all-gather
//                                   ring, collective_communication/cpu/cpu_all_gather.cpp:27-80)
// OneFlow's own control plane (gRPC ctrl server, transport over epoll) is out of scope
// (DESIGN.md §8): a host that embeds this library passes its store and point-to-point moves
// (torch.distributed's TCPStore and gloo in oneflow_spmm/ccl.py).
#ifndef OFX_ONEFLOW_SHIM_CTRL_CLIENT_H_
#define OFX_ONEFLOW_SHIM_CTRL_CLIENT_H_

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>

#include "ofx_spmm.h"
#include "oneflow/core/framework/framework.h"

namespace oneflow {

class GlobalProcessCtx {
 public:
  static int64_t Rank();
  static int64_t WorldSize();
};

class CtrlClient {
 public:
  static CtrlClient* Get();  // nullptr until the host has installed a control plane
  void PushKV(const std::string& key, const std::string& val) const;
  // Blocks until `key` exists, then hands its value to `cb`.
  void PullKV(const std::string& key, const std::function<void(const std::string&)>& cb) const;
};

// One step of a ring: send `send_bytes` to rank `to` while receiving `recv_bytes` from rank
// `from` (either size may be 0); returns when both are done.
Maybe<void> TransportSendRecv(const void* send, size_t send_bytes, int64_t to, void* recv,
                              size_t recv_bytes, int64_t from);

namespace ctrl {
// Installed by ofx_process_ctx_init.
void Install(int64_t rank, int64_t world, ofx_kv_push_fn push, ofx_kv_pull_fn pull,
             ofx_sendrecv_fn sendrecv, void* user);
}  // namespace ctrl

}  // namespace oneflow

#endif  // OFX_ONEFLOW_SHIM_CTRL_CLIENT_H_
