// ctrl_client.cpp — host-supplied control plane of the shim (see ctrl_client.h).
#include "oneflow/core/control/ctrl_client.h"

#include <mutex>
#include <vector>

#include "ofx_internal.h"

namespace oneflow {
namespace {

struct HostCtrl {
  std::mutex mu;
  bool installed = false;
  int64_t rank = 0, world = 1;
  ofx_kv_push_fn push = nullptr;
  ofx_kv_pull_fn pull = nullptr;
  ofx_sendrecv_fn sendrecv = nullptr;
  void* user = nullptr;
};

HostCtrl& Host() {
  static HostCtrl h;
  return h;
}

}  // namespace

int64_t GlobalProcessCtx::Rank() { return Host().rank; }
int64_t GlobalProcessCtx::WorldSize() { return Host().world; }

CtrlClient* CtrlClient::Get() {
  static CtrlClient client;
  return Host().installed && Host().push && Host().pull ? &client : nullptr;
}

void CtrlClient::PushKV(const std::string& key, const std::string& val) const {
  const int rc = Host().push(Host().user, key.c_str(), val.data(), val.size());
  OFX_KERNEL_CHECK(rc == 0, "CtrlClient::PushKV(" << key << ") failed in the host store");
}

void CtrlClient::PullKV(const std::string& key,
                        const std::function<void(const std::string&)>& cb) const {
  std::vector<char> buf(4096);
  size_t len = 0;
  const int rc = Host().pull(Host().user, key.c_str(), buf.data(), buf.size(), &len);
  OFX_KERNEL_CHECK(rc == 0 && len <= buf.size(),
                   "CtrlClient::PullKV(" << key << ") failed in the host store");
  cb(std::string(buf.data(), len));
}

Maybe<void> TransportSendRecv(const void* send, size_t send_bytes, int64_t to, void* recv,
                              size_t recv_bytes, int64_t from) {
  CHECK_OR_RETURN(Host().installed && Host().sendrecv != nullptr)
      << Error::RuntimeError() << "no host transport: call ofx_process_ctx_init with a sendrecv";
  const int rc = Host().sendrecv(Host().user, send, send_bytes, to, recv, recv_bytes, from);
  CHECK_EQ_OR_RETURN(rc, 0) << Error::RuntimeError() << "host transport send/recv failed";
  return Maybe<void>::Ok();
}

namespace ctrl {
void Install(int64_t rank, int64_t world, ofx_kv_push_fn push, ofx_kv_pull_fn pull,
             ofx_sendrecv_fn sendrecv, void* user) {
  HostCtrl& h = Host();
  std::lock_guard<std::mutex> lock(h.mu);
  h.rank = rank;
  h.world = world;
  h.push = push;
  h.pull = pull;
  h.sendrecv = sendrecv;
  h.user = user;
  h.installed = true;
}
}  // namespace ctrl

}  // namespace oneflow
