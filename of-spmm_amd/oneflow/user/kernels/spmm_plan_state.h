// spmm_plan_state.h — the static-CSR plan store of the spmm_csr family's HIP kernels (op attr
// static_csr): the kernel state that keeps work-list plans across calls, and the helper a
// Compute uses to launch over a kept plan.  Shared by spmm_kernel.cpp (spmm_csr,
// fused_spmm_csr, spmm_csr_gathered) and sddmm_kernel.cpp (sddmm_csr).
#ifndef OFX_ONEFLOW_USER_KERNELS_SPMM_PLAN_STATE_H_
#define OFX_ONEFLOW_USER_KERNELS_SPMM_PLAN_STATE_H_

#include <list>
#include <mutex>

#include "oneflow/core/framework/framework.h"
#include "ofx_spmm.h"

namespace oneflow {

// ---- static CSR: the work-list plan kept across calls (attr static_csr) -----
// The kernel state of OpKernel::CreateOpKernelState (oneflow/core/framework/op_kernel.h:292),
// which OneFlow keeps per StatefulOpKernel (eager: per op expression and device) or per
// UserKernel (lazy).  For a caller that promises an unchanged CSR (static_csr != 0) it holds the
// planner's work list in a device workspace of its own, so the launch skips the planner kernel
// (options.planned = 1, ofx_spmm_csr_plan).  A plan is a pure function of row_ptr, the row range,
// the shapes and the schedule; the key holds those plus the static_csr value (the caller's name
// for this CSR: a new CSR at reused addresses gets a new one) and the stream (the in-kernel hub
// reduce's arrival counters live in the workspace, so two streams never share one).
class SpmmCsrPlanState final : public user_op::OpKernelState {
 public:
  struct Key {
    int64_t static_csr;
    const void* row_ptr;
    const void* stream;
    int device, idx_dt, val_dt;
    int64_t m, k, n, nnz, row_begin, row_end, split, chunk, heavy, range_nnz;
    bool operator==(const Key& o) const {
      return static_csr == o.static_csr && row_ptr == o.row_ptr && stream == o.stream &&
             device == o.device && idx_dt == o.idx_dt && val_dt == o.val_dt && m == o.m &&
             k == o.k && n == o.n && nnz == o.nnz && row_begin == o.row_begin &&
             row_end == o.row_end && split == o.split && chunk == o.chunk && heavy == o.heavy &&
             range_nnz == o.range_nnz;
    }
  };
  static constexpr size_t kMaxPlans = 8;

  // key_on_stream: an eager op's state may see calls on any stream, so the stream is part of the
  // key; a lazy op's (a compiled job's) launches are ordered on its one named stream, and its
  // graph is captured on another stream than it replays on, so the key leaves the stream out.
  explicit SpmmCsrPlanState(bool key_on_stream) : key_on_stream_(key_on_stream) {}
  ~SpmmCsrPlanState() override { Release(); }
  bool key_on_stream() const { return key_on_stream_; }
  // Held by a static call from Acquire through its launch's enqueue, so no other thread evicts
  // (and frees) the workspace in between.
  std::recursive_mutex& launch_mutex() { return mu_; }

  // The workspace for `key`: *planned = true when it already holds key's plan (a hit).  On a miss
  // a workspace of `bytes` is allocated on the key's device (past kMaxPlans the least recently
  // used entry no capture has used is evicted) and the caller plans into it; a miss while the
  // stream is capturing a graph takes no workspace (*ws = NULL: the ordinary path), as
  // allocation and eviction are not capturable.  A hit while capturing pins the entry: the graph
  // holds its pointer and may replay at any later time, so the workspace is never evicted or
  // freed before Release (the state's end, or ofx_spmm_static_plans(release = 1)).
  int Acquire(const Key& key, size_t bytes, bool capturing, void** ws, bool* planned) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    *ws = nullptr;
    *planned = false;
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      if (it->key == key && it->bytes >= bytes) {
        entries_.splice(entries_.begin(), entries_, it);  // most recently used first
        if (capturing) it->pinned = true;
        *ws = it->ws;
        *planned = true;
        ++hits_;
        return OFX_OK;
      }
    }
    if (capturing) return OFX_OK;
    int rc = OFX_OK;
    if (entries_.size() >= kMaxPlans) {
      // the least recently used unpinned entry (none: the state grows past the cap); an
      // in-flight launch may still read its plan, so the device drains first
      auto victim = entries_.end();
      for (auto it = entries_.begin(); it != entries_.end(); ++it)
        if (!it->pinned) victim = it;
      if (victim != entries_.end()) {
        rc = WithDevice(victim->key.device, [&]() {
          const int r = ofx_device_synchronize();
          return r != OFX_OK ? r : ofx_free(victim->ws);
        });
        entries_.erase(victim);
        if (rc != OFX_OK) return rc;
      }
    }
    void* p = nullptr;
    rc = WithDevice(key.device, [&]() { return ofx_malloc(&p, bytes); });
    if (rc != OFX_OK) return rc;
    entries_.push_front(Entry{key, p, bytes, false});
    *ws = p;
    ++plans_;
    return OFX_OK;
  }

  // Forget key's plan (its launch failed): the next call plans again.  A pinned entry's
  // workspace (a captured graph holds it) is retired, not freed, until Release; so is one dropped
  // while the stream captures (the device cannot be drained inside a capture).
  void Drop(const Key& key, bool capturing) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      if (it->key == key) {
        if (capturing || it->pinned) {
          retired_.push_back(*it);
        } else {
          WithDevice(it->key.device, [&]() {
            ofx_device_synchronize();
            return ofx_free(it->ws);
          });
        }
        entries_.erase(it);
        return;
      }
    }
  }

  void Stats(int64_t* entries, int64_t* plans, int64_t* hits) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    *entries += (int64_t)entries_.size();
    *plans += plans_;
    *hits += hits_;
  }

  // Frees every workspace, pinned ones included: the graphs that captured static calls of this
  // state must be gone (the state's end, or the caller's explicit release).
  void Release() {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    for (auto* list : {&retired_, &entries_}) {
      for (Entry& e : *list) {
        WithDevice(e.key.device, [&]() {
          ofx_device_synchronize();
          return ofx_free(e.ws);
        });
      }
      list->clear();
    }
  }

 private:
  struct Entry {
    Key key;
    void* ws;
    size_t bytes;
    bool pinned;  // used by a graph capture: never evicted
  };
  template <typename F>
  static int WithDevice(int device, F&& f) {
    int prev = -1;
    if (ofx_get_device(&prev) != OFX_OK) prev = -1;
    if (prev != device && ofx_set_device(device) != OFX_OK) return OFX_EDEVICE;
    const int rc = f();
    if (prev >= 0 && prev != device) ofx_set_device(prev);
    return rc;
  }

  const bool key_on_stream_;
  std::recursive_mutex mu_;  // held by Acquire / Drop / Release, and by Compute across a launch
  std::list<Entry> entries_;
  std::list<Entry> retired_;  // dropped but possibly held by a captured graph: freed at Release
  int64_t plans_ = 0, hits_ = 0;
};

// A static call on a HIP kernel (attr static_csr != 0): the workspace of `plans` holding the
// plan for `key` -- built by plan_fn(ws) on a miss -- replaces the tmp buffer (*ws, *ws_bytes)
// and the function returns true (the caller launches with planned = 1).  sp->hold keeps the
// state's lock until the launch is enqueued (the caller's scope); sp->keyed says a plan is in use
// (the caller drops it if the launch fails).  `need` = 0 (no work list) or a miss while the
// stream captures keep the ordinary path (false).
struct StaticPlan {
  SpmmCsrPlanState::Key key{};
  bool keyed = false;
  std::unique_lock<std::recursive_mutex> hold;
};

template <typename PlanFn>
bool UseStaticPlan(SpmmCsrPlanState* plans, const SpmmCsrPlanState::Key& key, size_t need,
                   bool capturing, const char* op_name, PlanFn&& plan_fn, void** ws,
                   size_t* ws_bytes, StaticPlan* sp) {
  if (need == 0) return false;
  sp->hold = std::unique_lock<std::recursive_mutex>(plans->launch_mutex());
  sp->key = key;
  void* sws = nullptr;
  bool planned = false;
  int rc = plans->Acquire(key, need, capturing, &sws, &planned);
  OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " static_csr plan workspace: " << ofx_last_error());
  if (sws == nullptr) return false;
  sp->keyed = true;
  if (!planned) {
    rc = plan_fn(sws, need);
    if (rc != OFX_OK) plans->Drop(key, capturing);
    OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " kernel failed (" << rc << "): " << ofx_last_error());
  }
  *ws = sws;
  *ws_bytes = need;
  return true;
}

}  // namespace oneflow

#endif  // OFX_ONEFLOW_USER_KERNELS_SPMM_PLAN_STATE_H_
