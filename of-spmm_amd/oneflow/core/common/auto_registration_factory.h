// auto_registration_factory.h — keyed class registry of the OneFlow shim: the behaviour of
// oneflow/core/common/auto_registration_factory.h (REGISTER_CLASS / NewObj / NewObjUniquePtr /
// IsClassRegistered) that the collective-communication layer registers its per-device-type
// implementations with (REGISTER_COLLECTIVE_COMMUNICATION, collective_communication.h).
#ifndef OFX_ONEFLOW_SHIM_AUTO_REGISTRATION_FACTORY_H_
#define OFX_ONEFLOW_SHIM_AUTO_REGISTRATION_FACTORY_H_

#include <functional>
#include <map>
#include <memory>
#include <mutex>

#include "oneflow/core/framework/framework.h"

namespace oneflow {

template <typename Key, typename Base>
class AutoRegistrationFactory {
 public:
  using Creator = std::function<Base*()>;
  static AutoRegistrationFactory& Get() {
    static AutoRegistrationFactory f;
    return f;
  }
  void Register(const Key& k, Creator c) {
    std::lock_guard<std::mutex> lock(mu_);
    creators_[k] = std::move(c);  // one implementation per key (a later one replaces it)
  }
  Base* New(const Key& k) const {
    std::lock_guard<std::mutex> lock(mu_);
    auto it = creators_.find(k);
    return it == creators_.end() ? nullptr : it->second();
  }
  bool Has(const Key& k) const {
    std::lock_guard<std::mutex> lock(mu_);
    return creators_.count(k) > 0;
  }

 private:
  mutable std::mutex mu_;
  std::map<Key, Creator> creators_;
};

template <typename Key, typename Base>
struct AutoRegisterer {
  AutoRegisterer(const Key& k, typename AutoRegistrationFactory<Key, Base>::Creator c) {
    AutoRegistrationFactory<Key, Base>::Get().Register(k, std::move(c));
  }
};

template <typename Key, typename Base>
Base* NewObj(const Key& k) {
  return AutoRegistrationFactory<Key, Base>::Get().New(k);
}
template <typename Key, typename Base>
std::unique_ptr<Base> NewObjUniquePtr(const Key& k) {
  return std::unique_ptr<Base>(NewObj<Key, Base>(k));
}
template <typename Key, typename Base>
bool IsClassRegistered(const Key& k) {
  return AutoRegistrationFactory<Key, Base>::Get().Has(k);
}

}  // namespace oneflow

#define REGISTER_CLASS(KeyT, key, Base, Derived)                                          \
  static ::oneflow::AutoRegisterer<KeyT, Base> OFX_PP_CAT(g_auto_register, __COUNTER__)( \
      key, []() -> Base* { return new Derived(); })

#endif  // OFX_ONEFLOW_SHIM_AUTO_REGISTRATION_FACTORY_H_
