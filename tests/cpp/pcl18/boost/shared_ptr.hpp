// Stand-in for boost::shared_ptr (test fixture, see ../README.md): a distinct smart-pointer type
// with boost's surface; it deliberately does not convert to or from std::shared_ptr.
#pragma once
#include <cstddef>
#include <memory>

namespace boost {
template <class T>
class shared_ptr {
  public:
    using element_type = T;
    shared_ptr() noexcept = default;
    template <class Y>
    explicit shared_ptr(Y* p) : p_(p) {}
    template <class Y>
    shared_ptr(const shared_ptr<Y>& o) noexcept : p_(o.p_) {}  // Y* -> T* (e.g. T = const Y)
    T* get() const noexcept { return p_.get(); }
    T& operator*() const noexcept { return *p_; }
    T* operator->() const noexcept { return p_.get(); }
    explicit operator bool() const noexcept { return static_cast<bool>(p_); }
    void reset() noexcept { p_.reset(); }
    long use_count() const noexcept { return p_.use_count(); }

  private:
    template <class Y>
    friend class shared_ptr;
    std::shared_ptr<T> p_;  // storage only; never exposed as a std::shared_ptr
};
}  // namespace boost
