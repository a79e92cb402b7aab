// parallel-gcn_amd/csrc/host/runtime.hpp -- HIP-native RAII runtime.
//
// Plays the role of the reference's dev_shared_ptr / pinned_host_ptr / smart_stream /
// smart_event (include/shared_ptr.cuh:8-330, include/smart_object.cuh:13-52): reference
// counted device buffers, pinned host buffers, streams and events, written directly against
// the HIP runtime.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <vector>

#include "../common.hpp"

namespace pgcn {

template <class T>
class DeviceBuffer {
  struct Block {
    T *p = nullptr;
    size_t n = 0;
    bool owner = true;
    std::shared_ptr<void> parent;  // keeps the owning allocation alive for slices
    ~Block() {
      if (p && owner) (void)hipFree(p);
    }
  };
  std::shared_ptr<Block> b_;

 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t n) { allocate(n); }
  void allocate(size_t n) {
    auto b = std::make_shared<Block>();
    if (n) {
      hipError_t e = hipMalloc(&b->p, n * sizeof(T));
      if (e != hipSuccess)
        throw Error(PGCN_E_NOMEM, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B) failed: " +
                                      hipGetErrorString(e));
    }
    b->n = n;
    b_ = std::move(b);
  }
  // a non-owning view of elements [off, off+n) that keeps this allocation alive
  DeviceBuffer slice(size_t off, size_t n) const {
    DeviceBuffer v;
    v.b_ = std::make_shared<Block>();
    v.b_->p = get() + off;
    v.b_->n = n;
    v.b_->owner = false;
    v.b_->parent = b_;
    return v;
  }
  T *get() const { return b_ ? b_->p : nullptr; }
  size_t size() const { return b_ ? b_->n : 0; }
  explicit operator bool() const { return get() != nullptr; }
  void upload(const T *host, size_t n, size_t offset = 0) {
    if (n) PGCN_HIP(hipMemcpy(get() + offset, host, n * sizeof(T), hipMemcpyHostToDevice));
  }
  void upload(const std::vector<T> &v) { upload(v.data(), v.size()); }
  void download(T *host, size_t n, size_t offset = 0) const {
    if (n) PGCN_HIP(hipMemcpy(host, get() + offset, n * sizeof(T), hipMemcpyDeviceToHost));
  }
  void zero_async(hipStream_t s) const {
    if (size()) PGCN_HIP(hipMemsetAsync(get(), 0, size() * sizeof(T), s));
  }
  // Complete on return: the engine's streams are non-blocking, so a memset left pending on the
  // null stream is not ordered before their later kernels (a lazily allocated buffer -- the
  // next input mask, the train-ahead product -- could be zeroed after a kernel wrote it)
  void zero() const {
    if (size()) {
      PGCN_HIP(hipMemsetAsync(get(), 0, size() * sizeof(T), nullptr));
      PGCN_HIP(hipStreamSynchronize(nullptr));
    }
  }
};

template <class T>
class PinnedBuffer {
  struct Block {
    T *p = nullptr;
    ~Block() {
      if (p) (void)hipHostFree(p);
    }
  };
  std::shared_ptr<Block> b_;
  size_t n_ = 0;

 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t n) : n_(n) {
    b_ = std::make_shared<Block>();
    PGCN_HIP(hipHostMalloc(&b_->p, n * sizeof(T), hipHostMallocDefault));
    std::memset(b_->p, 0, n * sizeof(T));
  }
  T *get() const { return b_ ? b_->p : nullptr; }
  size_t size() const { return n_; }
};

class Stream {
  struct Block {
    hipStream_t s = nullptr;
    bool owner = true;
    ~Block() {
      if (s && owner) (void)hipStreamDestroy(s);
    }
  };
  std::shared_ptr<Block> b_;

 public:
  Stream() = default;
  static Stream create(int priority = 0) {
    Stream st;
    st.b_ = std::make_shared<Block>();
    PGCN_HIP(hipStreamCreateWithPriority(&st.b_->s, hipStreamNonBlocking, priority));
    return st;
  }
  // a view of a stream owned elsewhere (the public C++ API's smart_stream)
  static Stream wrap(hipStream_t s) {
    Stream st;
    st.b_ = std::make_shared<Block>();
    st.b_->s = s;
    st.b_->owner = false;
    return st;
  }
  hipStream_t get() const { return b_ ? b_->s : nullptr; }
  void sync() const { PGCN_HIP(hipStreamSynchronize(get())); }
};

class Event {
  struct Block {
    hipEvent_t e = nullptr;
    ~Block() {
      if (e) (void)hipEventDestroy(e);
    }
  };
  std::shared_ptr<Block> b_;

 public:
  Event() = default;
  static Event create(bool timing = false) {
    Event ev;
    ev.b_ = std::make_shared<Block>();
    PGCN_HIP(hipEventCreateWithFlags(&ev.b_->e, timing ? hipEventDefault : hipEventDisableTiming));
    return ev;
  }
  hipEvent_t get() const { return b_ ? b_->e : nullptr; }
  void record(hipStream_t s) const { PGCN_HIP(hipEventRecord(get(), s)); }
  void wait_on(hipStream_t s) const { PGCN_HIP(hipStreamWaitEvent(s, get(), 0)); }
};

inline int round_up4(int d) { return (d + 3) / 4 * 4; }

}  // namespace pgcn
