// buffer.h — device buffers (the reference's cuda_auto_ptr, include/cuda_wrapper.cuh:74-219) on
// a caching allocator (DevicePool): freed blocks stay cached for reuse, as the reference keeps
// its CUDA pool's blocks (src/context.cu:127-131).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "hip_check.h"

namespace phantom {

// Caching device allocator.  A freed block is kept with an event recorded on the stream that
// freed it; it is handed out again to the same stream at once (stream order protects it) or
// to another stream once that event has completed.  Blocks are never returned to the driver.
// Replaces hipMallocAsync / hipFreeAsync: with ROCm 7.2's stream-ordered pool, reused blocks
// were observed to still be in use (key-switching keys and ciphertexts corrupted; reproduced by
// examples/bootstrapping_example ops, gone with synchronous allocation).
class DevicePool {
 public:
  static DevicePool& instance();
  void* alloc(size_t bytes, hipStream_t s);
  // completed: the caller has synchronised the device (no event needed)
  void free(void* p, size_t bytes, hipStream_t s, bool completed = false);
  // size class of a request (blocks are reused only within a class)
  static size_t size_class(size_t bytes);
  // stream `s` is about to be destroyed and has been synchronised: its cached blocks become
  // plain free blocks (a later stream may reuse the handle value; an event recorded on a
  // destroyed stream must not be queried)
  void forget_stream(hipStream_t s);

 private:
  struct Block {
    void* p;
    hipStream_t stream;
    hipEvent_t ev;  // null when known complete
  };
  std::mutex mu_;
  static constexpr size_t kSlackMin = size_t(4) << 20;          // requests from here may take a block up to 1/4 larger
  std::map<std::pair<int, size_t>, std::vector<Block>> free_;  // (device, class) -> blocks
  std::map<void*, size_t> live_;                               // handed-out blocks (double-free check)
  std::vector<hipEvent_t> spare_;
  size_t held_ = 0;  // bytes obtained from hipMalloc and not returned (live + cached)
  hipEvent_t take_event();
  void release_cached_locked();
};

template <typename T>
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(size_t count, hipStream_t stream) { allocate(count, stream); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept { swap(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }

  void allocate(size_t count, hipStream_t stream) {
    release();
    if (count) {
      ptr_ = static_cast<T*>(DevicePool::instance().alloc(count * sizeof(T) + kGuardBytes, stream));
#ifdef PHX_GUARD
      PHX_CHECK(hipDeviceSynchronize());
      PHX_CHECK(hipMemset(reinterpret_cast<char*>(ptr_) + count * sizeof(T), 0xA5, kGuardBytes));
#endif
    }
    count_ = count;
    stream_ = stream;
  }
  void release() {
    if (ptr_) {
#ifdef PHX_GUARD
      check_guard();
#endif
      DevicePool::instance().free(ptr_, count_ * sizeof(T) + kGuardBytes, stream_);
    }
    ptr_ = nullptr;
    count_ = 0;
  }
#ifdef PHX_GUARD
  // debug builds: a 0xA5 guard region after every buffer, checked when the buffer is freed
  static constexpr size_t kGuardBytes = size_t(1) << 20;
  void check_guard() const {
    (void)hipDeviceSynchronize();
    std::vector<unsigned char> g(kGuardBytes);
    (void)hipMemcpy(g.data(), reinterpret_cast<const char*>(ptr_) + count_ * sizeof(T), kGuardBytes,
                    hipMemcpyDeviceToHost);
    for (size_t i = 0; i < kGuardBytes; ++i)
      if (g[i] != 0xA5) {
        std::fprintf(stderr, "GUARD VIOLATION: buffer of %zu bytes (%zu elements of %zu B), first bad guard byte +%zu\n",
                     count_ * sizeof(T), count_, sizeof(T), i);
        std::abort();
      }
  }
#else
  static constexpr size_t kGuardBytes = 0;
#endif
  // free without touching the owning stream (which may no longer exist); the caller has
  // synchronised the device
  void release_sync() {
    if (ptr_) DevicePool::instance().free(ptr_, count_ * sizeof(T) + kGuardBytes, nullptr, true);
    ptr_ = nullptr;
    count_ = 0;
  }
  // setup-path upload: waits for the copy so the host source may be a temporary
  void upload(const T* host, size_t count, hipStream_t stream) {
    allocate(count, stream);
    if (count) {
      PHX_CHECK(hipMemcpyAsync(ptr_, host, count * sizeof(T), hipMemcpyHostToDevice, stream));
      PHX_CHECK(hipStreamSynchronize(stream));
    }
  }
  void upload(const std::vector<T>& v, hipStream_t stream) { upload(v.data(), v.size(), stream); }
  std::vector<T> download(hipStream_t stream) const {
    std::vector<T> v(count_);
    if (count_) {
      PHX_CHECK(hipMemcpyAsync(v.data(), ptr_, count_ * sizeof(T), hipMemcpyDeviceToHost, stream));
      PHX_CHECK(hipStreamSynchronize(stream));
    }
    return v;
  }

  T* get() const { return ptr_; }
  size_t size() const { return count_; }
  hipStream_t stream() const { return stream_; }
  // make `s` the stream the buffer is freed on (its event and immediate reuse): for a buffer
  // made on one stream whose later uses are all ordered on `s`
  void set_stream(hipStream_t s) { stream_ = s; }
  explicit operator bool() const { return ptr_ != nullptr; }

 private:
  void swap(DeviceBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(count_, o.count_);
    std::swap(stream_, o.stream_);
  }
  T* ptr_ = nullptr;
  size_t count_ = 0;
  hipStream_t stream_ = nullptr;
};

// Scratch buffers reused across calls, one set per stream (the reference allocates its
// key-switch and rescale temporaries on every call, e.g. src/eval_key_switch.cu:150-160).
// A buffer only grows; the old one is freed stream-ordered on the stream that used it.
// Buffers of one stream are used in that stream's order, so reuse needs no synchronisation.
class Workspace {
 public:
  Workspace() = default;
  Workspace(const Workspace&) = delete;
  Workspace& operator=(const Workspace&) = delete;
  ~Workspace() {
    (void)hipDeviceSynchronize();
    for (auto& kv : bufs_)
      for (auto& b : kv.second) b.release_sync();
  }
  enum Slot : int { kModupInv = 0, kModdownDelta, kRescaleLast, kKsModup, kKsCx, kSlots };
  uint64_t* get(hipStream_t s, Slot slot, size_t count) {
    std::lock_guard<std::mutex> lk(mu_);
    DeviceBuffer<uint64_t>& b = bufs_[s][slot];
    if (b.size() < count) b.allocate(count, s);
    return b.get();
  }

 private:
  std::mutex mu_;
  std::map<hipStream_t, DeviceBuffer<uint64_t>[kSlots]> bufs_;
};

}  // namespace phantom
