// buffer.h — stream-ordered device buffers (the reference's cuda_auto_ptr,
// include/cuda_wrapper.cuh:74-219), on hipMallocAsync / hipFreeAsync.  PhantomContext raises the
// default pool's release threshold so freed blocks stay cached for reuse, as the reference
// does for its CUDA pool (src/context.cu:127-131).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "hip_check.h"

namespace phantom {

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

  // Stream-ordered allocation only on a real stream: on the null stream it corrupted live
  // buffers on ROCm 7.2 (a freed block handed out again while kernels still used it; reproduced
  // by examples/bootstrapping_example dbg, gone with synchronous allocation).  Null-stream
  // buffers therefore use plain hipMalloc / hipFree.
  void allocate(size_t count, hipStream_t stream) {
    release();
    async_ = stream != nullptr;
    if (count) {
      if (async_) PHX_CHECK(hipMallocAsync(reinterpret_cast<void**>(&ptr_), count * sizeof(T), stream));
      else PHX_CHECK(hipMalloc(reinterpret_cast<void**>(&ptr_), count * sizeof(T)));
    }
    count_ = count;
    stream_ = stream;
  }
  void release() {
    if (ptr_) {
      if (async_) (void)hipFreeAsync(ptr_, stream_);
      else (void)hipFree(ptr_);
    }
    ptr_ = nullptr;
    count_ = 0;
  }
  // free without touching the owning stream (which may no longer exist); the caller has
  // synchronised the device
  void release_sync() {
    if (ptr_) (void)hipFree(ptr_);
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
  explicit operator bool() const { return ptr_ != nullptr; }

 private:
  void swap(DeviceBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(count_, o.count_);
    std::swap(stream_, o.stream_);
    std::swap(async_, o.async_);
  }
  T* ptr_ = nullptr;
  size_t count_ = 0;
  hipStream_t stream_ = nullptr;
  bool async_ = false;
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
  enum Slot : int { kModupInv = 0, kModdownDelta, kRescaleLast, kRescaleTmp, kKsModup, kKsCx, kSlots };
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
