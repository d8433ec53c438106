#include "buffer.h"

namespace phantom {

DevicePool& DevicePool::instance() {
  static DevicePool* p = new DevicePool();  // never destroyed: blocks outlive static teardown
  return *p;
}

size_t DevicePool::size_class(size_t bytes) {
  if (bytes <= 512) return 512;
  if (bytes < (size_t(1) << 20)) {
    size_t c = 512;
    while (c < bytes) c <<= 1;
    return c;
  }
  const size_t g = size_t(2) << 20;  // 2 MiB granules above 1 MiB
  return (bytes + g - 1) / g * g;
}

hipEvent_t DevicePool::take_event() {
  if (!spare_.empty()) {
    hipEvent_t e = spare_.back();
    spare_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  PHX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

void DevicePool::release_cached_locked() {
  for (auto& kv : free_) {
    std::vector<Block> keep;
    for (Block& b : kv.second) {
      if (b.ev && hipEventQuery(b.ev) != hipSuccess) {
        keep.push_back(b);
        continue;
      }
      if (b.ev) spare_.push_back(b.ev);
      (void)hipFree(b.p);
    }
    kv.second.swap(keep);
  }
}

void* DevicePool::alloc(size_t bytes, hipStream_t s) {
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  const size_t c = size_class(bytes);
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = free_.find({dev, c});
    if (it != free_.end()) {
      auto& v = it->second;
      for (size_t i = v.size(); i-- > 0;) {
        Block& b = v[i];
        const bool ready = !b.ev || b.stream == s || hipEventQuery(b.ev) == hipSuccess;
        if (!ready) continue;
        void* p = b.p;
        if (b.ev) spare_.push_back(b.ev);
        v.erase(v.begin() + static_cast<long>(i));
        live_[p] = c;
        return p;
      }
    }
  }
  void* p = nullptr;
  if (hipMalloc(&p, c) != hipSuccess) {
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> lk(mu_);
      release_cached_locked();
    }
    PHX_CHECK(hipMalloc(&p, c));
  }
  std::lock_guard<std::mutex> lk(mu_);
  live_[p] = c;
  return p;
}

void DevicePool::free(void* p, size_t bytes, hipStream_t s, bool completed) {
  if (!p) return;
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu_);
  auto it = live_.find(p);
  if (it == live_.end() || it->second != size_class(bytes)) {
    std::fprintf(stderr, "DevicePool: free of %p (%zu bytes) that is not a live block (double free?)\n", p, bytes);
    std::abort();
  }
  live_.erase(it);
  Block b{p, s, nullptr};
  if (!completed) {
    b.ev = take_event();
    PHX_CHECK(hipEventRecord(b.ev, s));
  }
  free_[{dev, size_class(bytes)}].push_back(b);
}

}  // namespace phantom
