#include "buffer.h"
#include "traffic.h"

namespace phantom {

traffic::Counters& traffic::counters() {
  static Counters c;
  return c;
}

bool debug_sync_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_DEBUG_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

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

// hipEventQuery of a pending event returns hipErrorNotReady, and HIP keeps every API return value
// as the thread's last error: left there, it would be reported by the next launch's
// hipGetLastError() as that launch's failure.  Clear it.
static bool event_done(hipEvent_t e) {
  const hipError_t r = hipEventQuery(e);
  if (r == hipSuccess) return true;
  if (r == hipErrorNotReady) (void)hipGetLastError();
  return false;
}

void DevicePool::forget_stream(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : free_)
    for (Block& b : kv.second)
      if (b.stream == s) {
        // the caller has synchronised s: its blocks are free for any stream from now on
        if (b.ev) spare_.push_back(b.ev);
        b.ev = nullptr;
        b.stream = nullptr;
      }
}

// PHX_POOL_TRACE=1: one stderr line per out-of-memory release of the cache
static bool pool_trace() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_POOL_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

void DevicePool::release_cached_locked() {
  size_t cached = 0, freed = 0;
  for (auto& kv : free_) cached += kv.first.second * kv.second.size();
  const size_t held0 = held_;
  for (auto& kv : free_) {
    std::vector<Block> keep;
    for (Block& b : kv.second) {
      if (b.ev && !event_done(b.ev)) {
        keep.push_back(b);
        continue;
      }
      if (b.ev) spare_.push_back(b.ev);
      (void)hipFree(b.p);
      held_ -= kv.first.second;
      freed += kv.first.second;
    }
    kv.second.swap(keep);
  }
  if (pool_trace())
    std::fprintf(stderr, "{\"pool_release\": true, \"held_MiB\": %zu, \"cached_MiB\": %zu, \"freed_MiB\": %zu}\n",
                 held0 >> 20, cached >> 20, freed >> 20);
}

void* DevicePool::alloc(size_t bytes, hipStream_t s) {
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  const size_t c = size_class(bytes);
  {
    std::lock_guard<std::mutex> lk(mu_);
    // the exact class first; a large request may also take a cached block up to a quarter larger
    // (the bootstrap's per-level buffers differ by a limb or two: without the slack each level
    // keeps its own cached copies, and lockstep groups of them fill the GPU)
#ifndef PHX_POOL_SLACK_Q
#define PHX_POOL_SLACK_Q 1  // the slack in quarters of the request
#endif
    const size_t top = c >= kSlackMin ? c + c * PHX_POOL_SLACK_Q / 4 : c;
    for (auto it = free_.lower_bound({dev, c}); it != free_.end() && it->first.first == dev && it->first.second <= top;
         ++it) {
      auto& v = it->second;
      for (size_t i = v.size(); i-- > 0;) {
        Block& b = v[i];
        const bool ready = !b.ev || b.stream == s || event_done(b.ev);
        if (!ready) continue;
        void* p = b.p;
        if (b.ev) spare_.push_back(b.ev);
        v.erase(v.begin() + static_cast<long>(i));
        live_[p] = it->first.second;  // the block's own class: it returns there
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
  held_ += c;
  return p;
}

void DevicePool::free(void* p, size_t bytes, hipStream_t s, bool completed) {
  if (!p) return;
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu_);
  auto it = live_.find(p);
  if (it == live_.end() || it->second < size_class(bytes)) {
    std::fprintf(stderr, "DevicePool: free of %p (%zu bytes) that is not a live block (double free?)\n", p, bytes);
    std::abort();
  }
  const size_t cls = it->second;
  live_.erase(it);
  Block b{p, s, nullptr};
#ifdef PHX_GUARD
  // debug builds: poison the block in the freeing stream's order, so a stream that still reads it
  // after this free (a buffer freed on a stream other than its last user's) reads garbage and the
  // results show it
  if (!completed) PHX_CHECK(hipMemsetAsync(p, 0xFF, cls, s));
#endif
  if (!completed) {
    b.ev = take_event();
    PHX_CHECK(hipEventRecord(b.ev, s));
  }
  free_[{dev, cls}].push_back(b);
}

}  // namespace phantom
