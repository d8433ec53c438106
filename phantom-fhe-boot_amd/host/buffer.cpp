#include "buffer.h"

#include <algorithm>
#include <iterator>
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
  size_t c = 512;
  while (c < bytes) c <<= 1;
  return c;
}

// The pool's events only order device work (hipStreamWaitEvent) and tell the host that a block's
// last use has finished (hipEventQuery); nothing the host reads depends on them.  So they are
// recorded without the system-scope release fence: with it, every record is a marker that writes
// back the L2s before the stream's next kernel may start, and the frees of one operation (often
// ten or more between two kernels) left 10-55 us idle gaps on the device per operation
// (profiles/r06/pool_fence/).  Kernels end with a device-scope release, so a block's old contents
// are in memory before its event completes.
#ifndef PHX_POOL_SYSTEM_FENCE
#define PHX_POOL_SYSTEM_FENCE 0
#endif
hipEvent_t DevicePool::take_event() {
  if (!spare_.empty()) {
    hipEvent_t e = spare_.back();
    spare_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  PHX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | (PHX_POOL_SYSTEM_FENCE ? 0 : hipEventDisableSystemFence)));
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

void DevicePool::add_use(Pending& pend, Use u) {
  for (Use& x : pend)
    if (x.first == u.first) {
      if (u.stamp > x.stamp) x = u;
      return;
    }
  pend.push_back(u);
}

DevicePool::Use DevicePool::note_free(hipStream_t s) {
  Stamps& st = stamps_[s];
  st.dirty = true;
  return Use{s, st.open};
}

void DevicePool::stamp_dirty() {
  for (auto& kv : stamps_) {
    Stamps& st = kv.second;
    if (!st.dirty) continue;
    hipEvent_t ev = take_event();
    PHX_CHECK(hipEventRecord(ev, kv.first));
    st.recorded.emplace_back(st.open, ev);
    ++st.open;
    st.dirty = false;
  }
}

// a use is done when its stamp has completed; an unrecorded (open) stamp is not done
bool DevicePool::use_done(const Use& u) {
  Stamps& st = stamps_[u.first];
  size_t k = 0;
  while (u.stamp > st.done && k < st.recorded.size() && event_done(st.recorded[k].second)) {
    st.done = st.recorded[k].first;
    spare_.push_back(st.recorded[k].second);
    ++k;
  }
  if (k) st.recorded.erase(st.recorded.begin(), st.recorded.begin() + static_cast<long>(k));
  return u.stamp <= st.done;
}

void DevicePool::wait_use(hipStream_t s, const Use& u) {
  if (use_done(u)) return;
  for (const auto& r : stamps_[u.first].recorded)
    if (r.first >= u.stamp) {  // (stamp_dirty ran first: the use's stamp is recorded)
      PHX_CHECK(hipStreamWaitEvent(s, r.second, 0));
      return;
    }
  PHX_CHECK(hipStreamSynchronize(u.first));  // (unreachable: an unrecorded stamp) wait on the host
}

void DevicePool::drop_done(Pending& pend) {
  for (size_t i = pend.size(); i-- > 0;)
    if (use_done(pend[i])) pend.erase(pend.begin() + static_cast<long>(i));
}

// a block whose last uses were on `s` (stream order) or have completed may be reused on `s`
bool DevicePool::ready_for(Pending& pend, hipStream_t s) {
  bool ready = true;
  for (size_t i = pend.size(); i-- > 0;) {
    if (pend[i].first == s) continue;
    if (use_done(pend[i]))
      pend.erase(pend.begin() + static_cast<long>(i));
    else
      ready = false;
  }
  return ready;
}

void DevicePool::insert_free(Block* b) { by_size_.emplace(std::make_pair(b->chunk->dev, b->size), b); }

void DevicePool::erase_free(Block* b) {
  auto r = by_size_.equal_range({b->chunk->dev, b->size});
  for (auto it = r.first; it != r.second; ++it)
    if (it->second == b) {
      by_size_.erase(it);
      return;
    }
}

void DevicePool::note_live(long delta) {
  st_.live = static_cast<size_t>(static_cast<long>(st_.live) + delta);
  if (st_.live > st_.peak_live) st_.peak_live = st_.live;
  if (st_.held > st_.peak_held) st_.peak_held = st_.held;
}

// best fit among the free blocks of the device that are ready for `s`; splits off the rest.  With
// `wait`, the best fit among all free blocks: `s` is made to wait (on the device) for the pending
// uses of the block on other streams, as a stream-ordered allocator reuses another stream's block.
void* DevicePool::carve(int dev, size_t c, hipStream_t s, bool wait) {
  if (wait) stamp_dirty();  // (frees may have come in while grow() had the lock released)
  for (auto it = by_size_.lower_bound({dev, c}); it != by_size_.end() && it->first.first == dev; ++it) {
    Block* b = it->second;
    if (!ready_for(b->pending, s)) {
      if (!wait) continue;
      for (const Use& u : b->pending)
        if (u.first != s) wait_use(s, u);
    }
    by_size_.erase(it);
    if (b->size > c) {  // the remainder stays free with the pending uses of the whole block
      Block rest;
      rest.chunk = b->chunk;
      rest.off = b->off + c;
      rest.size = b->size - c;
      rest.pending = std::move(b->pending);
      Block* r = &b->chunk->blocks.emplace(rest.off, std::move(rest)).first->second;
      insert_free(r);
      b->size = c;
    }
    b->pending.clear();  // (all on `s`, or waited for: stream order covers them)
    b->free = false;
    b->req = c;
    void* p = b->chunk->base + b->off;
    live_[p] = b;
    note_live(static_cast<long>(c));
    return p;
  }
  return nullptr;
}

// hipMalloc of a 1 GiB chunk takes milliseconds: the other lanes' threads keep allocating and
// freeing meanwhile (the caller re-runs carve after the chunk is added, so a block freed in
// between is also found)
DevicePool::Chunk* DevicePool::grow(int dev, size_t c, std::unique_lock<std::mutex>& lk) {
  const size_t sz = std::max(c, kChunk);
  void* p = nullptr;
  lk.unlock();
  const hipError_t r = hipMalloc(&p, sz);
  lk.lock();
  if (r != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return add_chunk(dev, p, sz);
}

DevicePool::Chunk* DevicePool::add_chunk(int dev, void* p, size_t sz) {
  Chunk* ch = new Chunk();
  ch->base = static_cast<char*>(p);
  ch->size = sz;
  ch->dev = dev;
  Block b;
  b.chunk = ch;
  b.off = 0;
  b.size = sz;
  insert_free(&ch->blocks.emplace(0, std::move(b)).first->second);
  chunks_.push_back(ch);
  st_.held += sz;
  return ch;
}

void DevicePool::forget_stream(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : small_free_)
    for (Small& b : kv.second)
      if (b.stream == s) {
        // the caller has synchronised s: its blocks are free for any stream from now on
        b.stamp = 0;
        b.stream = nullptr;
      }
  for (auto& kv : by_size_) {
    Pending& pend = kv.second->pending;
    for (size_t i = pend.size(); i-- > 0;)
      if (pend[i].first == s) pend.erase(pend.begin() + static_cast<long>(i));
  }
  // (a later stream may reuse the handle value: it starts with fresh stamps)
  auto it = stamps_.find(s);
  if (it != stamps_.end()) {
    for (auto& r : it->second.recorded) spare_.push_back(r.second);
    stamps_.erase(it);
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

// frees the cached small blocks and the arena chunks that are wholly free, whose uses completed
void DevicePool::release_cached_locked() {
  const size_t held0 = st_.held;
  size_t freed = 0;
  for (auto& kv : small_free_) {
    std::vector<Small> keep;
    for (Small& b : kv.second) {
      if (b.stamp && !use_done(Use{b.stream, b.stamp})) {
        keep.push_back(b);
        continue;
      }
      (void)hipFree(b.p);
      st_.held -= kv.first.second;
      freed += kv.first.second;
    }
    kv.second.swap(keep);
  }
  for (size_t i = chunks_.size(); i-- > 0;) {
    Chunk* ch = chunks_[i];
    if (ch->blocks.size() != 1) continue;
    Block& b = ch->blocks.begin()->second;
    if (!b.free) continue;
    drop_done(b.pending);
    if (!b.pending.empty()) continue;
    erase_free(&b);
    (void)hipFree(ch->base);
    st_.held -= ch->size;
    freed += ch->size;
    delete ch;
    chunks_.erase(chunks_.begin() + static_cast<long>(i));
  }
  if (pool_trace())
    std::fprintf(stderr, "{\"pool_release\": true, \"held_MiB\": %zu, \"freed_MiB\": %zu, \"live_MiB\": %zu}\n",
                 held0 >> 20, freed >> 20, st_.live >> 20);
}

void* DevicePool::alloc(size_t bytes, hipStream_t s) {
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  if (bytes >= kArenaMin) {
    const size_t c = (bytes + kGrain - 1) / kGrain * kGrain;
    std::unique_lock<std::mutex> lk(mu_);
    stamp_dirty();
    if (void* p = carve(dev, c, s)) return p;
    // Free blocks that are still in use by other streams: once the cached space exceeds the slack,
    // reuse one behind a device-side wait instead of growing (the held memory then tracks the live
    // set plus the slack; the lanes of a batch wait at most for another lane's last use of a block)
    const size_t cached = st_.held - st_.live;
    if (cached > std::max(kSlackMin, st_.live / 16))
      if (void* p = carve(dev, c, s, true)) return p;
    if (grow(dev, c, lk)) return carve(dev, c, s);
    // out of device memory: return wholly free chunks and cached small blocks, then wait for every
    // pending use so that all free blocks coalesce into reusable space
    release_cached_locked();
    if (grow(dev, c, lk)) return carve(dev, c, s);
    if (void* p = carve(dev, c, s, true)) return p;
    stamp_dirty();
    PHX_CHECK(hipDeviceSynchronize());  // every stamp recorded so far completes
    if (void* p = carve(dev, c, s)) return p;
    release_cached_locked();
    if (!grow(dev, c, lk)) PHX_CHECK(hipErrorOutOfMemory);
    return carve(dev, c, s);
  }
  const size_t c = size_class(bytes);
  {
    std::lock_guard<std::mutex> lk(mu_);
    stamp_dirty();
    auto it = small_free_.find({dev, c});
    if (it != small_free_.end()) {
      auto& v = it->second;
      for (size_t i = v.size(); i-- > 0;) {
        Small& b = v[i];
        const bool ready = !b.stamp || b.stream == s || use_done(Use{b.stream, b.stamp});
        if (!ready) continue;
        void* p = b.p;
        v.erase(v.begin() + static_cast<long>(i));
        small_live_[p] = c;
        note_live(static_cast<long>(c));
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
  small_live_[p] = c;
  st_.held += c;
  note_live(static_cast<long>(c));
  return p;
}

void DevicePool::free(void* p, size_t bytes, hipStream_t s, bool completed) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(mu_);
  if (bytes >= kArenaMin) {
    auto it = live_.find(p);
    const size_t c = (bytes + kGrain - 1) / kGrain * kGrain;
    if (it == live_.end() || it->second->req != c) {
      std::fprintf(stderr, "DevicePool: free of %p (%zu bytes) that is not a live block of that size (double free?)\n",
                   p, bytes);
      std::abort();
    }
    Block* b = it->second;
    live_.erase(it);
    note_live(-static_cast<long>(b->size));
#ifdef PHX_GUARD
    // debug builds: poison the block in the freeing stream's order, so a stream that still reads it
    // after this free (a buffer freed on a stream other than its last user's) reads garbage and the
    // results show it
    if (!completed) PHX_CHECK(hipMemsetAsync(p, 0xFF, b->size, s));
#endif
    b->free = true;
    b->req = 0;
    if (!completed) add_use(b->pending, note_free(s));
    // coalesce with free neighbours (their pending uses move into the merged block)
    auto& blocks = b->chunk->blocks;
    auto me = blocks.find(b->off);
    if (me != blocks.begin()) {
      auto prev = std::prev(me);
      if (prev->second.free) {
        Block* pb = &prev->second;
        erase_free(pb);
        pb->size += b->size;
        for (const Use& u : b->pending) add_use(pb->pending, u);
        blocks.erase(me);
        b = pb;
        me = prev;
      }
    }
    auto nx = std::next(me);
    if (nx != blocks.end() && nx->second.free) {
      Block* nb = &nx->second;
      erase_free(nb);
      b->size += nb->size;
      for (const Use& u : nb->pending) add_use(b->pending, u);
      blocks.erase(nx);
    }
    drop_done(b->pending);
    insert_free(b);
    return;
  }
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  auto it = small_live_.find(p);
  if (it == small_live_.end() || it->second != size_class(bytes)) {
    std::fprintf(stderr, "DevicePool: free of %p (%zu bytes) that is not a live block (double free?)\n", p, bytes);
    std::abort();
  }
  const size_t cls = it->second;
  small_live_.erase(it);
  note_live(-static_cast<long>(cls));
  Small b{p, s, 0};
#ifdef PHX_GUARD
  if (!completed) PHX_CHECK(hipMemsetAsync(p, 0xFF, cls, s));
#endif
  if (!completed) b.stamp = note_free(s).stamp;
  small_free_[{dev, cls}].push_back(b);
}

DevicePool::Stats DevicePool::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

void DevicePool::reset_peak() {
  std::lock_guard<std::mutex> lk(mu_);
  st_.peak_live = st_.live;
  st_.peak_held = st_.held;
}

}  // namespace phantom
