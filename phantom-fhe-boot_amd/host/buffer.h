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
// to another stream once that event has completed.  Blocks are never returned to the driver
// (except to satisfy a failed hipMalloc).
// Replaces hipMallocAsync / hipFreeAsync: with ROCm 7.2's stream-ordered pool, reused blocks
// were observed to still be in use (key-switching keys and ciphertexts corrupted; reproduced by
// examples/bootstrapping_example ops, gone with synchronous allocation).
//  * Small requests (< kArenaMin) are cached by power-of-two size class.
//  * Large requests are carved best-fit out of arena chunks (kChunk, or the request when larger)
//    in kGrain units; a block is split on allocation and coalesced with free neighbours on free,
//    the merged block carrying every pending (stream, event) of its parts.  Held memory then tracks
//    the live set instead of one cached copy per distinct size (the bootstrap's per-level buffers
//    differ by a limb or two).
class DevicePool {
 public:
  static DevicePool& instance();
  void* alloc(size_t bytes, hipStream_t s);
  // completed: the caller has synchronised the device (no event needed)
  void free(void* p, size_t bytes, hipStream_t s, bool completed = false);
  // stream `s` is about to be destroyed and has been synchronised: its cached blocks become
  // plain free blocks (a later stream may reuse the handle value; an event recorded on a
  // destroyed stream must not be queried)
  void forget_stream(hipStream_t s);
  struct Stats {
    size_t held = 0;       // bytes obtained from hipMalloc and not returned
    size_t live = 0;       // bytes handed out and not freed
    size_t peak_live = 0;  // maximum of `live` since the last reset_peak()
    size_t peak_held = 0;
  };
  Stats stats();
  void reset_peak();
  static constexpr size_t kArenaMin = size_t(1) << 20;  // requests from here are carved from the arena
  static constexpr size_t kGrain = size_t(64) << 10;    // arena block granularity
  static constexpr size_t kChunk = size_t(1) << 30;     // arena growth step
  static constexpr size_t kSlackMin = size_t(2) << 30;  // cached arena space kept before waiting on reuse

 private:
  // Uses a block may still have: at most one per stream, the newest.  A use is a stream and a
  // stamp number: the free happened before that stream's stamp `stamp` (a marker event recorded on
  // the stream after the free; a stream's stamps complete in order).  Frees only take the stream's
  // open stamp number; the event is recorded once for all the frees since the last one, when the
  // pool is next asked for memory (stamp_dirty), so a burst of frees costs one marker on the
  // device instead of one each.
  struct Use {
    hipStream_t first;
    uint64_t stamp;
  };
  using Pending = std::vector<Use>;
  struct Stamps {
    uint64_t open = 1;   // the stamp the next frees belong to (not recorded yet)
    uint64_t done = 0;   // every stamp up to this one has completed
    bool dirty = false;  // frees took `open` since it was last recorded
    std::vector<std::pair<uint64_t, hipEvent_t>> recorded;  // in flight, oldest first
  };
  struct Small {
    void* p;
    hipStream_t stream;
    uint64_t stamp;  // 0 when known complete
  };
  struct Chunk;
  struct Block {
    Chunk* chunk = nullptr;
    size_t off = 0, size = 0;
    bool free = true;
    size_t req = 0;  // live blocks: the rounded request they were handed out for
    Pending pending;
  };
  struct Chunk {
    char* base = nullptr;
    size_t size = 0;
    int dev = 0;
    std::map<size_t, Block> blocks;  // by offset, covering the chunk
  };
  std::mutex mu_;
  // small blocks: (device, class) -> cached blocks
  std::map<std::pair<int, size_t>, std::vector<Small>> small_free_;
  std::map<void*, size_t> small_live_;  // handed-out small block -> its class
  // arena
  std::vector<Chunk*> chunks_;
  std::multimap<std::pair<int, size_t>, Block*> by_size_;  // free arena blocks by (device, size)
  std::map<void*, Block*> live_;                           // handed-out arena blocks
  std::vector<hipEvent_t> spare_;
  std::map<hipStream_t, Stamps> stamps_;
  Stats st_;
  static size_t size_class(size_t bytes);
  hipEvent_t take_event();
  bool ready_for(Pending& pend, hipStream_t s);  // drops completed uses
  void drop_done(Pending& pend);
  void add_use(Pending& pend, Use u);  // keeps the newest use per stream
  Use note_free(hipStream_t s);        // the use a free on `s` leaves
  void stamp_dirty();                  // records the open stamp of every stream with frees since its last
  bool use_done(const Use& u);
  void wait_use(hipStream_t s, const Use& u);  // device-side: `s` waits for the stamp of u
  Chunk* add_chunk(int dev, void* p, size_t sz);
  void insert_free(Block* b);
  void erase_free(Block* b);
  void* carve(int dev, size_t c, hipStream_t s, bool wait = false);
  Chunk* grow(int dev, size_t c, std::unique_lock<std::mutex>& lk);  // hipMalloc with lk released
  void release_cached_locked();
  void note_live(long delta);
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
