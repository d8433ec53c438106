// stream_fork.cpp — see stream_fork.h.
#include "stream_fork.h"

#include <map>
#include <mutex>
#include <utility>

namespace phx {

StreamFork& StreamFork::get(hipStream_t caller, int lanes) {
  static std::mutex mu;
  // never destroyed: the HIP runtime may already be torn down when static destructors run
  static auto* forks = new std::map<std::pair<int, hipStream_t>, StreamFork*>();
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  StreamFork*& f = (*forks)[{dev, caller}];
  if (!f) {
    f = new StreamFork();
    f->caller_ = caller;
  }
  // aux streams / events are created on first use, up to the lanes asked for
  for (; f->made_ < lanes && f->made_ < kMaxForkLanes; ++f->made_) {
    const int k = f->made_ - 1;
    if (hipStreamCreateWithFlags(&f->aux_[k], hipStreamNonBlocking) != hipSuccess) break;
    if (hipEventCreateWithFlags(&f->join_ev_[k], hipEventDisableTiming) != hipSuccess) {
      (void)hipStreamDestroy(f->aux_[k]);
      f->aux_[k] = nullptr;
      break;
    }
  }
  if (!f->fork_ev_ && hipEventCreateWithFlags(&f->fork_ev_, hipEventDisableTiming) != hipSuccess)
    f->fork_ev_ = nullptr;
  return *f;
}

hipError_t StreamFork::fork(int lanes) {
  if (lanes > made_ || !fork_ev_) return hipErrorNotReady;
  if (lanes <= 1) return hipSuccess;
  hipError_t e = hipEventRecord(fork_ev_, caller_);
  for (int k = 0; k + 1 < lanes && e == hipSuccess; ++k) e = hipStreamWaitEvent(aux_[k], fork_ev_, 0);
  return e;
}

hipError_t StreamFork::join(int lanes) {
  hipError_t e = hipSuccess;
  for (int k = 0; k + 1 < lanes && e == hipSuccess; ++k) {
    e = hipEventRecord(join_ev_[k], aux_[k]);
    if (e == hipSuccess) e = hipStreamWaitEvent(caller_, join_ev_[k], 0);
  }
  return e;
}

}  // namespace phx
