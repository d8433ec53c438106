// stream_fork.h — fork one caller stream into helper streams and join them back, for launchers
// that pipeline one operation's independent pieces (limb chunks of one NTT) across HIP streams.
//
// The reference enqueues everything on cudaStreamPerThread; a C-ABI caller here
// hands one hipStream_t per call.  A launcher that wants the GPU to overlap the column pass of
// chunk k+1 with the row pass of chunk k (each pass pays a ~2 us HBM-latency ramp and a ~3 us
// store tail) needs more than one hardware queue, so the helper keeps, per
// (device, caller stream), a few non-blocking aux streams and events:
//   fork:  record e_fork on the caller; every aux stream waits on it;
//   ...    the launcher enqueues piece i on lane i % lanes (lane 0 = the caller);
//   join:  every aux stream records e_join[k]; the caller waits on each.
// Stream semantics for the caller are unchanged: work enqueued on the caller after the join
// runs after every piece, and the pieces run after everything enqueued before the fork.
#pragma once

#include <hip/hip_runtime.h>

namespace phx {

constexpr int kMaxForkLanes = 4;

class StreamFork {
 public:
  // lanes (1..kMaxForkLanes) including the caller; fewer lanes than requested are never returned
  static StreamFork& get(hipStream_t caller, int lanes);
  // enqueue the fork; returns the lane streams (lane 0 = caller)
  hipError_t fork(int lanes);
  hipError_t join(int lanes);
  hipStream_t lane(int i) const { return i == 0 ? caller_ : aux_[i - 1]; }
  int lanes_available() const { return fork_ev_ ? made_ : 1; }

 private:
  hipStream_t caller_ = nullptr;
  hipStream_t aux_[kMaxForkLanes - 1] = {};
  hipEvent_t fork_ev_ = nullptr;
  hipEvent_t join_ev_[kMaxForkLanes - 1] = {};
  int made_ = 1;  // lanes created so far
};

}  // namespace phx
