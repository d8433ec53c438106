// traffic.h — algorithmic HBM bytes of homomorphic operations, counted at the operation level
// (not per kernel), for the bootstrap's roofline (bench.py "c4").
//
// "Algorithmic" = what the algorithm must move, whatever the kernels do:
//   keys        every key-switching key digit limb an inner product consumes (beta x 2 x (Ql + P)
//               limbs): keys are far larger than any cache and are read once per key switch;
//   plaintexts  every non-zero linear-transform diagonal, (Ql + P) limbs, once per level;
//   ciphertexts each homomorphic operation's operands read once and its result written once
//               (for the hoisted baby-step / giant-step transforms: the input, the baby steps
//               written and read once, the giant-step inner sums written and read once, the output).
// Intermediate traffic of this engine's kernels (modup digits, NTT passes, workspaces) is not
// counted: that is what the roofline fraction measures against.
#pragma once

#include <atomic>
#include <cstdint>

namespace phantom::traffic {

struct Counters {
  std::atomic<uint64_t> keys{0}, plaintexts{0}, ciphertexts{0};
};
Counters& counters();

inline void keys(uint64_t bytes) { counters().keys.fetch_add(bytes, std::memory_order_relaxed); }
inline void plaintexts(uint64_t bytes) { counters().plaintexts.fetch_add(bytes, std::memory_order_relaxed); }
inline void ciphertexts(uint64_t bytes) { counters().ciphertexts.fetch_add(bytes, std::memory_order_relaxed); }
// limbs x n x 8 bytes
inline uint64_t limb_bytes(uint64_t limbs, uint64_t n) { return limbs * n * 8; }

}  // namespace phantom::traffic
