// bootstrapping.h — the helpers bootstrapping/bootstrapping_example.cu takes from the
// reference's bootstrapping/bootstrapping.h and include/timer.h, written for this engine, so the
// example's body compiles unchanged against the phantom:: façade.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../host/bootstrap.h"
#include "../host/ckks_eval.h"
#include "../host/encoder.h"
#include "../host/evaluate.h"
#include "../host/keys.h"
#include "../host/modulus.h"

namespace phantom::util {}  // the example's `using namespace phantom::util`

#define AUX_MOD 60

// ComputeNumLargeDigits (bootstrapping/bootstrapping.h): 3 digits above 4 towers, 2 above 1
inline uint32_t ComputeNumLargeDigits(uint32_t numLargeDigits, uint32_t multDepth) {
  if (numLargeDigits > 0) return numLargeDigits;
  return multDepth > 3 ? 3 : (multDepth > 0 ? 2 : 1);
}

// uniform reals in [min_val, max_val] from a std::random_device-seeded Mersenne Twister
inline std::vector<double> GenerateRandomVector(size_t numSlots, double min_val = 1.0, double max_val = 5.0) {
  std::random_device rd;
  std::mt19937 gen(rd());
  std::uniform_real_distribution<double> dis(min_val, max_val);
  std::vector<double> v(numSlots);
  for (auto& x : v) x = dis(gen);
  return v;
}

inline double ComputeMSE(const std::vector<double>& a, const std::vector<double>& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += (a[i] - b[i]) * (a[i] - b[i]);
  return s / static_cast<double>(a.size());
}

// the first and last `print_size` entries with `prec` decimals
template <typename T>
inline void print_vector(const std::vector<T>& vec, std::size_t print_size = 4, int prec = 3) {
  const std::size_t n = vec.size();
  std::ostringstream os;
  os << std::fixed << std::setprecision(prec) << "    [";
  if (n <= 2 * print_size) {
    for (std::size_t i = 0; i < n; ++i) os << " " << vec[i] << (i + 1 < n ? "," : " ]");
  } else {
    for (std::size_t i = 0; i < print_size; ++i) os << " " << vec[i] << ",";
    os << " ...,";
    for (std::size_t i = n - print_size; i < n; ++i) os << " " << vec[i] << (i + 1 < n ? "," : " ]");
  }
  std::cout << os.str() << std::endl;
}

// Timer (include/timer.h): accumulated device-synchronised wall time per name.  The engine runs
// on non-blocking streams, so the device is synchronised at both ends instead of recording
// events on the legacy stream.
namespace Timer {
inline std::map<std::string, double>& totals() {
  static std::map<std::string, double> t;
  return t;
}
inline std::map<std::string, std::chrono::steady_clock::time_point>& starts() {
  static std::map<std::string, std::chrono::steady_clock::time_point> s;
  return s;
}
inline void startGPUTimer(const std::string& name) {
  (void)hipDeviceSynchronize();
  starts()[name] = std::chrono::steady_clock::now();
}
inline void stopGPUTimer(const std::string& name) {
  (void)hipDeviceSynchronize();
  auto it = starts().find(name);
  if (it == starts().end()) {
    std::cerr << "[Timer] Warning: stopGPUTimer called without a matching startGPUTimer for \"" << name << "\".\n";
    return;
  }
  totals()[name] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - it->second).count();
  starts().erase(it);
}
inline void printAccumulatedTimes() {
  for (const auto& kv : totals()) std::cout << "[GPU] " << kv.first << " : " << kv.second << " ms" << std::endl;
}
}  // namespace Timer
