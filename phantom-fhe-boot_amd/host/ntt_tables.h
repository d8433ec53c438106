// ntt_tables.h — host construction of device NTT tables (the reference's host NTT class,
// src/host/ntt.cu:11-56, uploaded like PhantomContext does at context.cu:170-183).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "../csrc/ntt.h"

namespace phantom {

struct HostNttTable {
  uint64_t q = 0;
  uint64_t psi = 0;
  std::vector<uint64_t> tw, tw_shoup, itw, itw_shoup;
  uint64_t n_inv = 0, n_inv_shoup = 0;
};

// tw[brv(i)] = psi^i, itw[brv(i)] = psi^-i with psi the minimal primitive 2n-th root.
HostNttTable make_host_ntt_table(size_t n, uint64_t q);

// Owns the device arrays of a phx::NttTables.
class DeviceNttTables {
 public:
  DeviceNttTables() = default;
  DeviceNttTables(size_t n, const std::vector<uint64_t>& moduli, hipStream_t stream);
  ~DeviceNttTables();
  DeviceNttTables(const DeviceNttTables&) = delete;
  DeviceNttTables& operator=(const DeviceNttTables&) = delete;

  const phx::NttTables& get() const { return t_; }
  size_t n() const { return t_.n; }
  size_t size() const { return t_.num_moduli; }
  const std::vector<uint64_t>& moduli() const { return moduli_; }

 private:
  phx::NttTables t_;
  std::vector<uint64_t> moduli_;
};

}  // namespace phantom
