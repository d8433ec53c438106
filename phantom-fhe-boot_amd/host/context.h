// context.h — EncryptionParameters, PhantomContext and per-level ContextData, mirroring the
// reference's include/host/encryptionparams.h and include/context.cuh:16-272 (CKKS subset).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <stdexcept>
#include <vector>

#include "modulus.h"
#include "ntt_tables.h"
#include "rns_tool.h"

namespace phantom {

enum class scheme_type : uint8_t { none = 0, bfv = 1, ckks = 2, bgv = 3 };

// EncryptionParameters (include/host/encryptionparams.h): the CKKS fields this engine uses.
class EncryptionParameters {
 public:
  explicit EncryptionParameters(scheme_type scheme = scheme_type::ckks) : scheme_(scheme) {}
  void set_poly_modulus_degree(size_t n) { poly_modulus_degree_ = n; }
  void set_coeff_modulus(const std::vector<arith::Modulus>& m) { coeff_modulus_ = m; }
  void set_special_modulus_size(size_t s) { special_modulus_size_ = s; }
  void set_galois_elts(const std::vector<uint32_t>& g) { galois_elts_ = g; }
  scheme_type scheme() const { return scheme_; }
  size_t poly_modulus_degree() const { return poly_modulus_degree_; }
  const std::vector<arith::Modulus>& coeff_modulus() const { return coeff_modulus_; }
  std::vector<arith::Modulus>& coeff_modulus() { return coeff_modulus_; }
  size_t special_modulus_size() const { return special_modulus_size_; }
  const std::vector<uint32_t>& galois_elts() const { return galois_elts_; }

 private:
  scheme_type scheme_;
  size_t poly_modulus_degree_ = 0;
  std::vector<arith::Modulus> coeff_modulus_;
  size_t special_modulus_size_ = 1;
  std::vector<uint32_t> galois_elts_;
};

// Per-level data: chain index 0 is the key level (Q u P), 1 the full data chain Q, and each
// further index drops the last data prime (src/context.cu:133-159).
class ContextData {
 public:
  ContextData(size_t chain_index, std::vector<uint64_t> moduli, const EncryptionParameters* parms = nullptr)
      : chain_index_(chain_index), moduli_(std::move(moduli)), parms_(parms) {}
  size_t chain_index() const { return chain_index_; }
  // the context's EncryptionParameters (key level Q u P; the reference's per-level parms carry the
  // level's moduli, which moduli() gives here)
  const EncryptionParameters& parms() const {
    if (!parms_) throw std::logic_error("context data without parameters");
    return *parms_;
  }
  const std::vector<uint64_t>& moduli() const { return moduli_; }
  size_t coeff_modulus_size() const { return moduli_.size(); }
  const RnsTool& gpu_rns_tool() const { return *rns_tool_; }
  RnsTool& gpu_rns_tool_mutable() { return *rns_tool_; }
  bool has_rns_tool() const { return rns_tool_ != nullptr; }
  void set_rns_tool(std::unique_ptr<RnsTool> t) { rns_tool_ = std::move(t); }

 private:
  size_t chain_index_;
  std::vector<uint64_t> moduli_;
  const EncryptionParameters* parms_;
  std::unique_ptr<RnsTool> rns_tool_;
};

// owns the context's default stream when none is supplied (the reference runs every op on
// cudaStreamPerThread); destroyed last, after every buffer that frees on it
struct OwnedStream {
  hipStream_t s = nullptr;
  bool owned = false;
  OwnedStream() = default;
  OwnedStream(const OwnedStream&) = delete;
  OwnedStream& operator=(const OwnedStream&) = delete;
  ~OwnedStream() {
    if (owned && s) {
      (void)hipStreamSynchronize(s);
      DevicePool::instance().forget_stream(s);
      (void)hipStreamDestroy(s);
    }
  }
};

// Thread-local stream override: while a StreamScope lives, every PhantomContext operation
// issued by this thread runs on `s` instead of the context's stream (each stream has its own
// key-switch workspace).  Used to run independent chains of a bootstrap concurrently.
class StreamScope {
 public:
  explicit StreamScope(hipStream_t s) : prev_(current()) { current() = s; }
  ~StreamScope() { current() = prev_; }
  StreamScope(const StreamScope&) = delete;
  StreamScope& operator=(const StreamScope&) = delete;
  static hipStream_t& current() {
    static thread_local hipStream_t s = nullptr;
    return s;
  }
  // a further stream this thread may hand to a nested concurrent section (run_parallel)
  static hipStream_t& spare() {
    static thread_local hipStream_t s = nullptr;
    return s;
  }

 private:
  hipStream_t prev_;
};

// lane of the calling thread (PhantomContext::lane_stream / aux_stream); see LaneScope below
class LaneScope {
 public:
  static int& current() {
    static thread_local int lane = 0;
    return lane;
  }
};

// 1 when every modulus is below 2^60 (the grouped baby-step kernel's approximate reduction)
inline uint32_t below_2_60(const std::vector<uint64_t>& moduli) {
  for (uint64_t q : moduli)
    if (q >> 60) return 0;
  return 1;
}

class PhantomContext {
 public:
  // stream: where setup work and the façade's operations run; nullptr = a stream owned by the
  // context (never the null stream: see DeviceBuffer::allocate)
  explicit PhantomContext(const EncryptionParameters& params, hipStream_t stream = nullptr);
  PhantomContext(const PhantomContext&) = delete;
  PhantomContext& operator=(const PhantomContext&) = delete;

  const EncryptionParameters& params() const { return params_; }
  size_t poly_degree() const { return n_; }
  size_t size_Q() const { return size_Q_; }
  size_t size_P() const { return size_P_; }
  size_t size_QP() const { return size_Q_ + size_P_; }
  const std::vector<uint64_t>& key_moduli() const { return qp_; }

  const ContextData& get_context_data(size_t chain_index) const { return *data_.at(chain_index); }
  size_t total_parm_size() const { return data_.size(); }
  size_t get_first_index() const { return 1; }
  size_t get_next_index(size_t i) const { return i + 1 < data_.size() ? i + 1 : i; }
  size_t get_previous_index(size_t i) const { return i > 0 ? i - 1 : 0; }
  size_t coeff_mod_size() const { return qp_.size(); }

  // NTT tables and per-modulus device constants over the whole Q u P chain
  const phx::NttTables& gpu_rns_tables() const { return ntt_->get(); }
  phx::ModView mod_QP() const { return {ntt_->get().modulus, ntt_->get().barrett}; }
  hipStream_t stream() const {
    const hipStream_t o = StreamScope::current();
    return o ? o : stream_.s;
  }
  // further streams owned by the context, for work that runs beside stream().  Streams come
  // in lanes: lane 0 is stream() + its aux streams; a thread inside a LaneScope(k) issues to
  // lane k's main stream and aux streams, so independent evaluations (a batch of bootstraps)
  // run side by side without sharing a stream.
  static constexpr int kAuxStreams = 3;
  static constexpr int kLanes = 4;
  hipStream_t aux_stream(int i = 0) const { return aux_[LaneScope::current()][i].s; }
  hipStream_t lane_stream(int lane) const { return lane == 0 ? stream_.s : lane_main_[lane].s; }
  Workspace& workspace() const { return *ws_; }

  // NTT-domain permutation of Galois element `elt`: out[j] = in[perm[j]] applies X -> X^elt to an
  // NTT-form polynomial (PrecomputeAutoMapKernel, src/util.cu:941-958; the reference rebuilds it
  // on every call).  Built once per context, so every table lives on the context's device.
  const uint32_t* galois_perm(uint32_t elt) const;
  // the Galois element list keys are indexed by (the reference's key_galois_tool_->galois_elts(),
  // src/context.cu:231): the parameters' list, or when none was set PhantomGaloisTool::get_elts_all
  // (src/galois.cu:41-65): 2N - 1, then 5^(2^i) and 5^(-2^i) for i < log2(N) - 1
  std::vector<uint32_t> key_galois_elts() const;
  // its block inverse: source block sb (min(n, phx::kGaloisBlock) consecutive indices) is read by
  // output block galois_block_inv(elt)[sb] (n / min(n, kGaloisBlock) entries)
  const uint32_t* galois_block_inv(uint32_t elt) const { return galois_perm(elt) + n_; }
  // NTT(X^power) over the first L key moduli ([L][n]), cached per context
  const uint64_t* monomial_ntt(uint32_t power, size_t L) const;

  // Opt-in mean-unbiased moddowns at every level (RnsTool::set_unbias): off by default, where each
  // division is the reference's bit for bit.  PHX_UNBIASED_MODDOWN=1 in the environment turns it
  // on at construction.  Call between operations, not while work on other streams is in flight.
  void set_unbiased_moddown(bool on);
  bool unbiased_moddown() const { return unbiased_; }

 private:
  OwnedStream stream_;  // first members: destroyed after everything that frees on them
  OwnedStream aux_[kLanes][kAuxStreams];
  OwnedStream lane_main_[kLanes];  // [0] unused: lane 0 runs on stream_
  EncryptionParameters params_;
  size_t n_ = 0, size_Q_ = 0, size_P_ = 0;
  std::vector<uint64_t> qp_;
  std::unique_ptr<Workspace> ws_;  // declared before the tools that point into it
  std::unique_ptr<DeviceNttTables> ntt_;
  std::vector<std::unique_ptr<ContextData>> data_;
  mutable std::mutex cache_mu_;
  mutable std::map<uint32_t, DeviceBuffer<uint32_t>> perms_;
  mutable std::map<std::pair<uint32_t, size_t>, DeviceBuffer<uint64_t>> monomials_;
  DeviceBuffer<uint64_t> ones_ntt_;  // NTT(1, ..., 1) over Q, for the unbiased moddown
  bool unbiased_ = false;
};

// runs the calling thread on lane `lane` of `cc`: its main stream (StreamScope) and aux streams
class LaneGuard {
 public:
  LaneGuard(const PhantomContext& cc, int lane) : prev_(LaneScope::current()), scope_(cc.lane_stream(lane)) {
    LaneScope::current() = lane;
  }
  ~LaneGuard() { LaneScope::current() = prev_; }
  LaneGuard(const LaneGuard&) = delete;
  LaneGuard& operator=(const LaneGuard&) = delete;

 private:
  int prev_;
  StreamScope scope_;
};

}  // namespace phantom
