#include "context.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <thread>

#include "hip_check.h"
#include "numth.h"
#include "../csrc/ntt.h"
#include "../csrc/rns.h"

namespace phantom {

PhantomContext::PhantomContext(const EncryptionParameters& params, hipStream_t stream) : params_(params) {
  if (stream) {
    stream_.s = stream;
  } else {
    PHX_CHECK(hipStreamCreateWithFlags(&stream_.s, hipStreamNonBlocking));
    stream_.owned = true;
  }
  for (int l = 1; l < kLanes; ++l) {
    PHX_CHECK(hipStreamCreateWithFlags(&lane_main_[l].s, hipStreamNonBlocking));
    lane_main_[l].owned = true;
  }
  for (auto& lane : aux_) {
    for (auto& a : lane) {
      PHX_CHECK(hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking));
      a.owned = true;
    }
  }
  hipStream_t s = stream_.s;
  if (params.scheme() != scheme_type::ckks) throw std::invalid_argument("only CKKS is supported by this engine");
  const auto& mods = params.coeff_modulus();
  if (mods.size() < 2) throw std::invalid_argument("The coefficient modulus must be a vector of at least two primes");
  n_ = params.poly_modulus_degree();
  size_P_ = params.special_modulus_size();
  if (size_P_ >= mods.size()) throw std::invalid_argument("special modulus size too large");
  size_Q_ = mods.size() - size_P_;
  for (const auto& m : mods) qp_.push_back(m.value());

  // keep freed stream-ordered allocations cached (src/context.cu:127-131)
  int dev = 0;
  PHX_CHECK(hipGetDevice(&dev));
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t threshold = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold);
  }

  ws_ = std::make_unique<Workspace>();
  ntt_ = std::make_unique<DeviceNttTables>(n_, qp_, s);
  data_.push_back(std::make_unique<ContextData>(0, qp_, &params_));
  for (size_t c = 1; c <= size_Q_; ++c) {
    std::vector<uint64_t> ql(qp_.begin(), qp_.begin() + (size_Q_ - (c - 1)));
    data_.push_back(std::make_unique<ContextData>(c, ql, &params_));
  }
  // per-level RNS tools (host constant generation is O(L^2) per level; run levels in parallel)
  std::vector<std::unique_ptr<RnsTool>> tools(size_Q_ + 1);
  {
    std::vector<std::thread> th;
    const unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 8u);
    std::vector<std::exception_ptr> errs(nt);
    for (unsigned w = 0; w < nt; ++w)
      th.emplace_back([&, w] {
        try {
          for (size_t c = 1 + w; c <= size_Q_; c += nt)
            tools[c] = std::make_unique<RnsTool>(n_, qp_, size_P_, size_Q_ - (c - 1), s);
        } catch (...) {
          errs[w] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  }
  for (size_t c = 1; c <= size_Q_; ++c) {
    tools[c]->set_workspace(ws_.get());
    data_[c]->set_rns_tool(std::move(tools[c]));
  }
  PHX_CHECK(hipStreamSynchronize(s));
  if (const char* e = std::getenv("PHX_UNBIASED_MODDOWN"); e && e[0] == '1') set_unbiased_moddown(true);
}

void PhantomContext::set_unbiased_moddown(bool on) {
  hipStream_t s = stream_.s;
  if (on && !ones_ntt_.get()) {
    std::vector<uint64_t> h(size_Q_ * n_, 1);
    ones_ntt_.upload(h, s);
    PHX_CHECK(phx::ntt_forward(ntt_->get(), ones_ntt_.get(), ones_ntt_.get(),
                               phx::LimbMap::contiguous(static_cast<int>(size_Q_), 0), s));
  }
  for (size_t c = 1; c <= size_Q_; ++c) data_[c]->gpu_rns_tool_mutable().set_unbias(on ? ones_ntt_.get() : nullptr, s);
  PHX_CHECK(hipStreamSynchronize(s));
  unbiased_ = on;
}

std::vector<uint32_t> PhantomContext::key_galois_elts() const {
  if (!params_.galois_elts().empty()) return params_.galois_elts();
  const uint64_t m = 2 * static_cast<uint64_t>(n_);
  std::vector<uint32_t> elts{static_cast<uint32_t>(m - 1)};
  uint64_t pos = 5, neg = arith::inv_mod(5, m);
  for (size_t i = 0; i + 1 < static_cast<size_t>(arith::log2_exact(n_)); ++i) {
    elts.push_back(static_cast<uint32_t>(pos));
    pos = pos * pos & (m - 1);
    elts.push_back(static_cast<uint32_t>(neg));
    neg = neg * neg & (m - 1);
  }
  return elts;
}

const uint32_t* PhantomContext::galois_perm(uint32_t elt) const {
  std::lock_guard<std::mutex> lk(cache_mu_);
  auto it = perms_.find(elt);
  if (it != perms_.end()) return it->second.get();
  if (!(elt & 1) || elt >= 2 * n_) throw std::invalid_argument("invalid Galois element");
  const int logn = arith::log2_exact(n_);
  std::vector<uint32_t> perm(n_);  // [n] permutation, then [n / bsz] block inverse
  for (uint32_t j = 0; j < n_; ++j) {
    const uint64_t idx = ((2ull * j + 1) * elt) % (2ull * n_);
    perm[arith::reverse_bits(j, logn)] = arith::reverse_bits(static_cast<uint32_t>(idx >> 1), logn);
  }
  // + the block inverse (galois_block_inv): output block ob reads source block perm[ob bsz] / bsz
  const uint32_t bsz = static_cast<uint32_t>(std::min<size_t>(n_, phx::kGaloisBlock)), nb = static_cast<uint32_t>(n_) / bsz;
  perm.resize(n_ + nb);
  for (uint32_t ob = 0; ob < nb; ++ob) perm[n_ + perm[static_cast<size_t>(ob) * bsz] / bsz] = ob;
  DeviceBuffer<uint32_t> d;
  d.upload(perm, stream_.s);
  return perms_.emplace(elt, std::move(d)).first->second.get();
}

const uint64_t* PhantomContext::monomial_ntt(uint32_t power, size_t L) const {
  const uint32_t pr = power % static_cast<uint32_t>(2 * n_);
  std::lock_guard<std::mutex> lk(cache_mu_);
  auto key = std::make_pair(pr, L);
  auto it = monomials_.find(key);
  if (it != monomials_.end()) return it->second.get();
  if (L > qp_.size()) throw std::invalid_argument("too many limbs");
  std::vector<uint64_t> h(L * n_, 0);
  for (size_t l = 0; l < L; ++l) h[l * n_ + pr % n_] = pr < n_ ? 1 : qp_[l] - 1;
  DeviceBuffer<uint64_t> d;
  d.upload(h, stream_.s);
  PHX_CHECK(phx::ntt_forward(ntt_->get(), d.get(), d.get(), phx::LimbMap::contiguous(static_cast<int>(L), 0), stream_.s));
  PHX_CHECK(hipStreamSynchronize(stream_.s));
  return monomials_.emplace(key, std::move(d)).first->second.get();
}

}  // namespace phantom
