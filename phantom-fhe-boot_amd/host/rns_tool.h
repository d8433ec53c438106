// rns_tool.h — per-level RNS constants and the key-switch / rescale drivers: the CKKS part
// of the reference's DRNSTool (include/rns.cuh:16-387, constants at src/rns.cu:11-190,
// modup src/rns_bconv.cu:530-628, moddown_from_NTT :791-843, divide_and_round_q_last_ntt
// src/rns.cu:1160-1184).  BFV/BGV-only members (BEHZ/HPS) are out of scope.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "../csrc/ntt.h"
#include "../csrc/rns.h"
#include "buffer.h"

namespace phantom {

// Fast base converter constants (the reference's BaseConverter, include/host/rns.h:135-199)
struct DeviceBaseConverter {
  std::vector<uint64_t> ibase, obase;
  DeviceBuffer<uint64_t> d_ibase, d_obase, d_obase_barrett;
  DeviceBuffer<uint64_t> d_qhat_inv, d_qhat_inv_shoup;  // [ibase] (qHat_i^-1 mod q_i)
  std::vector<uint64_t> qhat_inv_host;
  DeviceBuffer<uint64_t> d_qhat_mod_p;                  // [ibase][obase]
  // matrix-core form of the conversion (rns.h bconv_mfma_tables), empty when the shape has none
  DeviceBuffer<uint8_t> d_mfma_frag;
  DeviceBuffer<uint64_t> d_mfma_rows;
  void init(const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, hipStream_t s);
  phx::BconvArgs args(const uint64_t* in, uint64_t* out, bool prescale) const;
};

class RnsTool {
 public:
  // moduli_QP: the full key-level chain (size_Q data primes then size_P special primes);
  // size_Ql: number of data primes at this level (size_Q at chain index 1).
  RnsTool(size_t n, const std::vector<uint64_t>& moduli_QP, size_t size_P, size_t size_Ql, hipStream_t s);

  size_t n() const { return n_; }
  size_t size_Q() const { return size_Q_; }
  size_t size_P() const { return size_P_; }
  size_t size_QP() const { return size_Q_ + size_P_; }
  size_t size_Ql() const { return base_Ql_.size(); }
  size_t beta() const { return converters_.size(); }
  const std::vector<uint64_t>& base_Ql() const { return base_Ql_; }

  // modup (src/rns_bconv.cu:530-628): c2 [size_Ql][n] NTT form -> t_mod_up [beta][size_QlP][n];
  // `count` independent ones per launch: c2 of job k at c2 + k c2_stride, its digits at
  // t_mod_up + k beta size_QlP n
  void modup(uint64_t* t_mod_up, const uint64_t* c2, const phx::NttTables& ntt, hipStream_t s, size_t count = 1,
             size_t c2_stride = 0) const;
  // moddown_from_NTT (src/rns_bconv.cu:791-843) fused with add_to_ct_kernel, for `polys`
  // polynomials at once: cx is [polys][size_QlP][n] NTT form (its P limbs are clobbered);
  // ct [polys][size_Ql][n] (+)= moddown(cx).  With tmu/evk (a key switch's t_mod_up and key
  // digits, polys = 2): cx is not read, only its P limbs used as scratch; the inner product
  // sum_d tmu[d] evk[d][p] is formed in the INTT(P)'s prologue (its P limbs, ntt.h ntt_inverse_ks)
  // and in the finish's epilogue (its Ql limbs, NttEpilogue::ks_beta).
  void moddown_add(uint64_t* ct, uint64_t* cx, bool accumulate, const phx::NttTables& ntt, hipStream_t s,
                   size_t polys = 1, const uint64_t* tmu = nullptr, const uint64_t* const* evk = nullptr) const;
  // moddown of an extended-basis polynomial fused with the modup of its result (giant-step
  // rotations): c1 [size_QlP][n] NTT form holding P x (a polynomial over Ql) -> t_mod_up
  // [beta][size_QlP][n] = modup(round(c1 / P)).  The subtraction happens in the coefficient
  // domain: one INTT over Ql u P and one NTT over every digit replace moddown's INTT(P) + NTT(Ql)
  // and modup's INTT(Ql) + NTT(digits).  c1 is clobbered.
  // `count` independent ones in one launch per stage (the giant steps of a linear-transform
  // level): c1 of job i at c1 + i c1_stride, its digits at t_mod_up + i beta QlP n
  void moddown_modup(uint64_t* t_mod_up, uint64_t* c1, const phx::NttTables& ntt, hipStream_t s, size_t count = 1,
                     size_t c1_stride = 0) const;
  // moddown fused with the following rescale: cx [polys][size_QlP][n] NTT form holds P x (a
  // ciphertext at this level, scale S); out [polys][size_Ql - 1][n] = round(cx / (P q_last)),
  // the ciphertext rescaled to the next level (scale S / q_last).  One INTT over the 1 + size_P
  // dropped limbs, one base conversion, one NTT and one finish instead of a moddown (INTT P,
  // NTT Ql) followed by a rescale (INTT 1, NTT Ql - 1).  cx's dropped limbs are clobbered.
  // With `ks` (polys = 2, a key switch's t_mod_up / key digits / P-scaled addend): cx is not read,
  // only its dropped limbs used as scratch; the inner product's dropped limbs are formed in the
  // INTT's prologue (ntt_inverse_ks) and its first size_Ql - 1 limbs in the finish's epilogue.
  void moddown_rescale(uint64_t* out, uint64_t* cx, const phx::NttTables& ntt, hipStream_t s,
                       size_t polys = 1, const phx::NttEpilogue* ks = nullptr) const;
  // divide_and_round_q_last_ntt (src/rns.cu:1160-1184): in [polys][size_Ql][n] -> out
  // [polys][size_Ql-1][n], NTT form.  `in` is not modified.
  void rescale_ntt(const uint64_t* in, uint64_t* out, size_t polys, const phx::NttTables& ntt,
                   hipStream_t s) const;
  // the same for `cts` two-polynomial ciphertexts (in contiguous [cts][2][size_Ql][n]) whose
  // results go to their own buffers outs[k] ([2][size_Ql-1][n]); cts <= phx::kMaxKsProds
  void rescale_ntt_to(const uint64_t* in, uint64_t* const* outs, size_t cts, const phx::NttTables& ntt,
                      hipStream_t s) const;

  // Opt-in mean-unbiased moddown (PhantomContext::set_unbiased_moddown; DESIGN.md §3 "Where the
  // precision goes").  A division by D = P (moddown) or P q_last (moddown + rescale) through the
  // fast conversion of ibase limbs returns floor(c / D) - u with u the conversion's overflow, a
  // mean bias of -1/2 - (ibase - 1) / 2 per coefficient (src/rns_bconv.cu:791-843 has no overflow
  // correction).  With `ones_ntt` = NTT(1, ..., 1) over Q ([size_Q][n]), every such division adds
  // floor(ibase / 2) to each output coefficient: zero mean for an even ibase, +-1/2 for an odd
  // one (the plain rescale's own).  nullptr = off: the reference's arithmetic, bit for bit.
  void set_unbias(const uint64_t* ones_ntt, hipStream_t s);
  bool unbiased() const { return ones_ntt_ != nullptr; }

  // scratch space shared by the drivers (owned by the PhantomContext)
  void set_workspace(Workspace* ws) { ws_ = ws; }
  Workspace& workspace() const { return *ws_; }

  // device views over Ql
  phx::ModView mod_Ql() const { return {d_Ql_.get(), d_Ql_barrett_.get()}; }
  // the extended basis Ql u P in buffer order (limb i < size_Ql: q_i, then p_0 ..)
  phx::ModView mod_QlP() const { return {d_QlP_.get(), d_QlP_barrett_.get()}; }
  const uint64_t* bigP_mod_q() const { return d_bigP_mod_q_.get(); }
  const uint64_t* bigP_mod_q_shoup() const { return d_bigP_mod_q_shoup_.get(); }

 private:
  size_t n_, size_Q_, size_P_;
  Workspace* ws_ = nullptr;
  std::vector<uint64_t> base_Ql_, base_P_;
  DeviceBuffer<uint64_t> d_Ql_, d_Ql_barrett_, d_QlP_, d_QlP_barrett_;
  // key switching
  DeviceBuffer<uint64_t> d_partQlHatInv_, d_partQlHatInv_shoup_;
  DeviceBuffer<uint64_t> d_mm_scale_, d_mm_scale_shoup_;  // moddown_modup's INTT scale over Ql u P
  // the base conversion can run as the forward NTT's column-pass prologue (ntt.h BconvPrologue):
  // 2-D transform sizes and at most 15 input limbs; opt-in (PHX_FUSED_BCONV=1), see rns_tool.cpp
  bool fused_bconv_ok(size_t ibase) const;
  // `count` batches: t_cks [count][Ql][n] -> t_mod_up [count][beta][QlP][n]
  void digit_bconv(const uint64_t* t_cks, uint64_t* t_mod_up, hipStream_t s, size_t count = 1) const;
  std::vector<DeviceBaseConverter> converters_;  // digit beta: part -> complement of QlP
  std::vector<size_t> digit_start_, digit_size_;
  DeviceBaseConverter p_to_ql_;
  // fused moddown + rescale: {q_last} u P -> Q_{l-1}, and (P q_last)^-1 mod q_j
  DeviceBaseConverter pq_to_ql1_;
  DeviceBuffer<uint64_t> d_PQinv_, d_PQinv_shoup_;
  DeviceBuffer<uint64_t> d_bigP_mod_q_, d_bigP_mod_q_shoup_, d_bigPInv_mod_q_, d_bigPInv_mod_q_shoup_;
  // rescale
  DeviceBuffer<uint64_t> d_inv_qlast_, d_inv_qlast_shoup_;
  // unbiased moddown (set_unbias): k mod q_l and its Shoup quotient over Ql, for the moddown
  // (k = floor(size_P / 2)) and the moddown + rescale (k = floor((size_P + 1) / 2))
  const uint64_t* ones_ntt_ = nullptr;
  uint64_t k_md_ = 0, k_mdr_ = 0;
  DeviceBuffer<uint64_t> d_k_md_, d_k_md_shoup_, d_k_mdr_, d_k_mdr_shoup_;
  // out [polys][limbs][n] at poly stride `stride`, NTT form: += k NTT(1, ..., 1)
  void unbias_ntt(uint64_t* out, size_t polys, size_t limbs, size_t stride, bool rescale, hipStream_t s) const;
};

}  // namespace phantom
