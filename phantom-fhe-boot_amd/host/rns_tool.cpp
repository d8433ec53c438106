#include "rns_tool.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>

#include "numth.h"
#include "../csrc/ckks.h"

#ifndef PHX_DIAG_CENTRED
#define PHX_DIAG_CENTRED 0
#endif
#if PHX_DIAG_CENTRED
#include <cstdio>
#endif

namespace phantom {

using namespace phantom::arith;

#if PHX_DIAG_CENTRED
// DIAGNOSTIC BUILD ONLY (-DPHX_DIAG_CENTRED=1, tools/diag_centred.sh): never
// part of the product, which divides exactly as the reference does (floor division by a
// non-centred remainder, src/rns.cu:1160-1184, and the fast conversion without overflow
// correction, src/rns_bconv.cu:791-843).  Here every division of an NTT-form input by D (rescale:
// D = q_last; moddown: D = P; moddown + rescale: D = q_last P) is made mean-unbiased by adding H to
// every coefficient first: floor((c + H) / D) - u with u the conversion's overflow, E[u] =
// (ibase - 1) / 2, so H = (ibase / 2) D for an even input base and ((ibase - 1) / 2) D + floor(D/2)
// for an odd one (the rescale's single limb: floor(q_last / 2), plain centred rounding).  In NTT form,
// limb l += (H mod m_l) NTT_l(1, 1, ..., 1).  The fused key-switch forms never materialise their
// input, so this build needs PHX_KS_EPI=0.  PHX_DIAG_CENTRED=2: the rescales only; =3: the moddowns
// (and the fused moddown + rescale) only.
constexpr bool kDiagRescale = PHX_DIAG_CENTRED != 3, kDiagModdown = PHX_DIAG_CENTRED != 2;
namespace {
void diag_unbias(uint64_t* x, size_t polys, size_t poly_stride, const std::vector<uint64_t>& mods, int split,
                 size_t size_Q, const std::vector<uint64_t>& divisor, size_t ibase, size_t n, const phx::NttTables& ntt,
                 hipStream_t s) {
  const size_t L = mods.size();
  std::vector<uint64_t> c(L), cs(L);
  for (size_t l = 0; l < L; ++l) {
    const uint64_t m = mods[l];
    uint64_t d = 1 % m;
    for (uint64_t q : divisor) d = mul_mod(d, q % m, m);
    uint64_t h = mul_mod((ibase / 2) % m, d, m);
    if (ibase % 2) h = (h + mul_mod((d + m - 1) % m, (m + 1) / 2, m)) % m;  // + floor(D / 2) = (D - 1) / 2
    c[l] = h;
    cs[l] = shoup(h, m);
  }
  DeviceBuffer<uint64_t> ones(L * n, s), dq(L, s), dc(L, s), dcs(L, s);
  ones.upload(std::vector<uint64_t>(L * n, 1), s);
  dq.upload(mods, s);
  dc.upload(c, s);
  dcs.upload(cs, s);
  phx::LimbMap map;
  map.num_limbs = (int)L;
  map.split = split;
  map.first_a = 0;
  map.first_b = (int)size_Q;
  hip_ok(phx::ntt_forward(ntt, ones.get(), ones.get(), map, s), "diag NTT(1)");
  for (size_t p = 0; p < polys; ++p)
    hip_ok(phx::mul_scalar_add(ones.get(), dc.get(), dcs.get(), x + p * poly_stride, x + p * poly_stride, dq.get(), n, L, s),
           "diag unbias");
  PHX_CHECK(hipStreamSynchronize(s));
  static bool said = false;
  if (!said) {
    said = true;
    std::fprintf(stderr, "[diag] PHX_DIAG_CENTRED build: divisions made mean-unbiased (not the product)\n");
  }
}
}  // namespace
#endif

void DeviceBaseConverter::init(const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, hipStream_t s) {
  ibase = in;
  obase = out;
  const size_t I = in.size(), O = out.size();
  std::vector<uint64_t> qinv(I), qinvs(I), qhat(I * O), ob(2 * O);
  for (size_t i = 0; i < I; ++i) {
    uint64_t prod = 1 % in[i];
    for (size_t k = 0; k < I; ++k)
      if (k != i) prod = mul_mod(prod, in[k] % in[i], in[i]);
    qinv[i] = inv_mod(prod, in[i]);
    qinvs[i] = shoup(qinv[i], in[i]);
    for (size_t j = 0; j < O; ++j) {
      uint64_t pr = 1 % out[j];
      for (size_t k = 0; k < I; ++k)
        if (k != i) pr = mul_mod(pr, in[k] % out[j], out[j]);
      qhat[i * O + j] = pr;
    }
  }
  for (size_t j = 0; j < O; ++j) barrett_ratio(out[j], &ob[2 * j]);
  d_ibase.upload(in, s);
  d_obase.upload(out, s);
  d_obase_barrett.upload(ob, s);
  qhat_inv_host = qinv;
  d_qhat_inv.upload(qinv, s);
  d_qhat_inv_shoup.upload(qinvs, s);
  d_qhat_mod_p.upload(qhat, s);
  if (I <= (size_t)phx::kBconvMfmaMaxIbase && O <= (size_t)phx::kBconvMfmaMaxObase) {
    std::vector<uint8_t> frag(phx::bconv_mfma_frag_bytes((int)I, (int)O));
    std::vector<uint64_t> rows(2 * 16 * ((O + 15) / 16));
    phx::bconv_mfma_tables(qhat.data(), out.data(), (int)I, (int)O, frag.data(), rows.data());
    d_mfma_frag.upload(frag, s);
    d_mfma_rows.upload(rows, s);
  }
}

phx::BconvArgs DeviceBaseConverter::args(const uint64_t* in, uint64_t* out, bool prescale) const {
  phx::BconvArgs a;
  a.in = in;
  a.out = out;
  a.ibase = d_ibase.get();
  a.qhat_inv = prescale ? d_qhat_inv.get() : nullptr;
  a.qhat_inv_shoup = prescale ? d_qhat_inv_shoup.get() : nullptr;
  a.qhat_mod_p = d_qhat_mod_p.get();
  a.obase = d_obase.get();
  a.obase_barrett = d_obase_barrett.get();
  a.ibase_size = static_cast<int>(ibase.size());
  a.obase_size = static_cast<int>(obase.size());
  a.mfma_frag = d_mfma_frag.get();
  a.mfma_rows = d_mfma_rows.get();
  return a;
}

RnsTool::RnsTool(size_t n, const std::vector<uint64_t>& qp, size_t size_P, size_t size_Ql, hipStream_t s)
    : n_(n), size_Q_(qp.size() - size_P), size_P_(size_P) {
  if (size_Ql == 0 || size_Ql > size_Q_) throw std::invalid_argument("invalid level");
  base_Ql_.assign(qp.begin(), qp.begin() + size_Ql);
  base_P_.assign(qp.begin() + size_Q_, qp.end());
  std::vector<uint64_t> bar(2 * size_Ql);
  for (size_t i = 0; i < size_Ql; ++i) barrett_ratio(base_Ql_[i], &bar[2 * i]);
  d_Ql_.upload(base_Ql_, s);
  d_Ql_barrett_.upload(bar, s);

  // rescale constants: q_last^-1 mod q_i (src/rns.cu:64-82)
  if (size_Ql > 1) {
    const uint64_t ql = base_Ql_.back();
    std::vector<uint64_t> inv(size_Ql - 1), invs(size_Ql - 1);
    for (size_t i = 0; i + 1 < size_Ql; ++i) {
      inv[i] = inv_mod(ql % base_Ql_[i], base_Ql_[i]);
      invs[i] = shoup(inv[i], base_Ql_[i]);
    }
    d_inv_qlast_.upload(inv, s);
    d_inv_qlast_shoup_.upload(invs, s);
  }

  if (size_P == 0) return;
  // hybrid key switching constants (src/rns.cu:97-187)
  const size_t alpha = size_P;
  std::vector<uint64_t> pm(size_Ql), pms(size_Ql), pim(size_Ql), pims(size_Ql);
  for (size_t i = 0; i < size_Ql; ++i) {
    const uint64_t q = base_Ql_[i];
    uint64_t P = 1 % q;
    for (uint64_t p : base_P_) P = mul_mod(P, p % q, q);
    pm[i] = P;
    pms[i] = shoup(P, q);
    pim[i] = inv_mod(P, q);
    pims[i] = shoup(pim[i], q);
  }
  d_bigP_mod_q_.upload(pm, s);
  d_bigP_mod_q_shoup_.upload(pms, s);
  d_bigPInv_mod_q_.upload(pim, s);
  d_bigPInv_mod_q_shoup_.upload(pims, s);

  std::vector<uint64_t> qlp(base_Ql_);
  qlp.insert(qlp.end(), base_P_.begin(), base_P_.end());
  std::vector<uint64_t> qlpb(2 * qlp.size());
  for (size_t i = 0; i < qlp.size(); ++i) barrett_ratio(qlp[i], &qlpb[2 * i]);
  d_QlP_.upload(qlp, s);
  d_QlP_barrett_.upload(qlpb, s);
  const size_t beta = static_cast<size_t>(std::ceil(static_cast<double>(size_Ql) / static_cast<double>(alpha)));
  std::vector<uint64_t> hatinv(size_Ql), hatinvs(size_Ql);
  converters_.resize(beta);
  for (size_t b = 0; b < beta; ++b) {
    const size_t start = alpha * b;
    const size_t part = b == beta - 1 ? size_Ql - alpha * (beta - 1) : alpha;
    std::vector<uint64_t> pin(qlp.begin() + start, qlp.begin() + start + part), compl_;
    for (size_t j = 0; j < qlp.size(); ++j)
      if (j < start || j >= start + part) compl_.push_back(qlp[j]);
    converters_[b].init(pin, compl_, s);
    digit_start_.push_back(start);
    digit_size_.push_back(part);
    // partQlHatInv_mod_Ql_concat: the digit-local qHat^-1 of every Ql prime
    for (size_t i = 0; i < part; ++i) {
      uint64_t prod = 1 % pin[i];
      for (size_t k = 0; k < part; ++k)
        if (k != i) prod = mul_mod(prod, pin[k] % pin[i], pin[i]);
      hatinv[start + i] = inv_mod(prod, pin[i]);
      hatinvs[start + i] = shoup(hatinv[start + i], pin[i]);
    }
  }
  d_partQlHatInv_.upload(hatinv, s);
  d_partQlHatInv_shoup_.upload(hatinvs, s);
  p_to_ql_.init(base_P_, base_Ql_, s);
  {
    // moddown_modup's INTT over Ql u P: 1 on Ql (the finish reads those limbs as they are),
    // qHat_p^-1 on P (the P -> Ql conversion's prescale)
    std::vector<uint64_t> sc(base_Ql_.size() + size_P_), scs(sc.size());
    for (size_t i = 0; i < base_Ql_.size(); ++i) {
      sc[i] = 1;
      scs[i] = shoup(1, base_Ql_[i]);
    }
    for (size_t i = 0; i < size_P_; ++i) {
      sc[base_Ql_.size() + i] = p_to_ql_.qhat_inv_host[i];
      scs[base_Ql_.size() + i] = shoup(sc[base_Ql_.size() + i], base_P_[i]);
    }
    d_mm_scale_.upload(sc, s);
    d_mm_scale_shoup_.upload(scs, s);
  }
  if (size_Ql >= 2) {
    std::vector<uint64_t> ib{base_Ql_.back()};
    ib.insert(ib.end(), base_P_.begin(), base_P_.end());
    const std::vector<uint64_t> ob(base_Ql_.begin(), base_Ql_.end() - 1);
    pq_to_ql1_.init(ib, ob, s);
    std::vector<uint64_t> inv(ob.size()), invs(ob.size());
    for (size_t j = 0; j < ob.size(); ++j) {
      const uint64_t q = ob[j];
      inv[j] = mul_mod(pim[j], inv_mod(base_Ql_.back() % q, q), q);
      invs[j] = shoup(inv[j], q);
    }
    d_PQinv_.upload(inv, s);
    d_PQinv_shoup_.upload(invs, s);
  }
}

// Off by default: measured slower than the separate conversion + NTT on MI355X (C3 relinearize
// 0.416 vs 0.377 ms, bootstrap 32.4 vs 31.2 ms; profiles/r02/fused_bconv_ntt.txt): computed per
// output element, the conversion re-splits and re-reads its 15 inputs for every output limb
// (the separate kernel shares them across 5), and the column pass at 210 VGPRs runs 2 waves per
// SIMD.  PHX_FUSED_BCONV=1 selects it (bit-exact either way).
bool RnsTool::fused_bconv_ok(size_t ibase) const {
  static const bool on = [] {
    const char* e = std::getenv("PHX_FUSED_BCONV");
    return e && e[0] == '1';
  }();
  return on && n_ >= 1024 && ibase >= 1 && ibase <= 15;
}

// every digit's conversion to its complement of QlP (digit b: t_cks limbs [b alpha, b alpha + part)
// -> t_mod_up[b], skipping the digit's own limbs); the full digits in one launch (one converter
// per blockIdx.z), a short last digit apart
void RnsTool::digit_bconv(const uint64_t* t_cks, uint64_t* t_mod_up, hipStream_t s, size_t count) const {
  const size_t size_Ql = base_Ql_.size(), size_QlP = size_Ql + size_P_, alpha = size_P_, beta = converters_.size();
  const size_t full = digit_size_.back() == alpha ? beta : beta - 1;
  for (size_t b0 = 0; b0 < full; b0 += phx::BconvArgs::kMaxJobs) {
    const size_t cnt = std::min<size_t>(phx::BconvArgs::kMaxJobs, full - b0);
    phx::BconvArgs a = converters_[b0].args(t_cks + digit_start_[b0] * n_, t_mod_up + b0 * size_QlP * n_, false);
    a.skip_at = (int)digit_start_[b0];
    a.skip_len = (int)alpha;
    a.jobs = (int)cnt;
    a.polys = (int)(cnt * count);
    a.in_stride = alpha * n_;
    a.out_stride = size_QlP * n_;
    a.skip_step = (int)alpha;
    if (count > 1) {
      a.period = (int)cnt;
      a.in_outer = size_Ql * n_;
      a.out_outer = beta * size_QlP * n_;
    }
    for (size_t d = 0; d < cnt; ++d) {
      const DeviceBaseConverter& c = converters_[b0 + d];
      a.job_qhat_mod_p[d] = c.d_qhat_mod_p.get();
      a.job_obase[d] = c.d_obase.get();
      a.job_obase_barrett[d] = c.d_obase_barrett.get();
      a.job_mfma_frag[d] = c.d_mfma_frag.get();
      a.job_mfma_rows[d] = c.d_mfma_rows.get();
    }
    hip_ok(phx::bconv(a, n_, s), "digit bconv");
  }
  if (full < beta) {
    phx::BconvArgs a = converters_[full].args(t_cks + digit_start_[full] * n_, t_mod_up + full * size_QlP * n_, false);
    a.skip_at = (int)digit_start_[full];
    a.skip_len = (int)digit_size_[full];
    a.polys = (int)count;
    a.in_stride = size_Ql * n_;
    a.out_stride = beta * size_QlP * n_;
    hip_ok(phx::bconv(a, n_, s), "digit bconv (short digit)");
  }
}

void RnsTool::modup(uint64_t* t_mod_up, const uint64_t* c2, const phx::NttTables& ntt, hipStream_t s, size_t count,
                    size_t c2_stride) const {
  const size_t size_Ql = base_Ql_.size(), size_QlP = size_Ql + size_P_, alpha = size_P_;
  const size_t beta = converters_.size(), dig = beta * size_QlP * n_;  // one key switch's digits
  if (count < 1 || (count > 1 && c2_stride < size_Ql * n_)) throw std::invalid_argument("modup: bad batch");
  const int nc = static_cast<int>(count);
  uint64_t* t_cks = ws_->get(s, Workspace::kModupInv, count * size_Ql * n_);
  // INTT(c2) * partQlHatInv (nwt_2d_radix8_backward_scale)
  // and the digits' own limbs (modup_copy_partQl_kernel) stored by the INTT's first pass, which
  // reads c2 anyway; `count` key switches' c2 in one launch
  const phx::LimbMap im = phx::LimbMap::contiguous((int)size_Ql, 0).batched(nc, c2_stride, size_Ql * n_);
  if (n_ >= 1024) {
    phx::NttCopy cp;
    cp.out = t_mod_up;
    cp.digit_stride = size_QlP * n_;
    cp.alpha = (int)alpha;
    cp.poly_stride = dig;
    hip_ok(phx::ntt_inverse_copy(ntt, c2, t_cks, im, d_partQlHatInv_.get(), d_partQlHatInv_shoup_.get(), cp, s),
           "modup INTT + copy");
  } else {
    hip_ok(phx::ntt_inverse(ntt, c2, t_cks, im, d_partQlHatInv_.get(), d_partQlHatInv_shoup_.get(), s), "modup INTT");
    for (size_t k = 0; k < count; ++k)
      hip_ok(phx::modup_copy_digits(c2 + k * c2_stride, t_mod_up + k * dig, n_, size_Ql, size_QlP, alpha, s),
             "modup copy");
  }
  // per digit: the complement limbs = NTT(bconv(digit)), every limb but the digit's own
  // (include_special_mod_exclude_range); the full digits of every key switch in one launch
  // (digit b skips [b alpha, (b + 1) alpha)), a short last digit apart.  PHX_FUSED_BCONV=1: the
  // conversion is the column pass's prologue (ntt.h BconvPrologue), one key switch per launch.
  const size_t full = digit_size_.back() == alpha ? beta : beta - 1;
  const bool fused = fused_bconv_ok(alpha);
  if (!fused) digit_bconv(t_cks, t_mod_up, s, count);
  auto digit_map = [&](size_t b0) {
    phx::LimbMap m;
    m.num_limbs = (int)size_QlP;
    m.split = (int)size_Ql;
    m.first_a = 0;
    m.first_b = (int)size_Q_;
    m.skip_begin = (int)digit_start_[b0];
    m.skip_end = (int)(digit_start_[b0] + digit_size_[b0]);
    m.skip_step = (int)alpha;
    return m;
  };
  if (fused) {
    for (size_t k = 0; k < count; ++k) {
      auto run = [&](size_t b0, size_t cnt) {
        phx::BconvPrologue bcv;
        bcv.in = t_cks + k * size_Ql * n_ + digit_start_[b0] * n_;
        bcv.in_stride = alpha * n_;
        bcv.ob = (int)(size_QlP - digit_size_[b0]);
        for (size_t i = 0; i < cnt; ++i) {
          bcv.mat[i] = converters_[b0 + i].d_qhat_mod_p.get();
          bcv.ib[i] = (int)digit_size_[b0 + i];
        }
        uint64_t* dst = t_mod_up + k * dig + b0 * size_QlP * n_;
        hip_ok(phx::ntt_forward_bconv(ntt, dst, digit_map(b0).batched((int)cnt), bcv, phx::NttEpilogue{}, s),
               "modup bconv + NTT");
      };
      for (size_t b0 = 0; b0 < full; b0 += phx::kMaxBconvPolys) run(b0, std::min<size_t>(phx::kMaxBconvPolys, full - b0));
      if (full < beta) run(full, 1);
    }
    return;
  }
  if (full > 0)
    hip_ok(phx::ntt_forward(ntt, t_mod_up, t_mod_up,
                            digit_map(0).grouped(nc * (int)full, (int)full, size_QlP * n_, dig), s),
           "modup NTT");
  if (full < beta) {
    uint64_t* dst = t_mod_up + full * size_QlP * n_;
    hip_ok(phx::ntt_forward(ntt, dst, dst, digit_map(full).grouped(nc, 1, 0, dig), s), "modup NTT (short digit)");
  }
}

void RnsTool::moddown_add(uint64_t* ct, uint64_t* cx, bool accumulate, const phx::NttTables& ntt, hipStream_t s,
                          size_t polys, const uint64_t* tmu, const uint64_t* const* evk) const {
  // every stage runs once over all `polys` polynomials (ct [polys][Ql][n], cx [polys][QlP][n])
  const size_t size_Ql = base_Ql_.size(), size_QlP = size_Ql + size_P_;
#if PHX_DIAG_CENTRED
  if (tmu) throw std::runtime_error("PHX_DIAG_CENTRED build: run with PHX_KS_EPI=0");
  if (kDiagModdown) {
    std::vector<uint64_t> mods(base_Ql_);
    mods.insert(mods.end(), base_P_.begin(), base_P_.end());
    diag_unbias(cx, polys, size_QlP * n_, mods, (int)size_Ql, size_Q_, base_P_, size_P_, n_, ntt, s);
  }
#endif
  const int np = static_cast<int>(polys);
  uint64_t* cp = cx + size_Ql * n_;
  phx::LimbMap pm;
  pm.num_limbs = (int)size_P_;
  pm.split = 0;
  pm.first_a = 0;
  pm.first_b = (int)size_Q_;
  const bool fused = fused_bconv_ok(size_P_) && polys <= (size_t)phx::kMaxBconvPolys;
  phx::NttEpilogue ksf;  // the key-switch form: prologue of INTT(P), epilogue of the finish
  if (tmu) {
    if (beta() > (size_t)phx::kMaxKsBeta) throw std::invalid_argument("moddown_add: too many key-switch digits");
    ksf.ks_beta = (int)beta();
    ksf.tmu = tmu;
    ksf.tmu_stride = size_QlP * n_;
    ksf.evk = evk;
    ksf.evk_poly_stride = size_QP() * n_;
  }
  // the INTT also applies the converter's qHat^-1 (the conversion's prescale, otherwise redone
  // by every output group of the conversion); with tmu its input is the inner product's P limbs
  const phx::LimbMap pmb = pm.batched(np, size_QlP * n_, size_QlP * n_);
  if (tmu) {
    phx::NttEpilogue pro = ksf;
    pro.tmu_limb0 = size_Ql;
    hip_ok(phx::ntt_inverse_ks(ntt, cp, pmb, p_to_ql_.d_qhat_inv.get(), p_to_ql_.d_qhat_inv_shoup.get(), pro, s),
           "moddown inner product + INTT(P)");
  } else {
    hip_ok(phx::ntt_inverse(ntt, cp, cp, pmb, p_to_ql_.d_qhat_inv.get(), p_to_ql_.d_qhat_inv_shoup.get(), s),
           "moddown INTT(P)");
  }
  uint64_t* delta = ws_->get(s, Workspace::kModdownDelta, polys * size_Ql * n_);
  // NTT(delta) with the finish (cx - delta) P^-1 (+ ct) as its epilogue
  phx::NttEpilogue epi = ksf;
  epi.c = cx;
  epi.c_stride = size_QlP * n_;
  epi.out = ct;
  epi.out_stride = size_Ql * n_;
  epi.w = d_bigPInv_mod_q_.get();
  epi.ws = d_bigPInv_mod_q_shoup_.get();
  epi.accumulate = accumulate;
  const phx::LimbMap dm = phx::LimbMap::contiguous((int)size_Ql, 0).batched(np);
  if (fused) {
    phx::BconvPrologue bcv;
    bcv.in = cp;
    bcv.in_stride = size_QlP * n_;
    bcv.ob = (int)size_Ql;
    for (int p = 0; p < np; ++p) {
      bcv.mat[p] = p_to_ql_.d_qhat_mod_p.get();
      bcv.ib[p] = (int)size_P_;
    }
    hip_ok(phx::ntt_forward_bconv(ntt, delta, dm, bcv, epi, s), "moddown bconv + NTT + finish");
  } else {
    phx::BconvArgs ba = p_to_ql_.args(cp, delta, false);
    ba.polys = np;
    ba.in_stride = size_QlP * n_;
    ba.out_stride = size_Ql * n_;
    hip_ok(phx::bconv(ba, n_, s), "moddown bconv");
    hip_ok(phx::ntt_forward_fused(ntt, delta, delta, dm, nullptr, 0, epi, s), "moddown NTT + finish");
  }
  if (unbiased()) unbias_ntt(ct, polys, size_Ql, size_Ql * n_, false, s);
}

void RnsTool::moddown_modup(uint64_t* t_mod_up, uint64_t* c1, const phx::NttTables& ntt, hipStream_t s, size_t count,
                            size_t c1_stride) const {
  const size_t size_Ql = base_Ql_.size(), size_QlP = size_Ql + size_P_, alpha = size_P_, beta = converters_.size();
  if (size_P_ == 0) throw std::invalid_argument("no special primes");
  if (count < 1 || (count > 1 && c1_stride < size_QlP * n_)) throw std::invalid_argument("moddown_modup: bad batch");
  const int nc = static_cast<int>(count);
#if PHX_DIAG_CENTRED
  if (kDiagModdown) {
    std::vector<uint64_t> mods(base_Ql_);
    mods.insert(mods.end(), base_P_.begin(), base_P_.end());
    diag_unbias(c1, count, count > 1 ? c1_stride : 0, mods, (int)size_Ql, size_Q_, base_P_, size_P_, n_, ntt, s);
  }
#endif
  phx::LimbMap all;
  all.num_limbs = (int)size_QlP;
  all.split = (int)size_Ql;
  all.first_a = 0;
  all.first_b = (int)size_Q_;
  hip_ok(phx::ntt_inverse(ntt, c1, c1, all.batched(nc, c1_stride, c1_stride), d_mm_scale_.get(),
                          d_mm_scale_shoup_.get(), s),
         "moddown-modup INTT");
  uint64_t* delta = ws_->get(s, Workspace::kModdownDelta, count * size_Ql * n_);
  phx::BconvArgs ba = p_to_ql_.args(c1 + size_Ql * n_, delta, false);
  ba.polys = nc;
  ba.in_stride = c1_stride;
  ba.out_stride = size_Ql * n_;
  hip_ok(phx::bconv(ba, n_, s), "moddown-modup bconv P");
  uint64_t* t_cks = ws_->get(s, Workspace::kModupInv, count * size_Ql * n_);
  phx::ModdownModupConsts k{d_Ql_.get(), d_bigPInv_mod_q_.get(), d_bigPInv_mod_q_shoup_.get(), d_partQlHatInv_.get(),
                            d_partQlHatInv_shoup_.get(), unbiased() ? k_md_ : 0};
  hip_ok(phx::moddown_modup_finish(c1, delta, k, t_cks, t_mod_up, n_, size_Ql, size_QlP, alpha, s, count, c1_stride,
                                   beta * size_QlP * n_),
         "moddown-modup finish");
  digit_bconv(t_cks, t_mod_up, s, count);
  hip_ok(phx::ntt_forward(ntt, t_mod_up, t_mod_up, all.batched(nc * (int)beta), s), "moddown-modup NTT");
}

void RnsTool::moddown_rescale(uint64_t* out, uint64_t* cx, const phx::NttTables& ntt, hipStream_t s,
                              size_t polys, const phx::NttEpilogue* ks) const {
  const size_t size_Ql = base_Ql_.size(), size_QlP = size_Ql + size_P_;
  if (size_Ql < 2 || size_P_ == 0) throw std::invalid_argument("end of modulus switching chain reached");
  const size_t Ln = size_Ql - 1;
#if PHX_DIAG_CENTRED
  if (ks) throw std::runtime_error("PHX_DIAG_CENTRED build: run with PHX_KS_EPI=0");
  if (kDiagModdown) {
    std::vector<uint64_t> mods(base_Ql_), div(base_P_);
    mods.insert(mods.end(), base_P_.begin(), base_P_.end());
    div.push_back(base_Ql_.back());
    diag_unbias(cx, polys, size_QlP * n_, mods, (int)size_Ql, size_Q_, div, size_P_ + 1, n_, ntt, s);
  }
#endif
  const int np = static_cast<int>(polys);
  // the dropped limbs q_last, p_0 .. p_{P-1} are contiguous in the extended buffer
  uint64_t* dropped = cx + Ln * n_;
  phx::LimbMap dm;
  dm.num_limbs = (int)(1 + size_P_);
  dm.split = 1;
  dm.first_a = (int)Ln;
  dm.first_b = (int)size_Q_;
  const bool fused = fused_bconv_ok(1 + size_P_) && polys <= (size_t)phx::kMaxBconvPolys;
  const phx::LimbMap dmb = dm.batched(np, size_QlP * n_, size_QlP * n_);
  if (ks) {  // the inner product's dropped limbs (q_last with its addend, P) as the INTT's prologue
    if (ks->ks_beta > phx::kMaxKsBeta) throw std::invalid_argument("moddown_rescale: too many key-switch digits");
    phx::NttEpilogue pro = *ks;
    pro.tmu_limb0 = Ln;
    pro.add_limbs = ks->add_c ? 1 : 0;
    hip_ok(phx::ntt_inverse_ks(ntt, dropped, dmb, pq_to_ql1_.d_qhat_inv.get(), pq_to_ql1_.d_qhat_inv_shoup.get(), pro,
                               s),
           "moddown-rescale inner product + INTT");
  } else {
    hip_ok(phx::ntt_inverse(ntt, dropped, dropped, dmb, pq_to_ql1_.d_qhat_inv.get(), pq_to_ql1_.d_qhat_inv_shoup.get(),
                            s),
           "moddown-rescale INTT");
  }
  uint64_t* delta = ws_->get(s, Workspace::kModdownDelta, polys * Ln * n_);
  phx::NttEpilogue epi;
  epi.c = cx;
  epi.c_stride = size_QlP * n_;
  epi.out = out;
  epi.out_stride = Ln * n_;
  epi.w = d_PQinv_.get();
  epi.ws = d_PQinv_shoup_.get();
  if (ks) {
    epi.ks_beta = ks->ks_beta;
    epi.tmu = ks->tmu;
    epi.tmu_stride = ks->tmu_stride;
    epi.evk = ks->evk;
    epi.evk_poly_stride = ks->evk_poly_stride;
    epi.add_c = ks->add_c;
    epi.add_stride = ks->add_stride;
    epi.pmod = ks->pmod;
    epi.pmod_shoup = ks->pmod_shoup;
    epi.ks_prods = ks->ks_prods;
    epi.tmu_prod_stride = ks->tmu_prod_stride;
    for (int k = 0; k < phx::kMaxKsProds; ++k) {
      epi.out_p[k] = ks->out_p[k];
      epi.add_p[k] = ks->add_p[k];
    }
  }
  const phx::LimbMap om = phx::LimbMap::contiguous((int)Ln, 0).batched(np);
  if (fused) {
    phx::BconvPrologue bcv;
    bcv.in = dropped;
    bcv.in_stride = size_QlP * n_;
    bcv.ob = (int)Ln;
    for (int p = 0; p < np; ++p) {
      bcv.mat[p] = pq_to_ql1_.d_qhat_mod_p.get();
      bcv.ib[p] = (int)(1 + size_P_);
    }
    hip_ok(phx::ntt_forward_bconv(ntt, delta, om, bcv, epi, s), "moddown-rescale bconv + NTT + finish");
  } else {
    phx::BconvArgs ba = pq_to_ql1_.args(dropped, delta, false);
    ba.polys = np;
    ba.in_stride = size_QlP * n_;
    ba.out_stride = Ln * n_;
    hip_ok(phx::bconv(ba, n_, s), "moddown-rescale bconv");
    hip_ok(phx::ntt_forward_fused(ntt, delta, delta, om, nullptr, 0, epi, s), "moddown-rescale NTT + finish");
  }
  if (unbiased()) {
    if (epi.ks_prods > 1) {  // per-product outputs, [2][Ln][n] each
      for (int k = 0; k < epi.ks_prods; ++k) unbias_ntt(epi.out_p[k], 2, Ln, Ln * n_, true, s);
    } else {
      unbias_ntt(out, polys, Ln, Ln * n_, true, s);
    }
  }
}

void RnsTool::set_unbias(const uint64_t* ones_ntt, hipStream_t s) {
  ones_ntt_ = ones_ntt;
  if (!ones_ntt) return;
  const size_t size_Ql = base_Ql_.size();
  k_md_ = size_P_ / 2;
  k_mdr_ = (size_P_ + 1) / 2;
  std::vector<uint64_t> a(size_Ql), as(size_Ql), b(size_Ql), bs(size_Ql);
  for (size_t i = 0; i < size_Ql; ++i) {
    const uint64_t q = base_Ql_[i];
    a[i] = k_md_ % q;
    as[i] = shoup(a[i], q);
    b[i] = k_mdr_ % q;
    bs[i] = shoup(b[i], q);
  }
  d_k_md_.upload(a, s);
  d_k_md_shoup_.upload(as, s);
  d_k_mdr_.upload(b, s);
  d_k_mdr_shoup_.upload(bs, s);
}

void RnsTool::unbias_ntt(uint64_t* out, size_t polys, size_t limbs, size_t stride, bool rescale, hipStream_t s) const {
  const uint64_t* k = rescale ? d_k_mdr_.get() : d_k_md_.get();
  const uint64_t* ks = rescale ? d_k_mdr_shoup_.get() : d_k_md_shoup_.get();
  hip_ok(phx::mul_scalar_accumulate(ones_ntt_, k, ks, out, stride, polys, d_Ql_.get(), n_, limbs, s), "unbiased moddown");
}

void RnsTool::rescale_ntt_to(const uint64_t* in, uint64_t* const* outs, size_t cts, const phx::NttTables& ntt,
                             hipStream_t s) const {
  const size_t L = base_Ql_.size();
  if (L < 2) throw std::invalid_argument("end of modulus switching chain reached");
  if (cts < 1 || cts > static_cast<size_t>(phx::kMaxKsProds)) throw std::invalid_argument("rescale: bad batch");
  const size_t Ln = L - 1, polys = 2 * cts;
  const int np = static_cast<int>(polys);
#if PHX_DIAG_CENTRED
  DeviceBuffer<uint64_t> diag_in(polys * L * n_, s);
  PHX_CHECK(hipMemcpyAsync(diag_in.get(), in, polys * L * n_ * 8, hipMemcpyDeviceToDevice, s));
  if (kDiagRescale) diag_unbias(diag_in.get(), polys, L * n_, base_Ql_, (int)L, size_Q_, {base_Ql_.back()}, 1, n_, ntt, s);
  in = diag_in.get();
#endif
  uint64_t* last = ws_->get(s, Workspace::kRescaleLast, polys * n_);
  hip_ok(phx::ntt_inverse(ntt, in + Ln * n_, last, phx::LimbMap::contiguous(1, (int)Ln).batched(np, L * n_, n_),
                          nullptr, nullptr, s),
         "rescale INTT(last)");
  // the two passes' intermediate in scratch; the finish writes each ciphertext's own buffer
  uint64_t* mid = ws_->get(s, Workspace::kModdownDelta, polys * Ln * n_);
  phx::NttEpilogue epi;
  epi.c = in;
  epi.c_stride = L * n_;
  epi.out = outs[0];
  epi.out_stride = Ln * n_;
  epi.w = d_inv_qlast_.get();
  epi.ws = d_inv_qlast_shoup_.get();
  epi.ks_prods = static_cast<int>(cts);
  for (size_t k = 0; k < cts; ++k) epi.out_p[k] = outs[k];
  hip_ok(phx::ntt_forward_fused(ntt, nullptr, mid, phx::LimbMap::contiguous((int)Ln, 0).batched(np), last, n_, epi, s),
         "rescale NTT + finish");
}

void RnsTool::rescale_ntt(const uint64_t* in, uint64_t* out, size_t polys, const phx::NttTables& ntt,
                          hipStream_t s) const {
  const size_t L = base_Ql_.size();
  if (L < 2) throw std::invalid_argument("end of modulus switching chain reached");
  const size_t Ln = L - 1;
  const int np = static_cast<int>(polys);
#if PHX_DIAG_CENTRED
  DeviceBuffer<uint64_t> diag_in(polys * L * n_, s);
  PHX_CHECK(hipMemcpyAsync(diag_in.get(), in, polys * L * n_ * 8, hipMemcpyDeviceToDevice, s));
  if (kDiagRescale) diag_unbias(diag_in.get(), polys, L * n_, base_Ql_, (int)L, size_Q_, {base_Ql_.back()}, 1, n_, ntt, s);
  in = diag_in.get();
#endif
  uint64_t* last = ws_->get(s, Workspace::kRescaleLast, polys * n_);
  // all polynomials in one launch per stage
  hip_ok(phx::ntt_inverse(ntt, in + Ln * n_, last, phx::LimbMap::contiguous(1, (int)Ln).batched(np, L * n_, n_),
                          nullptr, nullptr, s),
         "rescale INTT(last)");
  // NTT of the last limb spread over the others (the prologue reduces it per limb), with the
  // finish (c - NTT) q_last^-1 as the epilogue; `out` holds the intermediate of the two passes
  phx::NttEpilogue epi;
  epi.c = in;
  epi.c_stride = L * n_;
  epi.out = out;
  epi.out_stride = Ln * n_;
  epi.w = d_inv_qlast_.get();
  epi.ws = d_inv_qlast_shoup_.get();
  hip_ok(phx::ntt_forward_fused(ntt, nullptr, out, phx::LimbMap::contiguous((int)Ln, 0).batched(np), last, n_, epi, s),
         "rescale NTT + finish");
}

}  // namespace phantom
