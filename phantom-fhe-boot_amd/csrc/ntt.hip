// ntt.hip — NTT launchers (include/ntt.cuh:157-226 replacements, csrc/ntt.h): degree dispatch over the
// 2-D kernels of ntt_impl.h (instantiated in ntt_n*.hip) and the 1-D radix-2 path for small degrees.
#include "ntt_impl.h"

namespace phx {
namespace nttd {
extern template hipError_t launch<5, 5>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<5, 6>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<6, 6>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<6, 7>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<7, 7>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<7, 8>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<8, 8>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
extern template hipError_t launch<8, 9>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);

hipError_t launch_1d(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                     const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream, const uint64_t* bcast,
                     size_t bcast_stride, const NttEpilogue& epi) {
  if (tb.log_n < 3 || tb.log_n > kMaxLog1D) return hipErrorInvalidValue;
  const int per_poly = map.num_limbs - (map.skip_end - map.skip_begin);
  if (per_poly <= 0 || map.polys <= 0) return hipSuccess;
  KArgs a{};
  a.in = in; a.out = out; a.modulus = tb.modulus;
  a.tw = inverse ? tb.itw : tb.tw;
  a.tws = inverse ? tb.itw_shoup : tb.tw_shoup;
  a.n_inv = tb.n_inv; a.n_inv_shoup = tb.n_inv_shoup;
  a.scale = scale; a.scale_shoup = scale_shoup;
  a.map = map; a.n = (int)tb.n; a.limbs = per_poly * map.polys; a.limbs_per_poly = per_poly;
  a.barrett = tb.barrett;
  a.bcast = inverse ? nullptr : bcast;
  a.bcast_stride = bcast_stride;
  a.epi = inverse ? NttEpilogue{} : epi;
  if (a.map.in_stride == 0) a.map.in_stride = (size_t)map.num_limbs * tb.n;
  if (a.map.out_stride == 0) a.map.out_stride = (size_t)map.num_limbs * tb.n;
  const dim3 grid(a.limbs), block(std::max<unsigned>(64, (unsigned)tb.n / 2));
  if (inverse) hipLaunchKernelGGL(ntt_1d<false>, grid, block, 0, stream, a);
  else hipLaunchKernelGGL(ntt_1d<true>, grid, block, 0, stream, a);
  return hipGetLastError();
}

hipError_t dispatch(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                    const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream,
                    const uint64_t* bcast = nullptr, size_t bcast_stride = 0, const NttEpilogue& epi = NttEpilogue{},
                    const BconvPrologue* bcv = nullptr, const NttCopy& copy = NttCopy{}) {
#define PHX_NTT_CASE(LOGN, A, B) \
  case LOGN: return launch<A, B>(tb, in, out, map, inverse, scale, scale_shoup, stream, bcast, bcast_stride, epi, bcv, copy);
  if (tb.log_n < 10) {
    if (bcv || copy.out) return hipErrorNotSupported;
    return launch_1d(tb, in, out, map, inverse, scale, scale_shoup, stream, bcast, bcast_stride, epi);
  }
  switch (tb.log_n) {
    PHX_NTT_CASE(10, 5, 5) PHX_NTT_CASE(11, 5, 6) PHX_NTT_CASE(12, 6, 6) PHX_NTT_CASE(13, 6, 7)
    PHX_NTT_CASE(14, 7, 7) PHX_NTT_CASE(15, 7, 8) PHX_NTT_CASE(16, 8, 8) PHX_NTT_CASE(17, 8, 9)
    default: return hipErrorInvalidValue;
  }
#undef PHX_NTT_CASE
}

// the key-switch form's operands (ntt.h NttEpilogue): every launcher that can receive one checks them
hipError_t check_ks(const NttTables& t, const LimbMap& map, const NttEpilogue& ks) {
  if (ks.ks_prods < 1 || ks.ks_prods > kMaxKsProds) return hipErrorInvalidValue;
  if (ks.ks_prods > 1) {  // per-pair outputs (and addends): the map must hold exactly those pairs
    if (map.polys != 2 * ks.ks_prods) return hipErrorInvalidValue;
    for (int k = 0; k < ks.ks_prods; ++k)
      if (!ks.out_p[k] || (ks.ks_beta > 0 && ks.add_c && !ks.add_p[k])) return hipErrorInvalidValue;
  }
  if (ks.ks_beta == 0) return hipSuccess;
  if (ks.ks_beta < 1 || ks.ks_beta > kMaxKsBeta || !ks.tmu || !ks.evk) return hipErrorInvalidValue;
  if (map.polys != 2 * ks.ks_prods) return hipErrorInvalidValue;
  if (t.log_n < 10) return hipErrorNotSupported;  // the 1-D path has no key-switch form
  return hipSuccess;
}

}  // namespace nttd

using namespace nttd;

hipError_t ntt_forward(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       hipStream_t stream) {
  return dispatch(t, in, out, map, false, nullptr, nullptr, stream);
}

hipError_t ntt_forward_fused(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                             const uint64_t* bcast, size_t bcast_stride, const NttEpilogue& epi, hipStream_t stream) {
  if (epi.out && (!epi.c || !epi.w || !epi.ws)) return hipErrorInvalidValue;
  if (hipError_t e = check_ks(t, map, epi)) return e;
  return dispatch(t, in, out, map, false, nullptr, nullptr, stream, bcast, bcast_stride, epi);
}

hipError_t ntt_forward_bconv(const NttTables& t, uint64_t* out, const LimbMap& map, const BconvPrologue& bcv,
                             const NttEpilogue& epi, hipStream_t stream) {
  if (epi.out && (!epi.c || !epi.w || !epi.ws)) return hipErrorInvalidValue;
  if (hipError_t e = check_ks(t, map, epi)) return e;
  if (!bcv.in || bcv.ob <= 0 || map.polys < 1 || map.polys > kMaxBconvPolys) return hipErrorInvalidValue;
  const int per_poly = map.num_limbs - (map.skip_end - map.skip_begin);
  for (int p = 0; p < map.polys; ++p) {
    if (!bcv.mat[p] || bcv.ib[p] < 1 || bcv.ib[p] > 15) return hipErrorInvalidValue;
    if (per_poly > bcv.ob) return hipErrorInvalidValue;
  }
  return dispatch(t, nullptr, out, map, false, nullptr, nullptr, stream, nullptr, 0, epi, &bcv);
}

hipError_t ntt_inverse(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  return dispatch(t, in, out, map, true, scale, scale_shoup, stream);
}

hipError_t ntt_inverse_ks(const NttTables& t, uint64_t* out, const LimbMap& map, const uint64_t* scale,
                          const uint64_t* scale_shoup, const NttEpilogue& ks, hipStream_t stream) {
  if (ks.ks_beta < 1) return hipErrorInvalidValue;
  if (hipError_t e = check_ks(t, map, ks)) return e;
  if (ks.add_limbs > 0 && (!ks.add_c || !ks.pmod || !ks.pmod_shoup)) return hipErrorInvalidValue;
  return dispatch(t, nullptr, out, map, true, scale, scale_shoup, stream, nullptr, 0, ks);
}

hipError_t ntt_inverse_copy(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                            const uint64_t* scale, const uint64_t* scale_shoup, const NttCopy& copy,
                            hipStream_t stream) {
  if (!copy.out || copy.alpha < 1 || in == out) return hipErrorInvalidValue;
  return dispatch(t, in, out, map, true, scale, scale_shoup, stream, nullptr, 0, NttEpilogue{}, nullptr, copy);
}

hipError_t ntt_1d_forward(const NttTables& t, uint64_t* inout, const LimbMap& map, hipStream_t stream) {
  return launch_1d(t, inout, inout, map, false, nullptr, nullptr, stream, nullptr, 0, NttEpilogue{});
}

hipError_t ntt_1d_inverse(const NttTables& t, uint64_t* inout, const LimbMap& map, const uint64_t* scale,
                          const uint64_t* scale_shoup, hipStream_t stream) {
  return launch_1d(t, inout, inout, map, true, scale, scale_shoup, stream, nullptr, 0, NttEpilogue{});
}

}  // namespace phx
