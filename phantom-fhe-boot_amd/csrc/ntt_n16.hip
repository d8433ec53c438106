// ntt_n16.hip — explicit instantiations of the 2-D NTT launch<S1, S2> (csrc/ntt_impl.h) for n = 2^16.
#include "ntt_impl.h"

namespace phx {
namespace nttd {
template hipError_t launch<8, 8>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
}  // namespace nttd
}  // namespace phx

#if PHX_NTT_STAMP
extern "C" int phantom_debug_ntt_stamps(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(phx::nttd::g_ntt_stamps), bytes);
}
extern "C" int phantom_debug_ntt_stamps_clear() {
  static uint64_t zeros[phx::nttd::kStampSlots * 8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(phx::nttd::g_ntt_stamps), zeros, sizeof(zeros));
}
#endif
