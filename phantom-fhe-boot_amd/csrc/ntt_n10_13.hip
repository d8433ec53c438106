// ntt_n10_13.hip — explicit instantiations of the 2-D NTT launch<S1, S2> (csrc/ntt_impl.h) for n = 2^10, n = 2^11, n = 2^12, n = 2^13.
#include "ntt_impl.h"

namespace phx {
namespace nttd {
template hipError_t launch<5, 5>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
template hipError_t launch<5, 6>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
template hipError_t launch<6, 6>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
template hipError_t launch<6, 7>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
}  // namespace nttd
}  // namespace phx
