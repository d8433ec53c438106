// ntt_n17.hip — explicit instantiations of the 2-D NTT launch<S1, S2> (csrc/ntt_impl.h) for n = 2^17.
#include "ntt_impl.h"

namespace phx {
namespace nttd {
template hipError_t launch<8, 9>(const NttTables&, const uint64_t*, uint64_t*, const LimbMap&, bool, const uint64_t*, const uint64_t*, hipStream_t, const uint64_t*, size_t, const NttEpilogue&, const BconvPrologue*, const NttCopy&);
}  // namespace nttd
}  // namespace phx
