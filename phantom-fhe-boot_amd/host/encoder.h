// encoder.h — PhantomCKKSEncoder (include/ckks.h, src/ckks.cu): slots <-> NTT-form plaintexts.
//
// Slot j sits at the root zeta^(5^j) of X^N + 1 (zeta = exp(2 pi i / 2N)) and its conjugate at
// zeta^(-5^j), the convention of the reference and of every 5^j rotation group.  The canonical
// embedding and its inverse are evaluated on the host in double precision with one size-N
// complex FFT each (the reference runs its special FFT on the GPU, src/fft.cu); coefficients
// are rounded to integers, reduced into each RNS limb exactly and moved to NTT form on the GPU.
#pragma once

#include <complex>
#include <cstdint>
#include <vector>

#include "ciphertext.h"
#include "context.h"

namespace phantom {

class PhantomCKKSEncoder {
 public:
  explicit PhantomCKKSEncoder(const PhantomContext& ctx);
  // host-only maps (slots_to_coeffs / coeffs_to_slots) for ring degree n, no device use
  explicit PhantomCKKSEncoder(size_t n);

  size_t slot_count() const { return n_ / 2; }

  // encode(context, values, scale, plain[, chain_index]) (src/ckks.cu): plaintext in the Ql basis
  // of `chain_index`, NTT form.  Fewer values than slots are zero-padded.
  void encode(const PhantomContext& ctx, const std::vector<std::complex<double>>& values, double scale,
              PhantomPlaintext& out, size_t chain_index = 1) const;
  void encode(const PhantomContext& ctx, const std::vector<double>& values, double scale, PhantomPlaintext& out,
              size_t chain_index = 1) const;
  // sparse packing (the reference's set_sparse_encode / encode_sparse, include/ckks.h:82-117,
  // bootstrapping_example.cu:262-263): `values` (at most sparse_slots of them, zero-padded) fill
  // every block of sparse_slots slots, i.e. the plaintext is m'(X^(N / (2 sparse_slots))), the form
  // a sparse bootstrap expects.  set_sparse_encode takes the subring dimension 2 * sparse_slots.
  void set_sparse_encode(size_t subring_degree) { sparse_slots_ = subring_degree / 2; }
  void set_sparse_encode(const EncryptionParameters& parms, size_t subring_degree) {
    (void)parms;
    set_sparse_encode(subring_degree);
  }
  void encode_sparse(const PhantomContext& ctx, const std::vector<double>& values, double scale, PhantomPlaintext& out,
                     size_t chain_index = 1) const;
  void encode_sparse(const PhantomContext& ctx, const std::vector<std::complex<double>>& values, double scale,
                     PhantomPlaintext& out, size_t chain_index = 1) const;
  size_t sparse_slots() const { return sparse_slots_; }

  // encode_ext (the hoisted linear transforms' plaintexts): the Ql basis of `chain_index`
  // followed by the special primes P, NTT form ([size_Ql + size_P][n]).
  void encode_ext(const PhantomContext& ctx, const std::vector<std::complex<double>>& values, double scale,
                  PhantomPlaintext& out, size_t chain_index) const;
  // encode_ext in two halves, so many plaintexts can be prepared on host threads at once: the
  // host residues (coefficient form, limb-major; `rns_threads` 0 = spread limbs over threads)
  // and their upload + NTT on the context's stream.  `host` must stay alive until the stream
  // has run the upload (synchronise it before reusing or freeing `host`).
  void encode_ext_host(const PhantomContext& ctx, const std::vector<std::complex<double>>& values, double scale,
                       size_t chain_index, std::vector<uint64_t>& host, unsigned rns_threads = 0) const;
  void upload_ext_async(const PhantomContext& ctx, const std::vector<uint64_t>& host, double scale,
                        PhantomPlaintext& out, size_t chain_index) const;

  // decode(context, plain, values) (src/ckks.cu): exact CRT composition of each coefficient,
  // centered, divided by the plaintext's scale, then the canonical embedding.
  void decode(const PhantomContext& ctx, const PhantomPlaintext& plain, std::vector<std::complex<double>>& out) const;
  void decode(const PhantomContext& ctx, const PhantomPlaintext& plain, std::vector<double>& out) const;
  // decode<T>(context, plain) (include/ckks.h:174-206): T = std::complex<double> (the reference's
  // cuDoubleComplex) or double
  template <class T>
  std::vector<T> decode(const PhantomContext& ctx, const PhantomPlaintext& plain) const {
    std::vector<T> v;
    decode(ctx, plain, v);
    return v;
  }

  // host-side maps, exposed for the bootstrap precomputation and tests
  // slots -> real coefficients (inverse canonical embedding, coefficients not scaled)
  std::vector<double> slots_to_coeffs(const std::vector<std::complex<double>>& values) const;
  // real coefficients -> slots
  std::vector<std::complex<double>> coeffs_to_slots(const std::vector<double>& coeffs) const;

 private:
  // rounds coeffs * scale and writes residues for `moduli` (limb-major) to `out` (host)
  static void to_rns(const std::vector<double>& coeffs, double scale, const std::vector<uint64_t>& moduli,
                     std::vector<uint64_t>& out, unsigned threads = 0);
  void fft(std::vector<std::complex<double>>& a, bool inverse) const;

  size_t n_ = 0;
  int logn_ = 0;
  size_t sparse_slots_ = 0;
  std::vector<std::complex<double>> zeta_pows_;  // zeta^j, j < 2n
  std::vector<uint32_t> slot_index_;             // (5^j mod 2n - 1) / 2 for j < n/2
  std::vector<uint32_t> brev_;
};

}  // namespace phantom
