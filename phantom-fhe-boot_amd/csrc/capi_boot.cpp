// capi_boot.cpp — C-ABI of the bootstrapping harness (declared in include/phantom_amd.h): the
// SimpleBootstrapExample set-up of bootstrapping/bootstrapping_example.cu:69-160 as one session
// object, and batches of bootstraps over serialized ciphertexts held in device memory — the form
// in which a multi-GPU job scatters its inputs and gathers its results (bench.py, config C5).
#include <cmath>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../host/bootstrap.h"
#include "../host/capi_internal.h"
#include "../host/ckks_eval.h"
#include "../host/encoder.h"
#include "../host/evaluate.h"
#include "../host/keys.h"
#include "../host/modulus.h"
#include "../host/serialize.h"
#include "../host/traffic.h"
#include "phantom_amd.h"

using phantom::capi::fail;
using phantom::capi::from_hip;
using namespace phantom;
using phantom::arith::CoeffModulus;

struct phantom_boot_session {
  std::unique_ptr<PhantomContext> ctx;
  std::unique_ptr<PhantomCKKSEncoder> enc;
  std::unique_ptr<PhantomSecretKey> sk;
  std::unique_ptr<FHECKKSRNS> boot;
  std::vector<double> sf;
  uint32_t slots = 0, iterations = 1, precision = 0;
};

namespace {

// a ciphertext from its serialized bytes in device memory (the format of PhantomCiphertext::save,
// include/ciphertext.h:184-225): the 58-byte header comes to the host, the words are copied device
// to device (they start at byte 58, so the copy also aligns them)
PhantomCiphertext load_device(const PhantomContext& ctx, const uint8_t* dev, size_t capacity) {
  if (capacity < ser::kCiphertextHeaderBytes) throw std::invalid_argument("serialized ciphertext truncated");
  hipStream_t s = ctx.stream();
  char hb[ser::kCiphertextHeaderBytes];
  PHX_CHECK(hipMemcpyAsync(hb, dev, sizeof(hb), hipMemcpyDeviceToHost, s));
  PHX_CHECK(hipStreamSynchronize(s));
  std::istringstream is(std::string(hb, sizeof(hb)));
  ser::CiphertextHeader h;
  ser::read_ciphertext_header(is, h);
  check_ciphertext_header(ctx, h);
  if (h.words() > (capacity - ser::kCiphertextHeaderBytes) / sizeof(uint64_t))
    throw std::invalid_argument("serialized ciphertext truncated");
  PhantomCiphertext ct;
  ct.resize(ctx, h.chain_index, h.size, s, false);
  PHX_CHECK(hipMemcpyAsync(ct.data(), dev + ser::kCiphertextHeaderBytes, h.words() * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, s));
  ct.set_scale(h.scale);
  ct.set_correction_factor(h.correction_factor);
  ct.SetNoiseScaleDeg(h.noise_scale_deg);
  ct.set_ntt_form(h.is_ntt_form);
  ct.set_asymmetric(h.is_asymmetric);
  return ct;
}

size_t serialized_bytes(const PhantomCiphertext& ct) {
  return ser::kCiphertextHeaderBytes + ct.size() * ct.coeff_modulus_size() * ct.poly_modulus_degree() * sizeof(uint64_t);
}

void save_device(const PhantomContext& ctx, const PhantomCiphertext& ct, uint8_t* dev, size_t capacity) {
  const size_t need = serialized_bytes(ct);
  if (capacity < need) throw std::invalid_argument("output slot too small for the serialized ciphertext");
  ser::CiphertextHeader h;
  h.chain_index = ct.chain_index();
  h.size = ct.size();
  h.poly_modulus_degree = ct.poly_modulus_degree();
  h.coeff_modulus_size = ct.coeff_modulus_size();
  h.scale = ct.scale();
  h.correction_factor = ct.correction_factor();
  h.noise_scale_deg = ct.GetNoiseScaleDeg();
  h.is_ntt_form = ct.is_ntt_form();
  h.is_asymmetric = ct.is_asymmetric();
  std::ostringstream os;
  ser::write_ciphertext_header(os, h);  // the words follow device to device
  const std::string hb = os.str();
  hipStream_t s = ctx.stream();
  PHX_CHECK(hipMemcpyAsync(dev, hb.data(), hb.size(), hipMemcpyHostToDevice, s));
  PHX_CHECK(hipMemcpyAsync(dev + ser::kCiphertextHeaderBytes, ct.data(), need - ser::kCiphertextHeaderBytes,
                           hipMemcpyDeviceToDevice, s));
  PHX_CHECK(hipStreamSynchronize(s));  // the header's host source is a temporary
}

phantom_boot_session& session(phantom_boot_session* s) {
  if (!s || !s->ctx) throw std::invalid_argument("null bootstrap session");
  return *s;
}

}  // namespace

extern "C" {

int phantom_traffic_read(uint64_t* out) {
  if (!out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
  auto& c = traffic::counters();
  out[0] = c.keys.load();
  out[1] = c.plaintexts.load();
  out[2] = c.ciphertexts.load();
  return PHANTOM_OK;
}

int phantom_traffic_reset(void) {
  auto& c = traffic::counters();
  c.keys = 0;
  c.plaintexts = 0;
  c.ciphertexts = 0;
  return PHANTOM_OK;
}

int phantom_pool_stats(uint64_t* out) {
  if (!out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
  const phantom::DevicePool::Stats st = phantom::DevicePool::instance().stats();
  out[0] = st.held;
  out[1] = st.live;
  out[2] = st.peak_live;
  out[3] = st.peak_held;
  return PHANTOM_OK;
}

int phantom_pool_reset_peak(void) {
  phantom::DevicePool::instance().reset_peak();
  return PHANTOM_OK;
}

int phantom_eval_mod_coefficients(uint32_t K, uint32_t double_angle_iterations, int degree, double* out) {
  PHX_CAPI_GUARD({
    if (!out || degree < 1 || degree > 1024 || K < 1) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad arguments");
    const double args[2] = {static_cast<double>(K), static_cast<double>(double_angle_iterations)};
    const std::vector<double> c = boot::chebyshev_coefficients(boot::scaled_cosine, args, degree);
    std::memcpy(out, c.data(), c.size() * sizeof(double));
    return PHANTOM_OK;
  });
}

int phantom_boot_session_create(int log_n, int depth, int special, const uint32_t* level_budget, uint32_t num_slots,
                                uint32_t num_iterations, uint32_t precision, const uint8_t* seed,
                                phantom_boot_session** out) {
  PHX_CAPI_GUARD({
    if (!level_budget || !seed || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (log_n < 10 || log_n > 17 || depth < 1 || special < 1) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad parameters");
    auto b = std::make_unique<phantom_boot_session>();
    const size_t N = size_t(1) << log_n;
    // bootstrapping_example.cu:76-116: {60, depth x 59, special x 60}, scale 2^59
    std::vector<int> bits(1, 60);
    bits.insert(bits.end(), static_cast<size_t>(depth), 59);
    bits.insert(bits.end(), static_cast<size_t>(special), 60);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(N);
    parms.set_special_modulus_size(static_cast<size_t>(special));
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    const double scale = std::pow(2.0, 59);
    b->ctx = std::make_unique<PhantomContext>(parms);
    b->enc = std::make_unique<PhantomCKKSEncoder>(*b->ctx);
    if (num_slots) b->enc->set_sparse_encode(2 * size_t(num_slots));
    b->sk = std::make_unique<PhantomSecretKey>(PhantomSecretKey::from_seed(*b->ctx, seed));
    PhantomCiphertext tmp;
    tmp.PreComputeScale(*b->ctx, scale);
    b->sf = tmp.getScalingFactorsReal();
    b->slots = num_slots ? num_slots : static_cast<uint32_t>(N / 2);
    b->iterations = num_iterations ? num_iterations : 1;
    b->precision = precision;
    b->boot = std::make_unique<FHECKKSRNS>(*b->enc);
    b->boot->EvalBootstrapSetup(*b->ctx, {level_budget[0], level_budget[1]}, scale, b->sf, 0, b->slots);
    b->boot->EvalMultKeyGen(*b->sk, *b->ctx);
    b->boot->EvalBootstrapKeyGen(*b->sk, *b->ctx, b->slots);
    PHX_CHECK(hipDeviceSynchronize());
    *out = b.release();
    return PHANTOM_OK;
  });
}

int phantom_boot_layout(int log_n, int depth, int special, const uint32_t* level_budget, uint32_t num_slots,
                        uint32_t num_iterations, size_t chain_index, size_t* in_bytes, size_t* out_bytes,
                        size_t* out_chain) {
  PHX_CAPI_GUARD({
    if (!level_budget || !in_bytes || !out_bytes || !out_chain) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (log_n < 10 || log_n > 17 || depth < 1 || special < 1) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad parameters");
    const size_t N = size_t(1) << log_n, size_Q = static_cast<size_t>(depth) + 1;
    const uint32_t slots = num_slots ? num_slots : static_cast<uint32_t>(N / 2);
    if (slots & (slots - 1)) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "slot count not a power of two");
    if (chain_index < 1 || chain_index + 1 > size_Q) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad chain index");
    const size_t oc = FHECKKSRNS::OutputChainIndex({level_budget[0], level_budget[1]},
                                                   static_cast<uint32_t>(__builtin_ctz(slots)), num_iterations);
    if (oc > size_Q) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "not enough levels for bootstrapping");
    *in_bytes = ser::kCiphertextHeaderBytes + 2 * (size_Q - (chain_index - 1)) * N * 8;
    *out_bytes = ser::kCiphertextHeaderBytes + 2 * (size_Q - (oc - 1)) * N * 8;
    *out_chain = oc;
    return PHANTOM_OK;
  });
}

int phantom_boot_session_destroy(phantom_boot_session* s) {
  if (s) (void)hipDeviceSynchronize();
  delete s;
  return PHANTOM_OK;
}

int phantom_boot_encrypt(phantom_boot_session* s, const double* values, size_t count, size_t chain_index,
                         uint8_t* dev_out, size_t stride, size_t* ct_bytes) {
  PHX_CAPI_GUARD({
    auto& b = session(s);
    if (!values || !dev_out || !ct_bytes) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (chain_index < 1 || chain_index > b.ctx->size_Q() - 1)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "a bootstrap input needs at least two limbs");
    const size_t need = ser::kCiphertextHeaderBytes +
                        2 * b.ctx->get_context_data(chain_index).coeff_modulus_size() * b.ctx->poly_degree() * 8;
    *ct_bytes = need;
    if (stride < need) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "stride smaller than one serialized ciphertext");
    for (size_t i = 0; i < count; ++i) {
      std::vector<double> v(values + i * b.slots, values + (i + 1) * b.slots);
      PhantomPlaintext pt;
      // FLEXIBLEAUTO: a ciphertext at level l carries scale sf[l] (chain index = l + 1)
      if (b.slots < b.ctx->poly_degree() / 2) b.enc->encode_sparse(*b.ctx, v, b.sf.at(chain_index - 1), pt, chain_index);
      else b.enc->encode(*b.ctx, v, b.sf.at(chain_index - 1), pt, chain_index);
      PhantomCiphertext ct = b.sk->encrypt_symmetric(*b.ctx, pt);
      save_device(*b.ctx, ct, dev_out + i * stride, stride);
    }
    return PHANTOM_OK;
  });
}

int phantom_boot_output_bytes(phantom_boot_session* s, size_t* bytes) {
  PHX_CAPI_GUARD({
    auto& b = session(s);
    if (!bytes) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    *bytes = ser::kCiphertextHeaderBytes +
             2 * b.ctx->get_context_data(b.boot->output_chain_index(b.slots, b.iterations)).coeff_modulus_size() * b.ctx->poly_degree() * 8;
    return PHANTOM_OK;
  });
}

int phantom_boot_run(phantom_boot_session* s, const uint8_t* dev_in, size_t in_stride, size_t count, uint8_t* dev_out,
                     size_t out_stride, int lanes) {
  return phantom_boot_run_grouped(s, dev_in, in_stride, count, dev_out, out_stride, lanes,
                                  static_cast<int>(FHECKKSRNS::kBootGroup));
}

int phantom_boot_run_grouped(phantom_boot_session* s, const uint8_t* dev_in, size_t in_stride, size_t count,
                             uint8_t* dev_out, size_t out_stride, int lanes, int group) {
  PHX_CAPI_GUARD({
    auto& b = session(s);
    if ((!dev_in || !dev_out) && count) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (group < 1 || group > phx::kLtGroupMax)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "group must be 1..kLtGroupMax");
    std::vector<PhantomCiphertext> in;
    in.reserve(count);
    for (size_t i = 0; i < count; ++i) in.push_back(load_device(*b.ctx, dev_in + i * in_stride, in_stride));
    std::vector<PhantomCiphertext> out;
    if (b.iterations > 1) {
      for (auto& c : in) out.push_back(b.boot->EvalBootstrap(c, *b.ctx, b.slots, b.iterations, b.precision));
    } else {
      out = b.boot->EvalBootstrapBatch(in, *b.ctx, lanes, b.slots, static_cast<size_t>(group));
    }
    for (size_t i = 0; i < count; ++i) save_device(*b.ctx, out[i], dev_out + i * out_stride, out_stride);
    return PHANTOM_OK;
  });
}

int phantom_boot_decrypt(phantom_boot_session* s, const uint8_t* dev_in, size_t capacity, double* values_out) {
  PHX_CAPI_GUARD({
    auto& b = session(s);
    if (!dev_in || !values_out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    PhantomCiphertext ct = load_device(*b.ctx, dev_in, capacity);
    // dropping limbs is exact (the plaintext is unchanged); decoding two limbs is cheaper
    const size_t two = b.ctx->size_Q() - 1;
    if (ct.chain_index() < two) mod_switch_to_inplace(*b.ctx, ct, two);
    PhantomPlaintext pt = b.sk->decrypt(*b.ctx, ct);
    std::vector<double> v;
    b.enc->decode(*b.ctx, pt, v);
    std::memcpy(values_out, v.data(), b.slots * sizeof(double));
    return PHANTOM_OK;
  });
}

}  // extern "C"
