// ckks_example — the reference's examples/3_ckks.cu on this engine: the same calls in the same
// order (encode/decode, symmetric and asymmetric encryption, add/sub, multiply_plain, the
// x*y*x HomMul with relinearize / rescale_to_next / mod_switch_to_next, fused rotation and
// conjugation, the small-parameter apply_galois), with the reference's correctness rule: every
// slot within |real difference| < 1e-3 (3_ckks.cu:19,33-41), a std::logic_error otherwise.
//
// Documented substitutions (no CUDA names in this engine): std::complex<double> for
// cuDoubleComplex, std::mt19937_64 for rand() so a failing run can be replayed (--seed).
//
// usage: ckks_example [alpha ...] [--seed S]
//   alpha selects the reference's parameter sets (3_ckks.cu:761-818): 1, 2, 3, 4 at N = 2^15 with
//   40-bit primes, 15 = the C3 chain at N = 2^16 (Q = {60, 44 x 50}, P = 15 x 60).
//   Default: 15.  Prints one JSON line per example; exit status 0 iff all pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../host/ckks_eval.h"
#include "../host/encoder.h"
#include "../host/evaluate.h"
#include "../host/keys.h"
#include "../host/modulus.h"

using namespace phantom;
using namespace phantom::arith;
using cplx = std::complex<double>;

static constexpr double EPSINON = 0.001;  // 3_ckks.cu:19
static std::mt19937_64 g_rng;

static double rnd() { return std::uniform_real_distribution<double>(0.0, 1.0)(g_rng); }
// operator== of 3_ckks.cu:33-36 compares the real parts only
static bool eq(const cplx& a, const cplx& b) { return std::fabs(a.real() - b.real()) < EPSINON; }
static bool eq(double a, double b) { return std::fabs(a - b) < EPSINON; }  // compare_double

static std::vector<cplx> random_msg(size_t n) {
  std::vector<cplx> v(n);
  for (auto& x : v) {
    const double re = rnd();
    x = cplx(re, rnd());
  }
  return v;
}

static void require(bool ok, const char* what) {
  if (!ok) throw std::logic_error(what);
}

static void example_ckks_enc(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomCKKSEncoder encoder(context);
  const size_t slot_count = encoder.slot_count();
  std::vector<cplx> input = random_msg(slot_count);
  PhantomPlaintext x_plain;
  encoder.encode(context, input, scale, x_plain, 1);
  std::vector<cplx> result;
  encoder.decode(context, x_plain, result);
  bool correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input[i]);
  require(correctness, "encode/decode complex vector error");

  std::vector<double> input_double(slot_count);
  for (auto& v : input_double) v = rnd();
  PhantomPlaintext pt;
  encoder.encode(context, input_double, scale, pt, 1);
  std::vector<double> result_double;
  encoder.decode(context, pt, result_double);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result_double[i], input_double[i]);
  require(correctness, "encode/decode double vector error");

  PhantomCiphertext x_symmetric_cipher;
  secret_key.encrypt_symmetric(context, x_plain, x_symmetric_cipher);
  PhantomPlaintext x_symmetric_plain;
  secret_key.decrypt(context, x_symmetric_cipher, x_symmetric_plain);
  encoder.decode(context, x_symmetric_plain, result);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input[i]);
  require(correctness, "Symmetric encryption error");

  PhantomCiphertext x_asymmetric_cipher;
  public_key.encrypt_asymmetric(context, x_plain, x_asymmetric_cipher);
  PhantomPlaintext x_asymmetric_plain;
  secret_key.decrypt(context, x_asymmetric_cipher, x_asymmetric_plain);
  encoder.decode(context, x_asymmetric_plain, result);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input[i]);
  require(correctness, "Asymmetric encryption error");
}

// seed-compressed symmetric ciphertexts (include/ciphertext.h:227-318): save_symmetric writes c0
// and the seed of c1, load_symmetric regenerates c1 bit for bit; the loaded ciphertext decrypts
// to the message, and the asymmetric / 3-polynomial cases throw as in the reference
static void example_ckks_save_symmetric(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomCKKSEncoder encoder(context);
  std::vector<cplx> input = random_msg(encoder.slot_count()), result;
  PhantomPlaintext plain;
  encoder.encode(context, input, scale, plain);
  PhantomCiphertext sym;
  secret_key.encrypt_symmetric(context, plain, sym);
  std::stringstream ss;
  sym.save_symmetric(ss);
  const size_t words = sym.coeff_modulus_size() * sym.poly_modulus_degree();
  require(ss.str().size() == 58 + words * 8 + PhantomCiphertext::kSeedBytes, "save_symmetric size");
  PhantomCiphertext loaded;
  loaded.load_symmetric(context, ss);
  require(loaded.to_host(context.stream()) == sym.to_host(context.stream()), "load_symmetric: c0 || c1 differ");
  require(loaded.chain_index() == sym.chain_index() && loaded.scale() == sym.scale(), "load_symmetric header");
  secret_key.decrypt(context, loaded, plain);
  encoder.decode(context, plain, result);
  bool correctness = true;
  for (size_t i = 0; i < input.size(); i++) correctness &= eq(result[i], input[i]);
  require(correctness, "seed-compressed ciphertext decrypt error");
  PhantomCiphertext asym;
  public_key.encrypt_asymmetric(context, plain, asym);
  bool threw = false;
  try {
    asym.save_symmetric(ss);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  require(threw, "save_symmetric of an asymmetric ciphertext must throw");
}

static void example_ckks_add(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomCKKSEncoder encoder(context);
  const size_t slot_count = encoder.slot_count();
  std::vector<cplx> input1 = random_msg(slot_count), input2 = random_msg(slot_count), result;
  PhantomPlaintext x_plain, y_plain;
  encoder.encode(context, input1, scale, x_plain);
  encoder.encode(context, input2, scale, y_plain);

  PhantomCiphertext x_sym_cipher, y_sym_cipher;
  secret_key.encrypt_symmetric(context, x_plain, x_sym_cipher);
  secret_key.encrypt_symmetric(context, y_plain, y_sym_cipher);
  add_inplace(context, x_sym_cipher, y_sym_cipher);
  PhantomPlaintext p;
  secret_key.decrypt(context, x_sym_cipher, p);
  encoder.decode(context, p, result);
  bool correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input1[i] + input2[i]);
  require(correctness, "Symmetric HomAdd error");
  sub_inplace(context, x_sym_cipher, y_sym_cipher);
  secret_key.decrypt(context, x_sym_cipher, p);
  encoder.decode(context, p, result);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input1[i]);
  require(correctness, "Symmetric HomSub error");

  PhantomCiphertext x_asym_cipher, y_asym_cipher;
  public_key.encrypt_asymmetric(context, x_plain, x_asym_cipher);
  public_key.encrypt_asymmetric(context, y_plain, y_asym_cipher);
  add_inplace(context, y_asym_cipher, x_asym_cipher);
  secret_key.decrypt(context, y_asym_cipher, p);
  encoder.decode(context, p, result);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input1[i] + input2[i]);
  require(correctness, "Asymmetric HomAdd error");
  sub_inplace(context, x_asym_cipher, y_asym_cipher, true);  // x <- y - x
  secret_key.decrypt(context, x_asym_cipher, p);
  encoder.decode(context, p, result);
  correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], input2[i]);
  require(correctness, "Asymmetric HomSub error");
}

static void example_ckks_mul_plain(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomCKKSEncoder encoder(context);
  const size_t slot_count = encoder.slot_count();
  size_t msg_size = slot_count;
  std::vector<cplx> msg_vec = random_msg(msg_size), const_vec = random_msg(slot_count), result;
  PhantomPlaintext plain, const_plain;
  encoder.encode(context, msg_vec, scale, plain);
  encoder.encode(context, const_vec, scale, const_plain);
  PhantomCiphertext sym_cipher;
  secret_key.encrypt_symmetric(context, plain, sym_cipher);
  multiply_plain_inplace(context, sym_cipher, const_plain);
  secret_key.decrypt(context, sym_cipher, plain);
  encoder.decode(context, plain, result);
  bool correctness = true;
  for (size_t i = 0; i < msg_size; i++) correctness &= eq(result[i], msg_vec[i] * const_vec[i]);
  require(correctness, "Symmetric cipher multiply plain vector error");

  msg_size >>= 2;
  msg_vec = random_msg(msg_size);
  const_vec.assign(128, cplx(0.0, 0.0));
  {
    const double re = rnd();
    const_vec[2] = cplx(re, rnd());
  }
  encoder.encode(context, msg_vec, scale, plain);
  encoder.encode(context, const_vec, scale, const_plain);
  PhantomCiphertext asym_cipher;
  public_key.encrypt_asymmetric(context, plain, asym_cipher);
  multiply_plain_inplace(context, asym_cipher, const_plain);
  secret_key.decrypt(context, asym_cipher, plain);
  encoder.decode(context, plain, result);
  correctness = true;
  for (size_t i = 0; i < msg_size; i++)
    correctness &= i == 2 ? eq(result[i], msg_vec[i] * const_vec[i]) : eq(result[i], cplx(0.0, 0.0));
  require(correctness, "Asymmetric cipher multiply plain vector error");
}

static void example_ckks_mul(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomRelinKey relin_keys = secret_key.gen_relinkey(context);
  PhantomCKKSEncoder encoder(context);
  const size_t slot_count = encoder.slot_count();
  std::vector<cplx> x_msg = random_msg(slot_count), y_msg = random_msg(slot_count);
  PhantomPlaintext x_plain, y_plain;
  encoder.encode(context, x_msg, scale, x_plain);
  encoder.encode(context, y_msg, scale, y_plain);
  PhantomCiphertext x_cipher, y_cipher;
  public_key.encrypt_asymmetric(context, x_plain, x_cipher);
  public_key.encrypt_asymmetric(context, y_plain, y_cipher);
  // Compute x*y*x (3_ckks.cu:538-549)
  PhantomCiphertext xy_cipher = multiply(context, x_cipher, y_cipher);
  relinearize_inplace(context, xy_cipher, relin_keys);
  rescale_to_next_inplace(context, xy_cipher);
  xy_cipher.set_scale(scale);
  mod_switch_to_next_inplace(context, x_cipher);
  PhantomCiphertext x2y_cipher = multiply(context, xy_cipher, x_cipher);
  relinearize_inplace(context, x2y_cipher, relin_keys);
  rescale_to_next_inplace(context, x2y_cipher);
  PhantomPlaintext x2y_plain = secret_key.decrypt(context, x2y_cipher);
  auto result = encoder.decode<cplx>(context, x2y_plain);
  bool correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], x_msg[i] * (x_msg[i] * y_msg[i]));
  require(correctness, "Homomorphic multiplication error");
}

static void example_ckks_rotation(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomGaloisKeyFused fused_keys = secret_key.EvalRotateKeyGen(context, {1, 11, 15, 35});
  const int step = 35;
  PhantomCKKSEncoder encoder(context);
  const size_t slot_count = encoder.slot_count();
  std::vector<cplx> x_msg = random_msg(slot_count), result;
  PhantomPlaintext x_plain, x_rot_plain;
  encoder.encode(context, x_msg, scale, x_plain);
  PhantomCiphertext x_cipher;
  public_key.encrypt_asymmetric(context, x_plain, x_cipher);
  PhantomCiphertext x_cipher_rot;
  EvalRotateFused(context, fused_keys, x_cipher, x_cipher_rot, step);
  secret_key.decrypt(context, x_cipher_rot, x_rot_plain);
  encoder.decode(context, x_rot_plain, result);
  bool correctness = true;
  for (size_t i = 0; i < slot_count; i++) correctness &= eq(result[i], x_msg[(i + step) % slot_count]);
  require(correctness, "Homomorphic rotation error");

  x_msg = random_msg(slot_count);
  PhantomPlaintext x_conj_plain;
  encoder.encode(context, x_msg, scale, x_plain);
  public_key.encrypt_asymmetric(context, x_plain, x_cipher);
  PhantomCiphertext x_cipher_conj;
  EvalConjFused(context, fused_keys, x_cipher, x_cipher_conj);
  secret_key.decrypt(context, x_cipher_conj, x_conj_plain);
  encoder.decode(context, x_conj_plain, result);
  correctness = true;
  // the reference compares real parts only; the imaginary parts are checked here as well
  for (size_t i = 0; i < slot_count; i++)
    correctness &= eq(result[i], std::conj(x_msg[i])) && std::fabs(result[i].imag() + x_msg[i].imag()) < EPSINON;
  require(correctness, "Homomorphic conjugate error");
}

// the rest of include/evaluate.cuh's CKKS surface (round 3): add_many, add/sub_plain, the squaring
// branch of multiply (bit-identical to the product of two copies), multiply_and_relin, plaintext
// mod_switch_to(_next), hoisting_inplace, rotations composed from their non-adjacent form, and the
// seed-compressed save's validity after in-place operations; each decrypted with the 1e-3 rule
static void example_ckks_api(PhantomContext& context, double scale) {
  PhantomSecretKey secret_key(context);
  PhantomCKKSEncoder encoder(context);
  const size_t slots = encoder.slot_count(), n = context.poly_degree();
  std::vector<cplx> a = random_msg(slots), b = random_msg(slots), c = random_msg(slots), out;
  PhantomPlaintext pa, pb, pc;
  encoder.encode(context, a, scale, pa);
  encoder.encode(context, b, scale, pb);
  encoder.encode(context, c, scale, pc);
  PhantomCiphertext ca = secret_key.encrypt_symmetric(context, pa), cb = secret_key.encrypt_symmetric(context, pb),
                    cc = secret_key.encrypt_symmetric(context, pc);
  auto check = [&](const PhantomCiphertext& ct, const std::vector<cplx>& want, const char* what) {
    PhantomPlaintext p = secret_key.decrypt(context, ct);
    encoder.decode(context, p, out);
    for (size_t i = 0; i < want.size(); ++i)
      if (!eq(out[i], want[i]) || std::fabs(out[i].imag() - want[i].imag()) >= EPSINON) throw std::logic_error(what);
  };
  // add_many
  std::vector<PhantomCiphertext> many = {ca, cb, cc};
  PhantomCiphertext sum;
  add_many(context, many, sum);
  std::vector<cplx> want(slots);
  for (size_t i = 0; i < slots; ++i) want[i] = a[i] + b[i] + c[i];
  check(sum, want, "add_many error");
  // add_plain / sub_plain
  PhantomCiphertext t = sub_plain(context, add_plain(context, ca, pb), pc);
  for (size_t i = 0; i < slots; ++i) want[i] = a[i] + b[i] - c[i];
  check(t, want, "add_plain / sub_plain error");
  // squaring kernel == product of two copies, bit for bit; then relinearize + rescale
  PhantomCiphertext sq = ca;
  multiply_inplace(context, sq, sq);
  PhantomCiphertext copy = ca;
  PhantomCiphertext prod = multiply(context, ca, copy);
  require(sq.to_host(context.stream()) == prod.to_host(context.stream()), "square differs from the product");
  PhantomRelinKey relin_key = secret_key.gen_relinkey(context);
  PhantomCiphertext ab = multiply_and_relin(context, ca, cb, relin_key);
  rescale_to_next_inplace(context, ab);
  for (size_t i = 0; i < slots; ++i) want[i] = a[i] * b[i];
  check(ab, want, "multiply_and_relin error");
  PhantomCiphertext a2 = multiply_and_relin(context, ca, ca, relin_key);
  rescale_to_next_inplace(context, a2);
  for (size_t i = 0; i < slots; ++i) want[i] = a[i] * a[i];
  check(a2, want, "multiply_and_relin (square) error");
  // plaintext modulus switching: c at the product's level times the product
  PhantomPlaintext pc1 = mod_switch_to_next(context, pc);
  require(pc1.chain_index() == ab.chain_index() && pc1.coeff_modulus_size() == ab.coeff_modulus_size(),
          "plaintext mod_switch_to_next level");
  PhantomPlaintext pc3 = mod_switch_to(context, pc, pc.chain_index() + 3);
  require(pc3.chain_index() == pc.chain_index() + 3, "plaintext mod_switch_to level");
  PhantomCiphertext abc = ab;
  pc1.set_scale(ab.scale());
  add_plain_inplace(context, abc, pc1);
  for (size_t i = 0; i < slots; ++i) want[i] = a[i] * b[i] + c[i] * (scale / ab.scale());
  check(abc, want, "plaintext mod_switch add error");
  bool threw = false;
  try {
    PhantomPlaintext top = pc;
    mod_switch_to_inplace(context, top, 0);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  require(threw, "plaintext mod_switch_to a higher level must throw");
  // rotations: hoisting over {1, 2}, and a rotation by 3 composed from its NAF {-1, 4}
  std::vector<uint32_t> elts;
  for (int st : {1, 2, 4, -1}) elts.push_back(galois_elt_from_step(st, n));
  PhantomGaloisKey galois_keys = secret_key.create_galois_keys(context, elts);
  PhantomCiphertext h = hoisting(context, ca, galois_keys, {1, 2});
  for (size_t i = 0; i < slots; ++i) want[i] = a[(i + 1) % slots] + a[(i + 2) % slots];
  check(h, want, "hoisting error");
  PhantomCiphertext r3 = rotate(context, ca, 3, galois_keys);
  for (size_t i = 0; i < slots; ++i) want[i] = a[(i + 3) % slots];
  check(r3, want, "rotation by 3 (NAF) error");
  threw = false;
  try {
    PhantomCiphertext r8 = rotate(context, ca, 8, galois_keys);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  require(threw, "a missing power-of-two key must throw");
  // seed-compressed save after in-place operations: add_plain keeps c1 (the seed stays valid),
  // a rotation or multiply_plain rewrites it (save_symmetric must refuse)
  {
    PhantomCiphertext s1 = ca;
    add_plain_inplace(context, s1, pb);
    std::stringstream ss;
    s1.save_symmetric(ss);
    PhantomCiphertext l1;
    l1.load_symmetric(context, ss);
    for (size_t i = 0; i < slots; ++i) want[i] = a[i] + b[i];
    check(l1, want, "seed-compressed save after add_plain");
    for (int op = 0; op < 2; ++op) {
      PhantomCiphertext s2 = ca;
      if (op == 0) rotate_inplace(context, s2, 1, galois_keys);
      else multiply_plain_inplace(context, s2, pb);
      threw = false;
      try {
        std::stringstream s3;
        s2.save_symmetric(s3);
      } catch (const std::runtime_error&) {
        threw = true;
      }
      require(threw, op == 0 ? "save_symmetric after a rotation must throw" : "save_symmetric after multiply_plain must throw");
    }
  }
  // keys regenerated from one seed: same secret, independent encryption randomness
  {
    uint8_t seed[32];
    for (int i = 0; i < 32; ++i) seed[i] = static_cast<uint8_t>(7 * i + 1);
    PhantomSecretKey k1 = PhantomSecretKey::from_seed(context, seed), k2 = PhantomSecretKey::from_seed(context, seed);
    require(k1.coefficients() == k2.coefficients(), "from_seed keys differ");
    PhantomCiphertext e1 = k1.encrypt_symmetric(context, pa), e2 = k2.encrypt_symmetric(context, pa);
    const std::vector<uint64_t> h1 = e1.to_host(context.stream()), h2 = e2.to_host(context.stream());
    const size_t half = h1.size() / 2;
    require(!std::equal(h1.begin() + half, h1.end(), h2.begin() + half), "from_seed replicas share encryption randomness");
    PhantomPlaintext d = k2.decrypt(context, e1);
    encoder.decode(context, d, out);
    for (size_t i = 0; i < slots; ++i) require(eq(out[i], a[i]), "from_seed replica cannot decrypt");
  }
}

static void example_ckks_small_param() {
  EncryptionParameters parms(scheme_type::ckks);
  const size_t N = 1 << 13;
  parms.set_poly_modulus_degree(N);
  parms.set_special_modulus_size(1);
  parms.set_coeff_modulus(CoeffModulus::Create(N, {60, 40, 60}));
  parms.set_galois_elts({1});
  PhantomContext context(parms);
  PhantomCKKSEncoder encoder(context);
  PhantomSecretKey secret_key(context);
  PhantomPublicKey public_key = secret_key.gen_publickey(context);
  PhantomRelinKey relin_key = secret_key.gen_relinkey(context);
  PhantomGaloisKey galois_keys = secret_key.create_galois_keys(context);
  std::vector<double> output, input(encoder.slot_count(), 1.0);
  PhantomPlaintext plain;
  PhantomCiphertext cipher;
  encoder.encode(context, input, std::pow(2.0, 40), plain);
  public_key.encrypt_asymmetric(context, plain, cipher);
  apply_galois_inplace(context, cipher, 1, galois_keys);
  secret_key.decrypt(context, cipher, plain);
  encoder.decode(context, plain, output);
  for (int i = 0; i < 10; i++)
    if (!eq(input[i], output[i])) throw std::logic_error("error in example_ckks_small_param");
}

// PhantomGaloisKey::save / load in the reference's bytes (include/secretkey.h:195-220): the
// context's default element list (get_elts_all: 2N - 1, then 5^(2^i), 5^(-2^i)), each key a relin
// key record (dnum, then dnum key-level ciphertexts); parsed back field by field, reloaded, and a
// rotation with the reloaded keys decrypts
static void example_ckks_galois_key_layout() {
  EncryptionParameters parms(scheme_type::ckks);
  const size_t N = 1 << 12;
  parms.set_poly_modulus_degree(N);
  parms.set_special_modulus_size(2);
  parms.set_coeff_modulus(CoeffModulus::Create(N, {60, 40, 40, 60, 60}));
  PhantomContext context(parms);
  PhantomSecretKey secret_key(context);
  PhantomCKKSEncoder encoder(context);
  PhantomGaloisKey gk = secret_key.create_galois_keys(context);
  const std::vector<uint32_t> elts = context.key_galois_elts();
  require(elts.size() == 1 + 2 * 11 && elts[0] == 2 * N - 1 && elts[1] == 5 && elts[3] == 25, "default element list");
  std::stringstream ss;
  gk.save(context, ss);
  const std::string bytes = ss.str();
  const size_t QP = 5, dnum = 2, ct_bytes = 58 + 2 * QP * N * 8;
  require(bytes.size() == 8 + elts.size() * (8 + dnum * ct_bytes), "Galois key byte count");
  auto u64_at = [&](size_t off) {
    uint64_t v;
    std::memcpy(&v, bytes.data() + off, 8);
    return v;
  };
  require(u64_at(0) == elts.size(), "Galois key count field");
  for (size_t k = 0; k < elts.size(); ++k) {
    const size_t base = 8 + k * (8 + dnum * ct_bytes);
    require(u64_at(base) == dnum, "relin key dnum field");
    for (size_t d = 0; d < dnum; ++d) {
      const size_t h = base + 8 + d * ct_bytes;
      require(u64_at(h) == 0 && u64_at(h + 8) == 2 && u64_at(h + 16) == N && u64_at(h + 24) == QP,
              "key digit header (chain 0, size 2, N, size_QP)");
      std::vector<uint64_t> dev(2 * QP * N);
      PHX_CHECK(hipMemcpy(dev.data(), gk.get(elts[k]).digit(d), dev.size() * 8, hipMemcpyDeviceToHost));
      require(std::memcmp(dev.data(), bytes.data() + h + 58, dev.size() * 8) == 0, "key digit words");
    }
  }
  PhantomGaloisKey loaded;
  try {
    loaded.load(context, ss);
  } catch (const std::exception& e) {
    throw std::logic_error(std::string("reference-layout reload: ") + e.what());
  }
  std::vector<cplx> x = random_msg(encoder.slot_count()), out;
  PhantomPlaintext p;
  encoder.encode(context, x, std::pow(2.0, 40), p);
  PhantomCiphertext c = secret_key.encrypt_symmetric(context, p);
  rotate_inplace(context, c, 2, loaded);
  secret_key.decrypt(context, c, p);
  encoder.decode(context, p, out);
  for (size_t i = 0; i < x.size(); ++i) require(eq(out[i], x[(i + 2) % x.size()]), "rotation with reloaded Galois keys");
  // a key set without the context's list cannot be written in the reference's format
  PhantomGaloisKey partial = secret_key.create_galois_keys(context, {5});
  bool threw = false;
  try {
    std::stringstream t;
    partial.save(context, t);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  require(threw, "save of a partial key set must throw");
  // ... and so can a set with a key outside the list (save_with_elements names it)
  PhantomGaloisKey extra = secret_key.create_galois_keys(context);
  extra.merge(secret_key.create_galois_keys(context, {125 * 125 % (2 * N)}));
  threw = false;
  try {
    std::stringstream t;
    extra.save(context, t);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  require(threw, "save of a key outside the context's list must throw");
  // a file of the round-3 build (keys in ascending element order, then the element list: the
  // save_with_elements layout) loads through load() with every key on its own element, and the
  // stream is left after the element list
  {
    std::stringstream legacy;
    gk.save_with_elements(context, legacy);
    const uint64_t marker = 0x5EEDC0DEull;
    legacy.write(reinterpret_cast<const char*>(&marker), sizeof(marker));
    PhantomGaloisKey l2;
    try {
      l2.load(context, legacy);
    } catch (const std::exception& e) {
      throw std::logic_error(std::string("legacy reload: ") + e.what());
    }
    uint64_t after = 0;
    legacy.read(reinterpret_cast<char*>(&after), sizeof(after));
    require(legacy && after == marker, "legacy Galois key stream consumed exactly");
    for (uint32_t e : elts) {
      std::vector<uint64_t> a(2 * QP * N), b(2 * QP * N);
      PHX_CHECK(hipMemcpy(a.data(), gk.get(e).digit(0), a.size() * 8, hipMemcpyDeviceToHost));
      PHX_CHECK(hipMemcpy(b.data(), l2.get(e).digit(0), b.size() * 8, hipMemcpyDeviceToHost));
      require(a == b, "legacy Galois key bound to its own element");
    }
    // the reference layout followed by other data is not mistaken for the legacy one
    std::stringstream ref;
    gk.save(context, ref);
    ref.write(reinterpret_cast<const char*>(&marker), sizeof(marker));
    PhantomGaloisKey l3;
    try {
      l3.load(context, ref);
    } catch (const std::exception& e) {
      throw std::logic_error(std::string("reference reload with trailing data: ") + e.what());
    }
    after = 0;
    ref.read(reinterpret_cast<char*>(&after), sizeof(after));
    require(ref && after == marker, "reference Galois key stream leaves the following data");
  }
}

// 3_ckks.cu:761-818
static EncryptionParameters params_for(int alpha, double& scale) {
  EncryptionParameters parms(scheme_type::ckks);
  size_t poly_modulus_degree = size_t(1) << 15;
  scale = std::pow(2.0, 40);
  std::vector<int> bits;
  switch (alpha) {
    case 1: bits = {60}; bits.insert(bits.end(), 18, 40); bits.push_back(60); break;
    case 2: bits = {60}; bits.insert(bits.end(), 15, 40); bits.insert(bits.end(), 2, 60); break;
    case 3: bits = {60}; bits.insert(bits.end(), 14, 40); bits.insert(bits.end(), 3, 60); break;
    case 4: bits = {60}; bits.insert(bits.end(), 11, 40); bits.insert(bits.end(), 4, 60); break;
    case 15:
      poly_modulus_degree = size_t(1) << 16;
      bits = {60};
      bits.insert(bits.end(), 44, 50);
      bits.insert(bits.end(), 15, 60);
      scale = std::pow(2.0, 50);
      break;
    default: throw std::invalid_argument("unsupported alpha params");
  }
  parms.set_poly_modulus_degree(poly_modulus_degree);
  parms.set_coeff_modulus(CoeffModulus::Create(poly_modulus_degree, bits));
  parms.set_special_modulus_size(static_cast<size_t>(alpha));
  return parms;
}

int main(int argc, char** argv) {
  std::vector<int> alphas;
  uint64_t seed = 1;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--seed") && i + 1 < argc) seed = std::strtoull(argv[++i], nullptr, 0);
    else alphas.push_back(std::atoi(argv[i]));
  }
  if (alphas.empty()) alphas = {15};
  g_rng.seed(seed);
  bool all = true;
  auto run = [&](const char* name, int alpha, auto&& fn) {
    bool ok = true;
    std::string err;
    try {
      fn();
    } catch (const std::exception& e) {
      ok = false;
      err = e.what();
    }
    all &= ok;
    std::printf("{\"example\": \"%s\", \"alpha\": %d, \"ok\": %s, \"error\": \"%s\"}\n", name, alpha,
                ok ? "true" : "false", err.c_str());
    std::fflush(stdout);
  };
  for (int alpha : alphas) {
    double scale = 0;
    EncryptionParameters parms = params_for(alpha, scale);
    PhantomContext context(parms);
    run("ckks_enc", alpha, [&] { example_ckks_enc(context, scale); });
    run("ckks_add", alpha, [&] { example_ckks_add(context, scale); });
    run("ckks_save_symmetric", alpha, [&] { example_ckks_save_symmetric(context, scale); });
    run("ckks_mul_plain", alpha, [&] { example_ckks_mul_plain(context, scale); });
    run("ckks_mul", alpha, [&] { example_ckks_mul(context, scale); });
    run("ckks_rotation", alpha, [&] { example_ckks_rotation(context, scale); });
    run("ckks_api", alpha, [&] { example_ckks_api(context, scale); });
  }
  run("ckks_small_param", 1, [&] { example_ckks_small_param(); });
  run("ckks_galois_key_layout", 2, [&] { example_ckks_galois_key_layout(); });
  std::printf("{\"done\": \"ckks_example\", \"ok\": %s}\n", all ? "true" : "false");
  return all ? 0 : 1;
}
