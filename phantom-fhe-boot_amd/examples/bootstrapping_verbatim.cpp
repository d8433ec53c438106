// bootstrapping_verbatim — the drop-in proof for bootstrapping/bootstrapping_example.cu: the body of
// SimpleBootstrapExample (lines 69-198) compiled unchanged against this engine's phantom:: façade.
// The only substitution is cudaSetDevice -> hipSetDevice (no CUDA names on this platform); the
// helpers of the reference's bootstrapping.h / timer.h come from examples/bootstrapping.h.  This
// includes the bare 25 x EvalMultConstInplace(x_cipher, 1) level drain (lazy rescale of a
// degree-2 input) and EvalBootstrap of the resulting degree-2 ciphertext.
//
// usage: bootstrapping_verbatim simple   (prints the reference's output; tests parse it)
#include "bootstrapping.h"

using namespace phantom;
using namespace phantom::arith;
using namespace phantom::util;

void SimpleBootstrapExample();

// bootstrapping_example.cu:17-41
double compute_bit_precision(const std::vector<double>& ref, const std::vector<double>& actual) {
    if (ref.size() != actual.size()) {
        std::cerr << "Size mismatch in compute_bit_precision!\n";
        return 0.0;
    }
    double sum_bit_precision = 0.0;
    int valid_count = 0;
    for (size_t i = 0; i < ref.size(); ++i) {
        double r = ref[i];
        double a = actual[i];
        if (std::abs(r) < 1e-20) continue;
        double rel_error = std::abs(r - a) / std::abs(r);
        if (rel_error < 1e-40) rel_error = 1e-40;
        sum_bit_precision += -std::log2(rel_error);
        ++valid_count;
    }
    return (valid_count == 0) ? 0.0 : sum_bit_precision / valid_count;
}

int main(int argc, char* argv[])
{
    if (argc < 2 || std::strcmp(argv[1], "simple") != 0)
    {
        printf("Usage: %s simple\n", argv[0]);
        return 1;
    }
    SimpleBootstrapExample();
    return 0;
}

void SimpleBootstrapExample()
{
    {
        EncryptionParameters parameters(scheme_type::ckks);

        size_t N = 1 << 16;

        int device_id = 0; // Change to the desired GPU index
        (void)hipSetDevice(device_id);

        uint32_t dcrtBits = 59;
        uint32_t firstMod = 60;
        uint32_t levelsAvailableAfterBootstrap = 11;
        std::vector<uint32_t> levelBudget = { 2, 2 };

        uint32_t depth = levelsAvailableAfterBootstrap + FHECKKSRNS::GetBootstrapDepth(levelBudget);
        std::cout << "Bootstrap depth : " << depth + 1 << std::endl;
        uint32_t numLargeDigits = ComputeNumLargeDigits(0, depth);
        (void)numLargeDigits;
        auto special_modulus_size = 10;

        std::vector<int> mod_vec = {};

        for (int i = 0; i < static_cast<int>(depth) + 1 + special_modulus_size; i++)
        {
            if (i == 0)
            {
                mod_vec.push_back(firstMod);
            }

            else
            {
                if (i < static_cast<int>(depth) + 1)
                {
                    mod_vec.push_back(dcrtBits);
                }
                else
                {
                    mod_vec.push_back(AUX_MOD);
                }
            }
        }
        std::cout << std::endl;
        std::cout << "Mod Size : " << mod_vec.size() << std::endl;

        parameters.set_poly_modulus_degree(N);
        parameters.set_special_modulus_size(special_modulus_size);
        parameters.set_coeff_modulus(CoeffModulus::Create(N, mod_vec));
        double scale = pow(2.0, 59);

        uint32_t numSlots = N / 2;
        std::cout << "CKKS scheme is using ring dimension " << N << std::endl
            << std::endl;

        Timer::startGPUTimer("Context Creation");
        PhantomContext context(parameters);
        Timer::stopGPUTimer("Context Creation");

        PhantomSecretKey secret_key(context);
        PhantomPublicKey public_key = secret_key.gen_publickey(context);

        PhantomCKKSEncoder encoder(context);

        std::vector<double> x = GenerateRandomVector(numSlots);

        size_t encodedLength = x.size();
        (void)encodedLength;

        PhantomPlaintext x_plain;
        PhantomCiphertext x_cipher;

        Timer::startGPUTimer("Encoding");
        encoder.encode(context, x, scale, x_plain);
        Timer::stopGPUTimer("Encoding");

        Timer::startGPUTimer("Encryption");
        public_key.encrypt_asymmetric(context, x_plain, x_cipher);
        Timer::stopGPUTimer("Encryption");

        x_cipher.PreComputeScale(context, scale);
        std::vector<double> m_scalingFactorsReal = x_cipher.getScalingFactorsReal();
        std::vector<double> m_scalingFactorsRealBig = x_cipher.getScalingFactorsRealBig();

        for (int i = 0; i < 25; i++)
        {
            EvalMultConstInplace(context, x_cipher, 1, m_scalingFactorsReal);
        }

        FHECKKSRNS bootstrapper(encoder);
        std::cout << "before setup"  << std::endl;

        Timer::startGPUTimer("Bootstrap Setup");
        bootstrapper.EvalBootstrapSetup(context, levelBudget, scale, m_scalingFactorsReal, m_scalingFactorsRealBig);
        Timer::stopGPUTimer("Bootstrap Setup");


        std::cout << "setup done"  << std::endl;
        Timer::startGPUTimer("Multiplication KeyGen");
        bootstrapper.EvalMultKeyGen(secret_key, context);
        Timer::stopGPUTimer("Multiplication KeyGen");

        Timer::startGPUTimer("Bootstrap KeyGen");
        bootstrapper.EvalBootstrapKeyGen(secret_key, context, numSlots);
        Timer::stopGPUTimer("Bootstrap KeyGen");

        std::cout << "Message vector: " << std::endl;
        print_vector(x, 3, 7);

        std::cout << "Before Bootstrapping : " << mod_vec.size() - x_cipher.chain_index() - special_modulus_size - 1 << std::endl;

        PhantomCiphertext result_cipher;

        Timer::startGPUTimer("Bootstrapping");
        result_cipher = bootstrapper.EvalBootstrap(x_cipher, context);
        Timer::stopGPUTimer("Bootstrapping");

        PhantomPlaintext result_plain;
        Timer::startGPUTimer("Decryption");
        result_plain = secret_key.decrypt(context, result_cipher);
        Timer::stopGPUTimer("Decryption");

        std::vector<double> result;
        encoder.decode(context, result_plain, result);
        result.resize(x.size());
        std::cout << "Result vector: " << std::endl;
        print_vector(result, 3, 7);
        std::cout << "After Bootstrapping : " << mod_vec.size() - result_cipher.chain_index() - special_modulus_size - 1 << std::endl;
        double avg_bits = compute_bit_precision(x, result);
        std::cout << "avg : " << avg_bits << std::endl;
        Timer::printAccumulatedTimes();
    }
}
