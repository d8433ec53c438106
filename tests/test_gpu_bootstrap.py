"""CKKS bootstrapping on the GPU through the C++ façade (examples/bootstrapping_example.cpp, the
reference's bootstrapping/bootstrapping_example.cu SimpleBootstrapExample parameters:
N = 2^16, Q = {60, 29 x 59}, P = 10 x 60, levelBudget {2, 2}, scale 2^59, 2^15 reals in [1, 5]).

Parity for bootstrapping is by decrypted precision, not bits (the reference's
encoder and plaintext precompute are FP64 and order-sensitive); the reference example prints the
average bit precision with the formula reproduced in the example.  The pieces underneath (NTT,
key switching, rescale, automorphism, ModRaise lift) are bit-exact against the oracle in
test_gpu_ntt.py / test_gpu_ckks.py."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "bootstrapping_example")


def _run(*args, timeout=110):
    out = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{") and '"sample"' not in l]
    return out.returncode, lines, out.stderr[-2000:]


def test_ckks_ops_hoisted_rotation_conjugation_rescale():
    rc, lines, err = _run("ops", "16")
    checks = {l["check"]: l for l in lines if "check" in l}
    assert rc == 0, (lines, err)
    for name in ["encrypt_decrypt", "rotate_1", "rotate_-3", "conjugate", "square_rescale", "add_auto_levels",
                 "monomial_i", "drain_const_mult", "save_load"]:
        assert checks[name]["ok"], checks[name]


def test_full_bootstrap_precision_and_levels():
    rc, lines, err = _run("boot", "16", "1", timeout=115)
    assert rc == 0, (lines, err)
    boot = [l for l in lines if l.get("stage") == "bootstrap"][0]
    # correction factor 7, inputs in [1, 5]: 10.0-10.08 measured on MI355X (profiles/r01/, r02/)
    assert boot["avg_bits"] > 9.85, boot
    # the reference's layout: levelsAvailableAfterBootstrap = 11 (bootstrapping_example.cu:81)
    assert boot["levels_after"] == 11, boot


def test_deferred_setup_reference_arguments():
    """EvalBootstrapSetup with the reference's argument list (bootstrap.cu:15-18): a
    scalingFactorsRealBig that is not sf^2 is refused; precompute = false keeps the level structure
    (the keys are generated from it) and the first EvalBootstrap encodes the plaintexts."""
    rc, lines, err = _run("deferred", "16", "1", timeout=115)
    assert rc == 0, (lines, err)
    checks = {l["check"]: l for l in lines if "check" in l}
    for name in ["sf_big_mismatch_refused", "deferred_not_encoded", "sf_big_kept", "deferred_encoded_by_bootstrap"]:
        assert checks[name]["ok"], checks[name]
    setup = [l for l in lines if l.get("stage") == "setup"][0]
    assert setup["setup_ms"] < 1000, setup  # structure only: 0.44 s measured (a full setup takes 1.2-1.5 s)
    boot = [l for l in lines if l.get("stage") == "bootstrap"][0]
    assert boot["avg_bits"] > 9.85 and boot["levels_after"] == 11, boot


def test_flexibleauto_surface():
    """EvalMultAuto / EvalSquare / EvalAddAuto / EvalSubAuto / EvalAddConst / EvalMultConst (lazy) /
    EvalMultAutoInplace with a plaintext / EvalChebyshevFunction (degree 4: the reference's linear
    method; degree 30: the reference's Paterson-Stockmeyer), each decrypted against the plaintext
    computation."""
    rc, lines, err = _run("flex", "16")
    checks = {l["check"]: l for l in lines if "check" in l}
    assert rc == 0, (lines, err)
    for name in ["flex_mult_auto", "flex_square", "flex_degrees", "flex_add_auto_degree", "flex_add_auto_levels",
                 "flex_sub_auto_levels", "flex_add_const", "flex_add_const_degree2", "flex_mult_const_lazy",
                 "flex_mult_plain_auto", "flex_chebyshev_linear", "flex_chebyshev_ps"]:
        assert checks[name]["ok"], checks[name]
    used = {l["chebyshev_degree"]: l["levels_used"] for l in lines if "chebyshev_degree" in l}
    assert used[30] == 7, used  # GetDepthByDegree(30) = 7 on [1, 5] (src/util.cu:44-58)


def test_reference_precompute_evaluate_api():
    """The reference-signature FHECKKSRNS surface (include/bootstrap.cuh:116-175) at N = 2^12:
    FindBootstrapRotationIndices equals the keys the setup generates; EvalCoeffsToSlotsPrecompute /
    EvalSlotsToCoeffsPrecompute from ksiPows + rotGroup (bootstrap.cu:92-107) with lEnc / lDec, then
    EvalCoeffsToSlots(A, ...) / EvalSlotsToCoeffs(A, ...) round-trip the message (and CoeffToSlot's
    slots carry its energy, Parseval); GetMultKey / GetGaloisKey; a dense 2048 x 2048
    EvalLinearTransformPrecompute + EvalLinearTransform against the host product; the evaluator's
    KeySwitchDownFirstElement (== c0 of KeySwitchDown, bit for bit), EvalAddExt and EvalMultExt."""
    rc, lines, err = _run("refapi", "12")
    checks = {l["check"]: l for l in lines if "check" in l}
    assert rc == 0, (lines, err)
    for name in ["refapi_rotation_indices", "refapi_get_keys", "refapi_cts_stc_roundtrip", "refapi_cts_parseval",
                 "refapi_add_ext_keyswitch_down", "refapi_keyswitch_down_first_element", "refapi_mult_ext",
                 "refapi_linear_transform", "refapi_rekey_bootstrap", "refapi_muladd_batch_bitexact"]:
        assert checks[name]["ok"], checks[name]


def test_bootstrapping_example_verbatim():
    """bootstrapping_example.cu:69-198 compiled unchanged (cudaSetDevice -> hipSetDevice):
    OS-entropy keys, public-key encryption, the bare 25 x EvalMultConstInplace(x, 1) drain and
    EvalBootstrap of the degree-2 result; the reference's own output lines are parsed."""
    exe = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "bootstrapping_verbatim")
    out = subprocess.run([exe, "simple"], capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-2000:]
    vals = {}
    for line in out.stdout.splitlines():
        if " : " in line:
            k, v = line.rsplit(" : ", 1)
            vals[k.strip()] = v.strip()
    assert vals["Bootstrap depth"] == "30" and vals["Mod Size"] == "40", vals
    # 25 lazy const-mults = 24 rescales (chain 25, degree 2): 40 - 25 - 10 - 1
    assert vals["Before Bootstrapping"] == "4", vals
    # the reference's output chain index 19 (raise to chain 1 + depth 18): 40 - 19 - 10 - 1
    assert vals["After Bootstrapping"] == "10", vals
    # one sample with fresh keys and public-key encryption: 9.44-10.0 bits seen on MI355X; the C5
    # fresh-key tail is 8.99 over 1024 (profiles/r03/api/bench.json)
    assert float(vals["avg"]) > 9.0, vals


def test_bootstrap_batch_one_lane():
    """EvalBootstrapBatch on one lane: 8 bootstraps as two lockstep groups of four on the caller's
    stream, every output equal to EvalBootstrap of its input bit for bit."""
    rc, lines, err = _run("batch", "16", "8", "1", timeout=150)
    assert rc == 0, (lines, err)
    b = [l for l in lines if l.get("stage") == "batch"][0]
    assert b["bootstraps"] == 8 and b["lanes"] == 1 and b["min_avg_bits"] > 9.85, b
    checks = {l["check"]: l for l in lines if "check" in l}
    assert checks["batch_equals_single_bitexact"]["ok"], checks


def test_bootstrap_batch_on_stream_lanes():
    """EvalBootstrapBatch: 10 bootstraps of distinct inputs, 2 stream lanes side by side, each lane
    bootstrapping its five as lockstep groups of three and two (ceil(5 / 4) groups of near-equal
    size; C5's per-GPU path: grouped
    linear-transform levels, EvalMod on eight lanes); every output keeps the single-bootstrap precision and equals
    EvalBootstrap of its input bit for bit."""
    rc, lines, err = _run("batch", "16", "10", "2", timeout=150)
    assert rc == 0, (lines, err)
    b = [l for l in lines if l.get("stage") == "batch"][0]
    assert b["bootstraps"] == 10 and b["lanes"] == 2, b
    assert b["min_avg_bits"] > 9.85, b
    checks = {l["check"]: l for l in lines if "check" in l}
    assert checks["batch_equals_single_bitexact"]["ok"], checks


def test_bootstrap_batch_groups_of_eight():
    """EvalBootstrapBatch with group = 8 (the grouped kernels' maximum, LtGroupArgs /
    KsRotateBatchGroupArgs at 8 ciphertexts): 8 bootstraps as one lockstep group on one lane, then
    11 on 2 lanes (groups of 6 and 5). Every output equals EvalBootstrap of its input bit for bit."""
    for n, lanes in (("8", "1"), ("11", "2")):
        rc, lines, err = _run("batch", "16", n, lanes, "8", timeout=150)
        assert rc == 0, (lines, err)
        b = [l for l in lines if l.get("stage") == "batch"][0]
        assert b["bootstraps"] == int(n) and b["group"] == 8 and b["min_avg_bits"] > 9.85, b
        checks = {l["check"]: l for l in lines if "check" in l}
        assert checks["batch_equals_single_bitexact"]["ok"], checks


# ---- bootstrapping sessions through the C-ABI (include/phantom_amd.h phantom_boot_*) ------------

def _session_run(num_slots=0, iterations=1, precision=0, count=2, chain=26, lanes=2):
    import numpy as np
    import torch
    import phantom_amd as PA
    sess = PA.BootSession(bytes(range(32)), num_slots=num_slots, iterations=iterations, precision=precision)
    rng = np.random.default_rng(0xB0 + num_slots + iterations)
    vals = rng.uniform(1.0, 5.0, size=(count, sess.slots))
    sin = sess.input_bytes(chain)
    sout = sess.output_bytes()
    dev_in = torch.empty((count, sin), dtype=torch.uint8, device="cuda")
    dev_out = torch.empty((count, sout), dtype=torch.uint8, device="cuda")
    assert sess.encrypt(vals, chain, dev_in.data_ptr(), sin) == sin
    sess.run(dev_in.data_ptr(), sin, count, dev_out.data_ptr(), sout, lanes)
    torch.cuda.synchronize()
    bits = [PA.bit_precision(vals[i], sess.decrypt(dev_out[i].data_ptr(), sout)) for i in range(count)]
    # the input itself decrypts to the message (encrypt / serialize path)
    in_bits = PA.bit_precision(vals[0], sess.decrypt(dev_in[0].data_ptr(), sin))
    sess.close()
    return bits, in_bits


def test_session_full_packing_bootstrap():
    bits, in_bits = _session_run()
    assert in_bits > 30, in_bits
    assert min(bits) > 9.85, bits


def test_sparse_bootstrap_n_over_8_slots():
    """SparseBootStrapping (bootstrapping_example.cu:200-309): numSlots = N/8, the message in every
    block of N/8 slots; partial sums, one EvalMod, SlotToCoeff + the fold rotation."""
    bits, in_bits = _session_run(num_slots=(1 << 16) // 8)
    assert in_bits > 30, in_bits
    assert min(bits) > 9.85, bits


def test_two_iteration_bootstrap_gains_precision():
    """EvalBootstrap(ct, cc, 0, numIterations = 2, precision) (bootstrap.cu:856-900): the second
    bootstrap removes most of the first one's error.  Gated on the median of 5 encryptions, not on
    one sample: measured on MI355X over 48 fresh encryptions each (the encryptor draws OS entropy;
    profiles/r05/two_iter/dist_48.jsonl), one iteration 9.84-10.13 bits, median 9.99; two
    iterations at precision 8: 20.24-22.57, median 22.47, 3 of 48 below 21.5, so a median of 5
    falls below 21.5 with probability ~0.2%, while a second iteration that lost 1 bit or more
    fails it."""
    import statistics
    one, _ = _session_run(count=3)
    two, _ = _session_run(iterations=2, precision=8, count=5)
    m1, m2 = statistics.median(one), statistics.median(two)
    assert m2 > 21.5 and min(two) > 19.5 and m2 > m1 + 11.0, (one, two)


def test_session_run_grouped_matches_default():
    """phantom_boot_run_grouped: 9 bootstraps on 1 lane as 3 groups of 3 (group 4), and on 2 lanes
    with group 2 (5 per lane as 2 + 2 + 1, a single bootstrap among them; 4 as 2 + 2), each
    byte-identical to phantom_boot_run's default (group 8 on one lane: groups of 5 and 4);
    a group outside 1..8 is PHANTOM_ERR_INVALID_ARGUMENT."""
    import numpy as np
    import torch
    import phantom_amd as PA
    sess = PA.BootSession(bytes(range(32)))
    count, chain = 9, 26
    vals = np.random.default_rng(0xB8).uniform(1.0, 5.0, size=(count, sess.slots))
    sin, sout = sess.input_bytes(chain), sess.output_bytes()
    dev_in = torch.empty((count, sin), dtype=torch.uint8, device="cuda")
    assert sess.encrypt(vals, chain, dev_in.data_ptr(), sin) == sin
    outs = []
    for lanes, group in ((1, None), (1, 4), (2, 2)):
        o = torch.zeros((count, sout), dtype=torch.uint8, device="cuda")
        sess.run(dev_in.data_ptr(), sin, count, o.data_ptr(), sout, lanes, group)
        torch.cuda.synchronize()
        outs.append(o.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    dev_out = outs[0].cuda()
    bits = [PA.bit_precision(vals[i], sess.decrypt(dev_out[i].data_ptr(), sout)) for i in range(2)]
    assert min(bits) > 9.85, bits
    with pytest.raises(PA.PhantomError):
        sess.run(dev_in.data_ptr(), sin, 1, dev_out.data_ptr(), sout, 1, 9)
    sess.close()


def test_bench_c5_leg_single_gpu():
    """bench.py's C5 leg at world size 1 with a small batch: encrypt on rank 0, scatter, batch
    bootstrap on lanes, gather, decrypt-check every result."""
    import json
    import sys
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-c3",
                          "--no-c4", "--no-cpu-baseline", "--c5-batch", "8", "--c5-lanes", "4",
                          "--c5-key-seed", bytes(range(32)).hex()],
                         capture_output=True, text=True, timeout=115)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    c5 = line["c5"]
    assert c5["bootstraps"] == 8 and c5["verified"] == 8 and c5["ranks"] == 1, c5
    # per-ciphertext precision depends on the key and the encryption noise: over 1,024 bootstraps
    # with fresh keys the mean is 10.0 bits and the minimum 9.2-9.5 (profiles/r02/); the keys here
    # are fixed, so the bound is reproducible
    assert c5["mean_avg_bits"] > 9.85 and c5["min_avg_bits"] > 9.0, c5
