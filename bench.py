#!/usr/bin/env python3
"""bench.py — headline benchmark: forward + inverse negacyclic NTT, N = 2^16, L = 44 limbs
(BASELINE.json configs[1]; limbs 0..43 of the examples/3_ckks.cu:796-803 chain).

One step = forward NTT followed by inverse NTT of one [44][65536] uint64 batch that is
already resident in HBM.  Each step uses the next buffer of a ring whose total size
(> 256 MiB) exceeds the Infinity Cache, so every forward transform reads its input from HBM.
The steps' batches are independent and are dealt round-robin to --c2-streams HIP streams (3), so
the transforms of one batch fill another's launch ramp and store tail; `single_stream` reports
the same steps on one stream.
value = algorithmic bytes (16 B per coefficient per transform, the convention of the
reference's benchmark/ntt_bench.cu:96-97) of all steps on all ranks / max-over-ranks time.

Multi-GPU: one process per GPU (`--gpus N` without a launcher spawns the N ranks itself); each
rank transforms its own independent batches (weak scaling, no data-path collective: ciphertext
limbs are independent).  The C5 leg scatters one fixed batch of bootstraps over the
ranks and gathers the results (strong scaling of that batch, RCCL over xGMI).

roofline: the forward transform (column pass + row pass kernels) timed with HIP events on
the stream the kernels run on; achieved = 46,137,344 B / average forward duration.
cpu_baseline: the oracle's scalar C restatement (oracle/liboracle.so) on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

N = 1 << 16
L = 44
C3_BITS = [60] + [50] * 44 + [60] * 15
BYTES_PER_TRANSFORM = 16 * N * L  # 46,137,344
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
RING_BYTES = 512 << 20  # > 2 x the 256 MiB Infinity Cache: a buffer is cold again when the ring comes back to it
FWD_LAUNCHES = 200  # forward launches behind the roofline's fwd_ms (independent of --steps)
TWO_PASS_FLOOR_US = 17.5  # two read+write passes over the [44][65536] batch, no arithmetic


def _oracle_ntt_rate(O, mods, threads, seconds):
    plan = O.lib().or_ntt_plan_create(N, L, O.P(O.arr(mods)))
    a = O.random_limbs(np.random.default_rng(0x5EED), N, mods)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.lib().or_ntt_plan_fwd(plan, O.P(a), L, threads)
        O.lib().or_ntt_plan_inv(plan, O.P(a), L, threads)
        steps += 1
    dt = time.perf_counter() - t0
    O.lib().or_ntt_plan_destroy(plan)
    return 2 * BYTES_PER_TRANSFORM * steps / dt / 1e9, steps, dt


def cpu_baseline(mods, seconds=8.0):
    """The oracle's C NTT (the reference has no CPU path), forward + inverse of the
    same [44][65536] batch on the host, OpenMP over limbs with the host's CPU share (at most 16
    threads, the GPU box's share per GPU), and the same on 1 thread for reference."""
    import oracle_lib as O
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    threads = max(1, min(16, share, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    v, steps, dt = _oracle_ntt_rate(O, mods, threads, seconds)
    v1, steps1, dt1 = _oracle_ntt_rate(O, mods, 1, seconds)
    return {
        "value": round(v, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{steps} steps of fwd+inv NTT on one [44][65536] batch, C oracle, {threads} OpenMP threads, {dt:.1f}s",
        "single_core": {"value": round(v1, 3), "cores": 1, "sample": f"{steps1} steps, {dt1:.1f}s"},
    }


C3_BYTES = (4 * 45 + 3 * 2 * 60 + 2 * 44) * N * 8  # 329,252,864 B


def c3_leg(PA, lib, torch, steps=20, warmup=3):
    """Config C3: HE multiply + relinearize + rescale at N=2^16, Q = {60, 44x50},
    P = 15x60 (dnum 3), ciphertexts at chain index 1 (45 limbs), uniform random ciphertexts and
    key digits (parity of these ops is bit-exact, tests/test_gpu_ckks.py).
    total_ms: `steps` back-to-back multiply -> relinearize -> rescale sequences between one pair of
    HIP events on the stream the kernels run on, per sequence.  ms: each op alone, `steps` calls back
    to back between one event pair, per call.  (An event pair around every op adds ~10 us of event
    processing to each op on the device timeline: rocprofv3 traces of that form show a ~10 us idle
    gap at every op boundary and none inside an op, profiles/r05/c3/.)"""
    mods = PA.coeff_modulus_create(N, C3_BITS)
    ctx = PA.Context(N, mods, 15)
    ql = mods[:45]
    rng = np.random.default_rng(0xC3)

    def rand_limbs(ms, polys=1):
        a = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for _ in range(polys) for q in ms])
        return torch.from_numpy(a.view(np.int64)).cuda()

    ct1, ct2 = rand_limbs(ql, 2), rand_limbs(ql, 2)
    keys = [rand_limbs(mods, 2) for _ in range(3)]
    kp = PA.ptr_array([k.data_ptr() for k in keys])
    prod = torch.empty(3 * 45 * N, dtype=torch.int64, device="cuda")
    resc = torch.empty(2 * 44 * N, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    ops = {
        "multiply": lambda: lib.phantom_multiply(ctx.handle, 1, ct1.data_ptr(), ct2.data_ptr(), prod.data_ptr(), sh),
        "relinearize": lambda: lib.phantom_relinearize(ctx.handle, 1, prod.data_ptr(), kp, 3, sh),
        "rescale": lambda: lib.phantom_rescale_to_next(ctx.handle, 1, prod.data_ptr(), resc.data_ptr(), 2, sh),
    }
    for _ in range(warmup):
        for f in ops.values():
            PA.check(f())
    torch.cuda.synchronize()

    def timed(fns):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(steps):
            for f in fns:
                PA.check(f())
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / steps

    total = timed(list(ops.values()))
    ms = {k: timed([f]) for k, f in ops.items()}
    ctx.close()
    achieved = C3_BYTES / (total * 1e-3) / 1e9
    return {
        "workload": "C3: multiply + relinearize + rescale_to_next, N=65536, 45->44 limbs, P=15, dnum=3",
        "ms": {k: round(v, 4) for k, v in ms.items()},
        "total_ms": round(total, 4),
        "sum_of_ops_ms": round(sum(ms.values()), 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes": C3_BYTES},
    }


# ---- the reference's bootstrap schedule, from its own parameter functions (util.cu) ------------
def select_layers(log_slots, budget):
    """SelectLayers (src/util.cu:733-763): {layers, rows, rem}."""
    import math
    layers = math.ceil(log_slots / budget)
    rows, rem = log_slots // layers, log_slots % layers
    dim = rows + (1 if rem else 0)
    if dim < budget:
        layers -= 1
        rows = log_slots // layers
        rem = log_slots - rows * layers
        dim = rows + (1 if rem else 0)
        while dim != budget:
            rows -= 1
            rem = log_slots - rows * layers
            dim = rows + (1 if rem else 0)
    return layers, rows, rem


def collapsed_fft_params(slots, budget):
    """GetCollapsedFFTParams (src/util.cu:765-816) with dim1 = 0: (layers, rem, rotations, b, g,
    rotations_rem, b_rem, g_rem); g baby steps, b giant steps per level."""
    log_slots = max(1, slots.bit_length() - 1)
    layers, _, rem = select_layers(log_slots, budget)
    rot = (1 << (layers + 1)) - 1
    rot_rem = (1 << (rem + 1)) - 1
    g = 1 << (layers // 2 + (2 if rot > 7 else 1))
    b = (rot + 1) // g
    g_rem = b_rem = 0
    if rem:
        g_rem = 1 << (rem // 2 + (2 if rot_rem > 7 else 1))
        b_rem = (rot_rem + 1) // g_rem
    return layers, rem, rot, b, g, rot_rem, b_rem, g_rem


def depth_by_degree(d):
    """GetDepthByDegree (src/util.cu:44-71)."""
    for hi, depth in ((4, 3), (5, 4), (13, 5), (27, 6), (59, 7), (119, 8), (247, 9), (495, 10), (1007, 11), (2031, 12)):
        if d <= hi:
            return depth
    raise ValueError(d)


def compute_degrees_ps(n):
    """ComputeDegreesPS (src/util.cu:260-296) for n <= 2204: (k, m)."""
    for hi, m in ((2, 1), (11, 2), (13, 3), (17, 2), (55, 3), (59, 4), (76, 3), (239, 4), (247, 5), (284, 4),
                  (991, 5), (1007, 6), (1083, 5), (2015, 6), (2031, 7), (2204, 6)):
        if n <= hi:
            return n // ((1 << m) - 1) + 1, m
    raise ValueError(n)


def c4_reference_bytes(N=N, size_Q=30, size_P=10, level_budget=(2, 2), degree=88, r_double=6, input_chain=26):
    """Algorithmic bytes of one bootstrap under the REFERENCE's schedule (engine-independent: the
    denominator does not move when this engine issues more or fewer key switches), derived from the
    reference's own parameter functions (ported above) for the given parameters; the defaults are
    config C4 (bootstrapping_example.cu:69-116: N 2^16, Q = {60, 29 x 59}, P = 10 x 60, budget {2, 2},
    EvalMod degree 88, R = 6; input at chain 26 after the example's 25 EvalMultConst drains).
    Chain c holds Ql = size_Q + 1 - c limbs; a key switch reads dnum = ceil(Ql / size_P) digits x 2 x
    (Ql + size_P) limbs of key; a diagonal plaintext is Ql + size_P limbs (encode_ext).
      * linear transforms (bootstrap.cu:1157-1655): per direction, the full levels (2^(layers+1) - 1
        diagonals, g - 1 baby + b - 1 giant rotations) then the remainder level (bootstrap.cu:240-330,
        470-540); CoeffToSlot from chain 2 (lEnc = L0 - budget - 1), SlotToCoeff from chain
        1 + depthBT - budget (lDec = L0 - depthBT);
      * EvalMod: the conjugation at CoeffToSlot's output chain; two Chebyshev series by
        Paterson-Stockmeyer, k + 2m + 2^(m-1) - 4 products each (ComputeDegreesPS), priced at the
        series' middle level; R double-angle squarings per half after it;
      * ciphertext I/O: the input read at `input_chain`, the output written at 1 + depthBT.
    Returns (total, {"keys", "plaintexts", "ciphertexts"}, derivation)."""
    import math
    word = 8 * N
    slots = N // 2

    def ql(c):
        return size_Q + 1 - c

    def key(c):
        return math.ceil(ql(c) / size_P) * 2 * (ql(c) + size_P) * word

    def pt(c):
        return (ql(c) + size_P) * word

    depth_mod = depth_by_degree(degree) + r_double
    depth_bt = depth_mod + level_budget[0] + level_budget[1]
    keys = pts = 0
    levels = []
    for direction, budget, first in (("cts", level_budget[0], 2), ("stc", level_budget[1], 1 + depth_bt - level_budget[1])):
        layers, rem, rot, b, g, rot_rem, b_rem, g_rem = collapsed_fft_params(slots, budget)
        full = budget - (1 if rem else 0)
        shapes = [(rot, g, b)] * full + ([(rot_rem, g_rem, b_rem)] if rem else [])  # remainder level last
        for i, (diags, gg, bb) in enumerate(shapes):
            c = first + i
            keys += (gg - 1 + bb - 1) * key(c)
            pts += diags * pt(c)
            levels.append({"dir": direction, "chain": c, "diagonals": diags, "g": gg, "b": bb})
    k, m = compute_degrees_ps(degree)
    mults = k + 2 * m + (1 << (m - 1)) - 4
    conj_chain = 2 + level_budget[0]
    # the series consumes chains conj .. conj + depth - 1: priced at their middle, rounded down
    ps_mid = conj_chain + (depth_by_degree(degree) + 1) // 2 - 1
    keys += key(conj_chain) + 2 * mults * key(ps_mid)
    da_first = conj_chain + depth_by_degree(degree) - 1
    keys += 2 * sum(key(c) for c in range(da_first, da_first + r_double))
    out_chain = 1 + depth_bt
    cts = 2 * ql(input_chain) * word + 2 * ql(out_chain) * word
    deriv = {"levels": levels, "ps_k_m": [k, m], "ps_products_per_half": mults, "depth_bt": depth_bt,
             "output_chain": out_chain, "conj_chain": conj_chain, "ps_mid_chain": ps_mid,
             "double_angle_chains": [da_first, da_first + r_double - 1]}
    return keys + pts + cts, {"keys": keys, "plaintexts": pts, "ciphertexts": cts}, deriv


def c4_leg(iters=3, timeout=240):
    """Config C4: full CKKS bootstrap, N=2^16, Q = {60, 29x59}, P = 10x60,
    levelBudget {2,2}, 2^15 reals in [1,5] (bootstrapping_example.cu:69-116), run by the C++
    example binary in its own process; latency = median wall time of EvalBootstrap between device
    synchronisations."""
    import subprocess
    exe = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "bootstrapping_example")
    out = subprocess.run([exe, "boot", "16", str(iters)], capture_output=True, text=True, timeout=timeout)
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{") and '"sample"' not in l]
    boot = [r for r in rows if r.get("stage") == "bootstrap"]
    setup = [r for r in rows if r.get("stage") == "setup"]
    if out.returncode != 0 or not boot:
        return {"error": (out.stderr or out.stdout)[-300:]}
    b = boot[0]
    res = {
        "workload": "C4: EvalBootstrap, N=65536, Q={60,29x59}, P=10x60, levelBudget {2,2}, full packing",
        "ms_median": b["ms_median"], "ms_min": b["ms_min"], "runs": b["runs"],
        "avg_bits": b["avg_bits"], "levels_after": b["levels_after"],
        "setup_ms": setup[0]["setup_ms"] if setup else None,
        "keygen_ms": setup[0]["keygen_ms"] if setup else None,
    }
    # roofline: the reference schedule's bytes (c4_reference_bytes) over the latency; the bytes
    # this engine's own kernels stream (host/traffic.h counters) are reported beside it
    total, parts, deriv = c4_reference_bytes()
    # the derivation must describe the run it prices: the example's output chain and level count
    if deriv["output_chain"] != b.get("chain_out") or b.get("levels_after") != 30 - deriv["output_chain"]:
        return {**res, "error": f"reference schedule (output chain {deriv['output_chain']}) does not match the run {b}"}
    achieved = total / (b["ms_median"] * 1e-3) / 1e9
    res["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes": total, "bytes": parts,
                       "source": "bench.c4_reference_bytes: key + diagonal bytes of the reference's own schedule "
                                 "(SelectLayers / GetCollapsedFFTParams / ComputeDegreesPS ported) + ciphertext I/O",
                       "derivation": deriv}
    ab = b.get("alg_bytes")
    if ab:
        eng = ab["keys"] + ab["plaintexts"] + ab["ciphertexts"]
        res["engine_streamed_bytes"] = {**ab, "total": eng}
        # the same latency over the bytes this engine's kernels stream (host/traffic.h counters)
        e_ach = eng / (b["ms_median"] * 1e-3) / 1e9
        res["roofline_engine_bytes"] = {"bound": "hbm", "achieved": round(e_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": round(e_ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": eng}
    return res


def max_over_ranks(dist, values, device):
    """MAX all-reduce of per-rank timings: the slowest rank defines the job's time."""
    import torch
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def all_ranks_ok(dist, ok, device):
    """True only if every rank reports success (MIN all-reduce of a flag)."""
    import torch
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() > 0.5)


def job_throughput(units_per_rank, world, max_seconds):
    """Whole-job throughput: the units every rank processed over the max-over-ranks time."""
    return units_per_rank * world / max_seconds


def c5_shape(per, lanes=None, group=None):
    """Lanes x lockstep group for `per` bootstraps on one GPU (explicit values win).  Groups of 8
    share the most key and diagonal reads; 3 lanes fill one bootstrap's serial tails best, at 1,024
    and at the 8-GPU job's 128 per rank alike (profiles/r06/c5_share/: 128 per rank at 3 x 8 60.7-61.1/s,
    2 x 8 60.1-60.5, 4 x 8 60.6, 4 x 4 59.1).  Each lane's m ciphertexts form ceil(m / group) groups
    of near-equal size (EvalBootstrapBatch), so no lane ends on a small group; with fewer than a group
    per lane the lanes shrink instead."""
    group = 8 if group is None else group
    if lanes is None:
        lanes = max(1, min(3, -(-per // group)))
    return lanes, group


def c5_leg(dist, torch, world, rank, local_rank, total=1024, lanes=None, chain=26, verify=None, key_seed=None,
           group=None):
    """Config C5: `total` independent C4 bootstraps sharded over the ranks, one
    process per GPU.  Every rank regenerates the same keys from a 32-byte seed rank 0 broadcasts
    (no key traffic).  Rank 0 encrypts the batch — 2^15 reals in [1, 5] per ciphertext at chain
    index `chain` (the level the example's 25 EvalMultConst drains leave, bootstrapping_example.cu:
    150-153) — and the timed region is first scatter -> bootstraps (EvalBootstrapBatch, `lanes`
    side by side per GPU) -> last gather of the serialized results (RCCL over xGMI for N > 1).
    Afterwards rank 0 decrypts every gathered result (or the first `verify`) and reports the worst
    average bit precision (compute_bit_precision, bootstrapping_example.cu:17-41).
    Throughput = total / max-over-ranks time."""
    import phantom_amd as PA
    import shard
    if total % world:
        raise ValueError(f"C5 batch {total} does not divide over {world} ranks")
    per = total // world
    lanes, group = c5_shape(per, lanes, group)
    dev = torch.device("cuda", local_rank)
    # fresh OS entropy by default; a fixed seed (--c5-key-seed) makes the keys, and with them the
    # per-ciphertext precision, reproducible
    seed = bytes.fromhex(key_seed) if key_seed else shard.broadcast_seed(dist, dev)
    t_setup = time.perf_counter()
    sess = PA.BootSession(seed)
    setup_s = time.perf_counter() - t_setup
    align = 256
    in_bytes = sess.input_bytes(chain)
    out_bytes = sess.output_bytes()
    sin = (in_bytes + align - 1) // align * align
    sout = (out_bytes + align - 1) // align * align
    rng = np.random.default_rng(0xC5)
    values = rng.uniform(1.0, 5.0, size=(total if rank == 0 else 0, sess.slots))
    full = None
    if rank == 0:
        full = torch.empty((total, sin), dtype=torch.uint8, device=dev)
        sess.encrypt(values, chain, full.data_ptr(), sin)
    # warm-up on every rank (first-use allocations and code loading), untimed: one full lockstep
    # group per lane, so the grouped path's buffers are in the pool before the timed region
    warm_n = min(lanes * group, per)
    warm_in = torch.empty((warm_n, sin), dtype=torch.uint8, device=dev)
    sess.encrypt(rng.uniform(1.0, 5.0, size=(warm_n, sess.slots)), chain, warm_in.data_ptr(), sin)
    warm_out = torch.empty((warm_n, sout), dtype=torch.uint8, device=dev)
    sess.run(warm_in.data_ptr(), sin, warm_n, warm_out.data_ptr(), sout, lanes, group)
    del warm_in, warm_out
    local_out = torch.empty((per, sout), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    PA.pool_reset_peak()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    local_in = shard.scatter_rows(dist, full, per, sin, dev)
    torch.cuda.synchronize()
    sess.run(local_in.data_ptr(), sin, per, local_out.data_ptr(), sout, lanes, group)
    torch.cuda.synchronize()
    gathered = shard.gather_rows(dist, local_out, dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    max_s = max_over_ranks(dist, [elapsed], "cuda")[0]
    pool = PA.pool_stats()  # the engine's device allocator on this rank (batch buffers are torch's)
    # every rank's wall time and pool figures, so a multi-rank line shows any imbalance
    ranks = shard.gather_stats(dist, [elapsed, pool["held"] / 2**30, pool["peak_live"] / 2**30], dev)
    res = None
    if rank == 0:
        nver = total if verify is None else min(verify, total)
        bits, flat, low = [], [], 0
        for i in range(nver):
            got = np.asarray(sess.decrypt(gathered[i].data_ptr(), sout), dtype=np.float64)
            bits.append(PA.bit_precision(values[i], got))
            # the same with the error's mean over the slots removed: the bootstrap's precision tail is
            # a constant offset of every slot (coefficient 0); what is left is the rest
            flat.append(PA.bit_precision(values[i], got - np.mean(got - values[i])))
            low += bits[-1] < 9.6
        res = {
            "workload": f"C5: {total} independent C4 bootstraps (input chain index {chain}) sharded over {world} rank(s), "
                        "scatter -> EvalBootstrapBatch -> gather of serialized ciphertexts",
            "bootstraps": total, "bootstraps_per_rank": per, "lanes_per_rank": lanes, "lockstep_group": group, "ranks": world,
            "bootstraps_per_s": round(total / max_s, 3), "max_rank_s": round(max_s, 3),
            "scatter_gather_bytes": total * (sin + sout),
            "verified": nver, "min_avg_bits": round(min(bits), 2), "mean_avg_bits": round(float(np.mean(bits)), 2),
            "min_offset_free_bits": round(min(flat), 2), "below_9_6_bits": low,
            "setup_s": round(setup_s, 2), "scaling": "strong",
            "keys": "regenerated on every rank from a broadcast 32-byte seed",
            "rank0_pool_GiB": {"held": round(pool["held"] / 2**30, 2), "peak_held": round(pool["peak_held"] / 2**30, 2),
                               "peak_live": round(pool["peak_live"] / 2**30, 2)},
            "per_rank": {"wall_s": [round(r[0], 3) for r in ranks],
                         "min_wall_s": round(min(r[0] for r in ranks), 3),
                         "max_wall_s": round(max(r[0] for r in ranks), 3),
                         "pool_held_GiB": [round(r[1], 2) for r in ranks],
                         "pool_peak_live_GiB": [round(r[2], 2) for r in ranks]},
        }
        # roofline per GPU: the reference schedule's key and diagonal bytes (c4_reference_bytes) read
        # once per lockstep group (the grouped kernels share them through each XCD's L2), plus each
        # bootstrap's own ciphertext I/O, over the measured per-GPU bootstrap rate
        _, parts, _ = c4_reference_bytes(input_chain=chain)
        per_boot = (parts["keys"] + parts["plaintexts"]) / max(1, group) + parts["ciphertexts"]
        ach = per_boot * (total / max_s) / world / 1e9
        res["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_bootstrap": int(per_boot),
                           "source": "bench.c4_reference_bytes: (keys + diagonals) / lockstep group + ciphertext I/O "
                                     "per bootstrap, per GPU"}
    del full, gathered, local_out
    sess.close()
    return res


# HBM bytes per forward-NTT launch (column + row pass) from PMC counters: FETCH_SIZE and
# WRITE_SIZE collected in separate rocprofv3 --pmc passes over the same NTT shape
# (tools/gpu_pmc_traffic.sh), gfx950 FETCH_SIZE correction applied (tools/pmc_traffic.py).
PMC_TRAFFIC_FILE = "profiles/r06/c2/ntt_pmc_traffic.json"


def pmc_traffic():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), PMC_TRAFFIC_FILE)
    try:
        with open(path) as f:
            return json.load(f).get("forward_ntt_bytes_per_launch")
    except (OSError, ValueError):
        return None


# rocprofv3 kernel-trace average durations of the forward's two kernels at HEAD (bench.py's own C2
# command profiled on MI355X): fwd_ms minus their sum is the column -> row launch gap
KERNEL_SUM_SOURCE = "profiles/r06/c2/c2_fwd_kernels.json"


def _kernel_sum_ms():
    path = os.path.join(ROOT, KERNEL_SUM_SOURCE)
    try:
        with open(path) as f:
            k = json.load(f)
        return round((k["ntt_col_fwd_us"] + k["ntt_row_fwd_us"]) * 1e-3, 5)
    except (OSError, ValueError, KeyError):
        return None


KERNEL_SUM_MS = _kernel_sum_ms()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c2-streams", type=int, default=3, help="C2: HIP streams the independent batches are dealt to")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 (mult+relin+rescale) leg")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (bootstrap latency) leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (sharded bootstrap batch) leg")
    ap.add_argument("--c5-batch", type=int, default=1024, help="C5: bootstraps in the whole batch")
    ap.add_argument("--c5-lanes", type=int, default=None,
                    help="C5: stream lanes per GPU (each runs lockstep groups); default from the per-rank count (c5_shape)")
    ap.add_argument("--c5-group", type=int, default=None,
                    help="C5: at most this many bootstraps per lane in lockstep (1..8, default 8); 3 x 8 holds ~86 GiB, "
                         "4 x 8 ~107 GiB, 2 x 4 ~56 GiB (profiles/r05/c5_pool/)")
    ap.add_argument("--c5-verify", type=int, default=None, help="C5: decrypt-check only the first K results")
    ap.add_argument("--c5-key-seed", default=None, help="C5: 64 hex digits of key seed (default: OS entropy)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: become the launcher (one process per GPU), before anything touches a GPU
        import shard
        sys.exit(shard.spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import phantom_amd as PA
    lib = PA.load()
    mods = PA.coeff_modulus_create(N, C3_BITS)[:L]
    tables = PA.NttTables(N, mods)

    # the steps (independent batches) are dealt round-robin to `c2_streams` HIP streams, so one
    # batch's transforms fill the launch ramp and store tail of another's (a pass waits ~2 us for
    # its first data and drains its stores for ~3 us: profiles/r03/ntt_experiments/); a buffer of
    # the ring always stays on one stream (nbuf is a multiple of the stream count)
    K = max(1, args.c2_streams)
    nbuf = max(2, RING_BYTES // (8 * N * L) + 1)
    nbuf = -(-nbuf // K) * K
    rng = np.random.default_rng(0x5EED + rank)
    base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
    ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(nbuf)]
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    lanes = [torch.cuda.Stream() for _ in range(K)]
    for ls in lanes:
        ls.wait_stream(stream)

    def step(i, ev=None, k=None, buf=None):
        d = ring[(i if buf is None else buf) % nbuf].data_ptr()
        st = stream if k is None else lanes[i % k]
        h = st.cuda_stream
        if ev is not None:
            ev[0].record(st)
        PA.check(lib.phantom_nwt_forward_inplace(d, tables.handle, L, 0, h))
        if ev is not None:
            ev[1].record(st)
        PA.check(lib.phantom_nwt_backward_inplace(d, tables.handle, L, 0, h))

    # warm-up steps use ring buffers 0 .. W-1 and the timed steps continue from buffer W, so no timed
    # step reads a buffer an earlier step left in the Infinity Cache: the ring (> 2 x 256 MiB) comes
    # back to a buffer only after every other buffer has been read and written since
    def timed(k):
        for i in range(args.warmup):
            step(i, k=k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, k=k, buf=args.warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    elapsed = timed(K)
    elapsed_1 = timed(1) if K > 1 else elapsed  # the same steps on one stream, for reference
    for ls in lanes:
        stream.wait_stream(ls)

    # forward-NTT launch duration for the roofline: HIP events on the launch stream around
    # FWD_LAUNCHES back-to-back forward transforms over the cold buffer ring (average per launch;
    # rocprofv3's kernel sum col + row of the same launches misses only the col -> row launch gap),
    # and the median of single forwards bracketed by events (adds the event overhead)
    for i in range(5):
        PA.check(lib.phantom_nwt_forward_inplace(ring[i % nbuf].data_ptr(), tables.handle, L, 0, sh))
    fa, fb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fa.record(stream)
    for i in range(FWD_LAUNCHES):
        PA.check(lib.phantom_nwt_forward_inplace(ring[(5 + i) % nbuf].data_ptr(), tables.handle, L, 0, sh))
    fb.record(stream)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
    for i, ev in enumerate(events):
        step(i, ev, buf=5 + FWD_LAUNCHES + i)
    torch.cuda.synchronize()
    fwd_ms = fa.elapsed_time(fb) / FWD_LAUNCHES
    fwd_ms_isolated = float(np.median([a.elapsed_time(b) for a, b in events]))
    elapsed, elapsed_1, fwd_ms, fwd_ms_isolated = max_over_ranks(
        dist if world > 1 else None, [elapsed, elapsed_1, fwd_ms, fwd_ms_isolated], "cuda")

    c5 = None
    if not args.no_c5:
        c5 = c5_leg(dist if world > 1 else None, torch, world, rank, local_rank, total=args.c5_batch,
                    lanes=args.c5_lanes, verify=args.c5_verify, key_seed=args.c5_key_seed,
                    group=args.c5_group)

    # parity spot-check of the last buffer state is done by tests/; here just sanity
    value = job_throughput(2 * BYTES_PER_TRANSFORM * args.steps, world, elapsed) / 1e9
    value_1 = job_throughput(2 * BYTES_PER_TRANSFORM * args.steps, world, elapsed_1) / 1e9
    achieved = BYTES_PER_TRANSFORM / (fwd_ms * 1e-3) / 1e9

    if rank == 0:
        out = {
            "metric": "NTT GB/s vs HBM roofline (fwd+inv NTT, N=2^16, L=44)",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic uniform residues in [0, q_i), seed 0x5EED",
            "config": {
                "workload": "C2: forward+inverse negacyclic NTT, N=65536, 44 RNS limbs of the 3_ckks.cu C3 chain",
                "poly_modulus_degree": N,
                "limbs": L,
                "batch_per_rank": 1,
                "buffer_ring": nbuf,
                "streams_per_rank": K,
                "parallelism": f"replicas x{world} (independent batches per rank, dealt to {K} HIP streams)",
            },
            # the same steps on one stream (no overlap of independent batches): the per-transform rate
            "single_stream": {"value": round(value_1, 2), "ms_per_step": round(elapsed_1 / args.steps * 1e3, 5),
                              "per_transform_ms": round(elapsed_1 / args.steps * 1e3 / 2, 5)},
            "roofline": {
                "bound": "hbm",
                "kernel": "forward NTT (ntt_col_pass + ntt_row_pass)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "job_frac": round(value / world / HBM_PEAK_GBS, 4),
                "fwd_ms": round(fwd_ms, 5),
                "fwd_launches": FWD_LAUNCHES,
                "fwd_ms_isolated_median": round(fwd_ms_isolated, 5),
                "kernel_sum_ms": KERNEL_SUM_MS,
                "kernel_sum_source": KERNEL_SUM_SOURCE,
                "launch_gap_ms": round(fwd_ms - KERNEL_SUM_MS, 5) if KERNEL_SUM_MS else None,
                "traffic": pmc_traffic(),
                "traffic_source": PMC_TRAFFIC_FILE,
                # the two-pass design's own ceiling: one read + write of the batch per pass, measured as
                # a plain two-pass copy of the same tiles (17.5 us): 0.60 of 8 TB/s
                # (9.6 us per forward) is beyond any two-pass transform
                "two_pass_floor_us": TWO_PASS_FLOOR_US,
                "two_pass_floor_frac": round(BYTES_PER_TRANSFORM / (TWO_PASS_FLOOR_US * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "two_pass_floor_source": "profiles/r01/ubench_fused.txt, profiles/r02/ubench_stream.txt",
            },
        }
        if not args.no_c3:
            out["c3"] = c3_leg(PA, lib, torch)
        if not args.no_c4 and world == 1:
            out["c4"] = c4_leg()
        if c5 is not None:
            out["c5"] = c5
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(mods)
        print(json.dumps(out), flush=True)
    tables.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
