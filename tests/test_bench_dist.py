"""The N > 1 path of bench.py on CPU: two `gloo` ranks (one process each, as torchrun launches
them) aggregate per-rank timings with a MAX all-reduce, agree on success with a MIN all-reduce,
and report whole-job throughput = units of every rank / max-over-ranks time.  The C5 leg is
replicas only (no collective on the data path), so these reductions are its only communication.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r took (1 + r) s for its steps and (2 - r) ms per forward transform
        elapsed, fwd = bench.max_over_ranks(dist, [1.0 + rank, 2.0 - rank], "cpu")
        ok_all = bench.all_ranks_ok(dist, True, "cpu")
        ok_one_failed = bench.all_ranks_ok(dist, rank == 0, "cpu")
        thr = bench.job_throughput(100, world, elapsed)
        q.put((rank, elapsed, fwd, ok_all, ok_one_failed, thr))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, fwd, ok_all, ok_one_failed, thr in res:
        assert elapsed == 2.0 and fwd == 2.0  # the slowest rank's numbers, on every rank
        assert ok_all is True and ok_one_failed is False
        assert thr == pytest.approx(100 * 2 / 2.0)


def test_single_process_helpers_without_a_group():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.max_over_ranks(None, [3.0, 4.0], "cpu") == [3.0, 4.0]
    assert bench.all_ranks_ok(None, False, "cpu") is False
    assert bench.job_throughput(10, 1, 2.0) == 5.0


def test_c5_shape_from_the_per_rank_count():
    """bench.c5_shape: groups of 8 on 3 lanes at the 1-GPU and 8-GPU per-rank counts, fewer lanes
    below one group per lane, explicit values kept"""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.c5_shape(1024) == (3, 8) and bench.c5_shape(128) == (3, 8)
    assert bench.c5_shape(8) == (1, 8) and bench.c5_shape(12) == (2, 8) and bench.c5_shape(1) == (1, 8)
    assert bench.c5_shape(128, lanes=2) == (2, 8) and bench.c5_shape(128, group=4) == (3, 4)


def test_c5_spawn_scatter_gather_two_ranks_gloo():
    """bench.py's C5 data path end to end on host buffers: shard.spawn_ranks starts 2 ranks with the
    rendezvous environment (what `bench.py --gpus 2` does without a launcher), rank 0 scatters
    session-format serialized ciphertexts at the C5 shape (N = 2^16, chain 26 in, the session's
    output chain out, strides from phantom_boot_layout), each rank checks and transforms its
    slice, rank 0 gathers and verifies order and every byte (tests/c5_gloo_worker.py)."""
    import json
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); import shard; "
            "sys.exit(shard.spawn_ranks(2, [sys.executable, %r], timeout=240))"
            % (os.path.join(ROOT, "phantom-fhe-boot_amd", "py"), os.path.join(ROOT, "tests", "c5_gloo_worker.py")))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 1 and rows[0]["ok"], (rows, out.stderr[-2000:])
    # 5 input limbs, 12 output limbs (chain 19: the reference's output level) at N = 2^16
    assert rows[0] == {"ok": True, "world": 2, "total": 4, "seed_bytes": 32, "in_bytes": 58 + 2 * 5 * 65536 * 8,
                       "out_bytes": 58 + 2 * 12 * 65536 * 8, "out_chain": 19}, rows


def test_c4_reference_bytes_by_hand():
    """The C4 roofline denominator is the reference schedule's work, recomputed here term by term
    (bench.c4_reference_bytes docstring): it depends on no engine counter."""
    sys.path.insert(0, ROOT)
    import bench
    w = 8 * 65536
    key = {2: 3 * 2 * 39, 3: 3 * 2 * 38, 4: 3 * 2 * 37, 7: 3 * 2 * 34, 11: 2 * 2 * 30, 12: 2 * 2 * 29,
           13: 2 * 2 * 28, 14: 2 * 2 * 27, 15: 2 * 2 * 26, 16: 2 * 2 * 25, 17: 2 * 2 * 24, 18: 2 * 2 * 23}
    keys = (70 * key[2] + 38 * key[3] + 70 * key[17] + 38 * key[18] + key[4] + 36 * key[7]
            + 2 * sum(key[c] for c in range(11, 17))) * w
    pts = (511 * 39 + 255 * 38 + 511 * 24 + 255 * 23) * w
    cts = (2 * 5 + 2 * 12) * w
    total, parts, der = bench.c4_reference_bytes()
    assert parts == {"keys": keys, "plaintexts": pts, "ciphertexts": cts}
    # the schedule the terms above hard-code, as bench derives it from the reference's level
    # selection (SelectLayers / GetCollapsedFFTParams / ComputeDegreesPS)
    assert [(l["dir"], l["chain"], l["diagonals"]) for l in der["levels"]] == [
        ("cts", 2, 511), ("cts", 3, 255), ("stc", 17, 511), ("stc", 18, 255)]
    assert der["ps_k_m"] == [6, 4] and der["output_chain"] == 19 and der["double_angle_chains"] == [11, 16]
    assert total == keys + pts + cts == 48196747264
