"""Multi-GPU data path of config C5: a batch of independent ciphertexts spread
over one process per GPU.

The reference has no multi-device layer; the build adds batch data-parallelism:
  * spawn_ranks: `bench.py --gpus N` launched without a launcher starts N copies of itself, one
    per GPU, with torch.distributed's rendezvous environment (as torch.distributed.run would),
    before anything touches a GPU;
  * scatter_rows / gather_rows: rank 0 holds the batch as serialized ciphertexts (the byte format
    of PhantomCiphertext::save, include/ciphertext.h:184-225), one fixed-stride row each; it
    scatters equal slices to the ranks and gathers the results back.  On GPUs the rows are device
    tensors and the collectives run over RCCL (xGMI); on CPU (tests) over gloo.
Nothing else is exchanged: every rank derives the same keys from a broadcast 32-byte seed, and the
bootstraps themselves need no communication (replicas only).
"""
import os
import socket
import subprocess


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, extra_env=None, timeout=None):
    """Run `argv` as n ranks (RANK = LOCAL_RANK = 0..n-1, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1)
    and wait for all; returns 0 if every rank exited 0, else the first non-zero exit status.
    Call only from a process that has not initialised a GPU (the children each take one)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen(argv, env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            rcs.append(124)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def _world(dist):
    if dist is None or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(), dist.get_rank()


def broadcast_seed(dist, device, nbytes=32):
    """32 bytes of OS entropy drawn on rank 0 and broadcast: the key seed every rank shares."""
    import torch
    world, rank = _world(dist)
    seed = torch.tensor(list(os.urandom(nbytes)) if rank == 0 else [0] * nbytes, dtype=torch.uint8, device=device)
    if world > 1:
        dist.broadcast(seed, src=0)
    return bytes(seed.cpu().tolist())


def scatter_rows(dist, full, rows_per_rank, row_bytes, device):
    """Rank 0's `full` ([world * rows_per_rank, row_bytes] uint8) -> each rank's own slice."""
    import torch
    world, rank = _world(dist)
    if world == 1:
        return full
    local = torch.empty((rows_per_rank, row_bytes), dtype=torch.uint8, device=device)
    chunks = list(full.chunk(world)) if rank == 0 else None
    dist.scatter(local, chunks, src=0)
    return local


def gather_rows(dist, local, device):
    """Every rank's `local` rows -> rank 0 gets them stacked in rank order; others get None."""
    import torch
    world, rank = _world(dist)
    if world == 1:
        return local
    if rank == 0:
        out = torch.empty((world * local.shape[0], local.shape[1]), dtype=torch.uint8, device=device)
        dist.gather(local, list(out.chunk(world)), dst=0)
        return out
    dist.gather(local, None, dst=0)
    return None


def gather_stats(dist, values, device):
    """Every rank's list of floats -> the per-rank lists in rank order, on every rank (an all-gather
    of one small float64 tensor; at world 1 just [values])."""
    import torch
    world, _ = _world(dist)
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if world == 1:
        return [t.tolist()]
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.tolist() for p in parts]
