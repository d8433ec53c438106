"""RCCL probe for C5's data path: N ranks (one per GPU) run the collectives bench.py's C5 leg
uses (py/shard.py: broadcast_seed, scatter_rows, gather_rows) over the "nccl" backend (RCCL) on
uint8 device tensors, and rank 0 checks the bytes.  At N = 1 (a one-GPU box: RCCL refuses two
ranks on one device, "Duplicate GPU detected") the shard helpers' world-1 shortcuts are bypassed
and dist.broadcast / scatter / gather run through a one-rank RCCL communicator.
usage: python tools/rccl_probe.py [N] [rows_per_rank] [row_bytes]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import shard  # noqa: E402


def rank_main(rows, row_bytes):
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("PROBE_DEVICE", os.environ["LOCAL_RANK"])))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    seed = shard.broadcast_seed(dist, dev)
    if world == 1:  # the helpers skip the collectives at world 1: issue them here
        t = torch.tensor(list(seed), dtype=torch.uint8, device=dev)
        dist.broadcast(t, src=0)
        seed = bytes(t.cpu().tolist())
    g = torch.Generator().manual_seed(int.from_bytes(seed[:8], "little"))
    full = None
    if rank == 0:
        full = torch.randint(0, 256, (world * rows, row_bytes), dtype=torch.uint8, generator=g).to(dev)
    if world == 1:
        local = torch.empty((rows, row_bytes), dtype=torch.uint8, device=dev)
        dist.scatter(local, list(full.chunk(1)), src=0)
    else:
        local = shard.scatter_rows(dist, full, rows, row_bytes, dev)
    local = (local.to(torch.int32) + rank + 1).to(torch.uint8)  # each rank's "work": a rank-dependent map
    if world == 1:
        out = torch.empty_like(local)
        dist.gather(local, [out], dst=0)
    else:
        out = shard.gather_rows(dist, local, dev)
    seeds = [None] * world
    dist.all_gather_object(seeds, seed)
    ok = True
    if rank == 0:
        expect = torch.cat([((c.to(torch.int32) + r + 1).to(torch.uint8)) for r, c in enumerate(full.chunk(world))])
        ok = bool(torch.equal(out, expect)) and all(s == seed for s in seeds)
        print(json.dumps({"backend": dist.get_backend(), "world": world, "rows_per_rank": rows,
                          "row_bytes": row_bytes, "bytes_scattered": world * rows * row_bytes,
                          "seed_agrees": all(s == seed for s in seeds), "gather_equal": ok,
                          "device": torch.cuda.get_device_name(dev)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    row_bytes = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    if "RANK" in os.environ:
        sys.exit(rank_main(rows, row_bytes))
    sys.exit(shard.spawn_ranks(n, [sys.executable, os.path.abspath(__file__), str(n), str(rows), str(row_bytes)],
                               timeout=150))
