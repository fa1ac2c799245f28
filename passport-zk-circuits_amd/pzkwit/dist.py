"""Multi-GPU sharding of independent witnesses.

One process per GPU. A batch of independent passports is split into contiguous shards;
each rank generates/receives only its shard, computes its witnesses with no data-path
collective, and the small per-lane results (status + public signals, 160 B/witness) are
all-gathered. Over torch.distributed: "nccl" (= RCCL over xGMI) on GPUs, "gloo" on CPU.
"""


def shard_range(total, world, rank):
    """Contiguous shard [lo, hi) of `total` witnesses for `rank` (sizes differ by at most 1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_results(dist, status, public, device=None):
    """All-gather per-lane status (int32 [n]) and public signals (uint8 [n, k, 32]) from every
    rank; returns (status, public) of the whole job, rank-major (= global witness order)."""
    import torch
    world = dist.get_world_size()
    n = torch.tensor([status.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    k = public.shape[1]
    st_pad = torch.zeros(mx, dtype=torch.int32, device=device)
    st_pad[: status.shape[0]] = status
    pub_pad = torch.zeros((mx, k, 32), dtype=torch.uint8, device=device)
    pub_pad[: public.shape[0]] = public
    st_all = [torch.zeros_like(st_pad) for _ in range(world)]
    pub_all = [torch.zeros_like(pub_pad) for _ in range(world)]
    dist.all_gather(st_all, st_pad)
    dist.all_gather(pub_all, pub_pad)
    st = torch.cat([st_all[r][: int(sizes[r].item())] for r in range(world)])
    pub = torch.cat([pub_all[r][: int(sizes[r].item())] for r in range(world)])
    return st, pub
