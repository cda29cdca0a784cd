"""Multi-GPU layout: scenario instances are independent, so a batch is split into contiguous shards, one
per rank (one process per GPU), solved with no data-path collective, and the per-instance outputs are
collected on rank 0 with a single gather (RCCL over xGMI with the "nccl" backend; gloo on CPU)."""
import torch
import torch.distributed as dist


def shard_range(B, rank, world):
    """Contiguous [lo, hi) slice of a global batch of B for `rank` (sizes differ by at most one)."""
    base, rem = divmod(B, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_to_root(local, B, rank, world, root=0):
    """Gather the per-rank output rows (local: [rows_r, k]) into a [B, k] tensor on `root`."""
    if world == 1:
        return local
    sizes = [shard_range(B, r, world) for r in range(world)]
    cap = max(h - l for l, h in sizes)
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[:local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, parts, dst=root)
    if rank != root:
        return None
    return torch.cat([p[:h - l] for p, (l, h) in zip(parts, sizes)])
