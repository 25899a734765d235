"""Multi-GPU plumbing: one process per GPU, batch sharding, no data-path collective.

The hot path partitions naturally: every signal is independent, so rank r
transforms its own contiguous slice of the batch.  torch.distributed (RCCL over xGMI on the
MI355X node, gloo on CPU for tests) is used only for rendezvous, barriers and the small
reductions of the benchmark (max time, max error, checksums) -- never for signal data.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None, device=None):
    """Initialise the default process group from RANK / WORLD_SIZE / MASTER_* (127.0.0.1)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    dist.init_process_group(backend, **kw)
    return dist.get_rank(), dist.get_world_size()


def shard_range(n_items, rank, world):
    """Contiguous split of n_items over world ranks: (start, count); the first n % world
    ranks take one extra item."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _device(device=None):
    """Where a collective's tensor lives: the rank's GPU under RCCL, host memory under gloo
    (whatever device the caller names)."""
    if dist.get_backend() == "nccl":
        return device or torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def max_over_ranks(value, device=None):
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def sum_over_ranks(value, device=None):
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.item()


def gather_values(values, device=None):
    """All-gather a per-rank list of floats (equal lengths) -> flat list in rank order."""
    t = torch.tensor(list(values), dtype=torch.float64, device=_device(device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [v for o in out for v in o.tolist()]
