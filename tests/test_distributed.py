"""The N>1 path on CPU: world_size-2 gloo ranks shard a batch, check their slices against
the oracle, and combine max / gather exactly as bench.py does on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from jwave import distributed as jdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_items, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import oracle as orc
    from jwave.transforms import wavelets as W
    jdist.init_from_env("gloo")
    start, count = jdist.shard_range(n_items, rank, world)
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    sums, errs = [], []
    for gidx in range(start, start + count):
        x = orc.fill_uniform(256, 42 + gidx)
        c = orc.modwt_forward(x, 4, g, h, "direct_nz")
        sums.append(float(np.sum(c)))
        errs.append(float(np.max(np.abs(orc.modwt_inverse(c, g, h, "direct_nz") - x))))
    # equal-length gather: pad to the largest shard
    width = n_items // world + 1
    padded = sums + [float("nan")] * (width - len(sums))
    allv = jdist.gather_values(padded)
    merged = [v for v in allv if v == v]
    q.put((rank, start, count, jdist.max_over_ranks(max(errs)), merged,
           jdist.sum_over_ranks(count)))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_shard_range_covers_batch():
    for n in (0, 1, 7, 1024, 8192, 1001):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = jdist.shard_range(n, r, world)
                seen.extend(range(s, s + c))
            assert seen == list(range(n))


def test_two_rank_gloo_sharding_matches_single_process():
    import oracle as orc
    from jwave.transforms import wavelets as W
    n_items, world = 11, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    expect = [float(np.sum(orc.modwt_forward(orc.fill_uniform(256, 42 + i), 4, g, h, "direct_nz")))
              for i in range(n_items)]
    for rank, start, count, maxerr, merged, total in res:
        assert merged == expect          # all-gather in rank order == serial order
        assert total == n_items          # every signal processed exactly once
        assert maxerr < 1e-11        # db4 DIRECT recon of uniform input is ~2e-12
    assert [r[1] for r in res] == [0, 6] and [r[2] for r in res] == [6, 5]
