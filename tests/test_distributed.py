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
    # bench.py passes its GPU to the reductions; under gloo (its shared-GPU rehearsal, and
    # here, with no GPU at all) they must run on host tensors whatever device is named
    import torch
    gpu = torch.device("cuda", 0)
    q.put((rank, start, count, jdist.max_over_ranks(max(errs), device=gpu), merged,
           jdist.sum_over_ranks(count, device=gpu)))
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


# ---------------------------------------------------------------- the bench's launcher
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_ranks(world, args, local_ranks=None, timeout=240):
    """Start `world` children of tests/_rank_worker.py (one process per rank, as
    torch.distributed.run would) and return rank 0's JSON line."""
    import json
    import subprocess
    import sys
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port),
                   LOCAL_RANK=str(r if local_ranks is None else local_ranks[r]))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_rank_worker.py")]
                                      + args, env=env, stdout=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=timeout)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), [p.returncode for p in procs]
    return json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("gpus,extra,total", [(2, ["--global-batch", "8192", "--wavelet", "Symlet8",
                                                   "--levels", "6"], 8192),
                                              (4, [], 4096), (3, ["--global-batch", "1001"], 1001)])
def test_bench_launcher_ranks_and_shards(gpus, extra, total):
    # bench.py --gpus N (no torchrun): N rank processes with distinct RANK / LOCAL_RANK, one
    # gloo group of N, and contiguous shards that cover the global batch exactly once
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus),
                        "--launch-check"] + extra, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted((json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")),
                   key=lambda d: d["rank"])
    assert [d["rank"] for d in lines] == list(range(gpus))
    assert [d["local_rank"] for d in lines] == list(range(gpus))
    assert all(d["world"] == gpus and d["dist_world"] == gpus for d in lines)
    assert all(d["global_batch"] == total for d in lines)
    covered = []
    for d in lines:
        covered.extend(range(d["shard_start"], d["shard_start"] + d["shard_count"]))
        assert d["seed_first"] == 42 + d["shard_start"]
    assert covered == list(range(total))


def test_rank_worker_oracle_shards_match_serial():
    # the worker the GPU test drives, here on the oracle: 3 ranks, 11 signals
    import oracle as orc
    from jwave.transforms import wavelets as W
    res = _run_ranks(3, ["--oracle", "--n", "512", "--levels", "5", "--items", "11"])
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    expect = [float(np.sum(orc.modwt_forward(orc.fill_uniform(512, 42 + i), 5, g, h, "direct_nz")))
              for i in range(11)]
    assert res["sums"] == expect
    assert res["shards"] == [[0, 4], [4, 4], [8, 3]] and res["world"] == 3
    assert res["recon"] < 1e-11
