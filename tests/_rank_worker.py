"""One rank of the multi-process tests (started by tests/test_distributed*.py as a child
process): joins the gloo group (or, --backend nccl, the RCCL communicator bench.py builds for
N > 1) from RANK / WORLD_SIZE / MASTER_*, takes its contiguous shard
of the global batch (jwave.distributed.shard_range, the bench's split), runs MODWT
forward + inverse on it through the HIP C-ABI on cuda:LOCAL_RANK (or through the oracle
with --oracle, for CPU-only runs), and all-gathers per-signal checksums in rank order.

Rank 0 prints one JSON line: {"sums": [...], "recon": max error, "shards": [[start, count]...]}.
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--levels", type=int, default=8)
    ap.add_argument("--items", type=int, default=11)
    ap.add_argument("--wavelet", default="Daubechies4")
    ap.add_argument("--oracle", action="store_true", help="CPU: the oracle instead of the engine")
    ap.add_argument("--backend", default="gloo", choices=("gloo", "nccl"))
    args = ap.parse_args()

    import torch.distributed as dist
    from jwave import distributed as jdist
    from jwave.transforms import wavelets as W
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    if args.backend == "nccl":  # as bench.py: the device first, then the communicator on it
        import torch
        torch.cuda.set_device(local_rank)
        rank, world = jdist.init_from_env("nccl", device=torch.device("cuda", local_rank))
    else:
        rank, world = jdist.init_from_env("gloo")
    start, count = jdist.shard_range(args.items, rank, world)
    n, J = args.n, args.levels
    wv = W.by_name(args.wavelet)
    if args.oracle:
        import oracle as orc
        g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        c = np.stack([orc.modwt_forward(orc.fill_uniform(n, 42 + i), J, g, h, "direct_nz")
                      for i in range(start, start + count)]) if count else np.zeros((0, J + 1, n))
        xr = np.stack([orc.modwt_inverse(ci, g, h, "direct_nz") for ci in c]) if count else c[:, 0]
        x = np.stack([orc.fill_uniform(n, 42 + i) for i in range(start, start + count)]) \
            if count else xr
    else:
        import torch
        from jwave import MODWTTransform, _native
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        xd = torch.empty((max(count, 1), n), dtype=torch.float64, device=dev)
        if count:  # the bench's inputs: java.util.Random(42 + global index), made in HBM
            _native.check(_native.lib().jw_synth_uniform(ctypes.c_void_p(xd.data_ptr()), n, count,
                                                         42 + start, None))
        m = MODWTTransform(wv)
        m.setConvolutionMethod(MODWTTransform.ConvolutionMethod.DIRECT)
        cd = m.forwardMODWT(xd[:count], J) if count else None
        xrd = m.inverseMODWT(cd) if count else None
        torch.cuda.synchronize()
        x = xd[:count].cpu().numpy()
        c = cd.cpu().numpy() if count else np.zeros((0, J + 1, n))
        xr = xrd.cpu().numpy() if count else x
    sums = [float(np.sum(ci)) for ci in c]
    width = args.items // world + 1  # equal-length all-gather: pad the shorter shards
    allv = jdist.gather_values(sums + [float("nan")] * (width - len(sums)))
    shards = jdist.gather_values([float(start), float(count)])
    recon = jdist.max_over_ranks(float(np.max(np.abs(xr - x))) if count else 0.0)
    if rank == 0:
        print(json.dumps({"sums": [v for v in allv if v == v], "recon": recon,
                          "shards": [[int(shards[2 * r]), int(shards[2 * r + 1])]
                                     for r in range(world)], "world": dist.get_world_size(),
                          "backend": dist.get_backend()}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
