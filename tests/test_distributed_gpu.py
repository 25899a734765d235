"""The N>1 path on the engine: two rank processes share cuda:0 (one box has one GPU; the
driver's 8-GPU run gives each rank its own), join one gloo group, run MODWT forward + inverse
through the HIP C-ABI on their contiguous shards, and all-gather per-signal checksums.  The
gathered checksums must equal the serial order computed by the oracle bit for bit (DIRECT,
STRICT arithmetic is bit-exact), so every signal was transformed exactly once, by the engine.
The RCCL variant runs the same worker as one rank on the nccl backend (RCCL refuses two ranks
on one GPU): bench.py's communicator setup, device-tensor all-reduce and all-gather.
"""
import numpy as np
import pytest

import oracle as orc
from jwave.transforms import wavelets as W
from test_distributed import _run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wname,n,J,items", [("Daubechies4", 4096, 8, 11), ("Symlet8", 8192, 6, 6)])
def test_two_ranks_share_gpu_engine_shards(wname, n, J, items, device):
    res = _run_ranks(2, ["--n", str(n), "--levels", str(J), "--items", str(items),
                         "--wavelet", wname], local_ranks=[0, 0])
    wv = W.by_name(wname)
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    expect = [float(np.sum(orc.modwt_forward(orc.fill_uniform(n, 42 + i), J, g, h, "direct_nz")))
              for i in range(items)]
    assert res["sums"] == expect
    half = (items + 1) // 2
    assert res["shards"] == [[0, half], [half, items - half]] and res["world"] == 2
    assert res["recon"] < 1e-11


def test_rccl_communicator_one_rank(device):
    # bench.py --gpus N's setup on RCCL: set_device, init_process_group("nccl", device_id=...),
    # then the max / all-gather reductions on device tensors
    n, J, items = 4096, 8, 5
    res = _run_ranks(1, ["--n", str(n), "--levels", str(J), "--items", str(items), "--backend",
                         "nccl"], local_ranks=[0])
    wv = W.by_name("Daubechies4")
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    expect = [float(np.sum(orc.modwt_forward(orc.fill_uniform(n, 42 + i), J, g, h, "direct_nz")))
              for i in range(items)]
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["sums"] == expect and res["shards"] == [[0, items]]
    assert res["recon"] < 1e-11
