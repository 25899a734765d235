#!/usr/bin/env python3
"""Headline benchmark: MODWT db4 forward+inverse, 8 levels, N=2^20, batch 1024 per GPU.

BASELINE.json metric: "Msamples/s forward+inverse MODWT (db4, 8 levels, N=2^20); max recon
error".  One step = jw_modwt_forward + jw_modwt_inverse over the whole batch, inputs
already resident in HBM (generated on-device: java.util.Random(42 + global signal index)).

Multi-GPU (one process per GPU, launched by torch.distributed.run): the batch is sharded --
every rank transforms its own 1024 independent signals, with no collective in the data
path (weak scaling); RCCL is used only for the barrier and the max-over-ranks time.

Also reported (rank 0): the roofline of the dominant kernel from HIP events on the kernel's
own stream, HBM traffic from the committed rocprofv3 PMC pass (profiles/), the max
reconstruction error, a bit-exact spot check of one signal against the oracle, and the
oracle's CPU time on a bounded sample ("port" CPU baseline).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Msamples/s forward+inverse MODWT (db4, 8 levels, N=2^20); max recon error"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "modwt_pmc_traffic.json")
# cwt / fwt2d HBM bytes per step at their default configs (tools/evidence.sh TAG traffic W,
# tools/summarize.py traffic)
TRAFFIC_STEP_FILE = os.path.join(ROOT, "profiles", "r06", "traffic_step.json")


def generate_inputs(gen, min_seconds=1.0):
    """Input generation (setup, untimed), repeated for about min_seconds: every call rewrites the
    same synthetic inputs, and the repetition brings a freshly started GPU to its steady clocks
    before the warmup steps (the first process on a fresh box otherwise timed 10-20x slow)."""
    t0 = time.perf_counter()
    while True:
        gen()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= min_seconds:
            return


def step_traffic(workload, is_default):
    if not is_default or not os.path.exists(TRAFFIC_STEP_FILE):
        return None
    try:
        return json.load(open(TRAFFIC_STEP_FILE))[workload]["bytes_per_step"]
    except Exception:
        return None


def host_cpu():
    """Threads the CPU baseline uses and what the host is: the GPU box allots 16 threads per
    GPU (OMP_NUM_THREADS there); elsewhere every CPU this process may run on."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or affinity
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, {"host_cpus": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": model}


REHEARSAL = {}  # JW_BENCH_SHARE_GPU=1: added to the JSON line (main)


def spawn_ranks(n):
    """bench.py --gpus N without a launcher: start N rank processes of this script (one per
    GPU, RANK = LOCAL_RANK = r, rendezvous on 127.0.0.1) and return the worst exit code.  This
    parent makes no GPU call (it only waits), so nothing initialises HIP before the fork."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def inv_kernel_name(L, J, n, arith="fma"):
    """Which inverse MODWT kernel the library launches (csrc/jw_modwt_fast.hpp launch_inv,
    jw_modwt_wave2.hpp inv_ok / inv_prefer2 and jw_modwt_wave.hpp inv_wave_ok restated): two
    outputs per lane (wave2) where it fits and is preferred, else one stream per wave, else the
    workgroup-shared kernel; JW_INV_KERNEL forces one of them."""
    fast = L in (2, 4, 6, 8, 12, 16, 20) and J <= 10 and 512 <= n < (1 << 27)
    if not fast:
        return "modwt_inv_fused"
    env = os.environ.get("JW_INV_KERNEL", "")
    if L % 2:
        return "modwt_inv_fast"
    hist = [(L - 1) << (j - 1) for j in range(1, J + 1)]
    rtot = sum((L - 1) * (1 << (j - 7)) + 1 for j in range(7, J + 1))
    nx_nz = max(L // 2, 2) + L // 2
    lds1 = sum(64 + hist[j - 1] for j in range(1, min(J, 5) + 1)) * 16
    wave1 = J >= 6 and lds1 <= 20 * 1024 and rtot + nx_nz <= 31
    lds2 = 0
    for j in range(1, min(J, 5) + 1):
        d = 1 << (j - 1)
        nblk = (128 + hist[j - 1]) // d
        half = ((((nblk + 1) // 2) * d + 7) & ~7) + (d if d < 8 else 0)
        lds2 += 2 * half * 16
    wave2 = (n % 2 == 0 and lds2 <= 20 * 1024 and
             (rtot if J >= 7 else 0) + (nx_nz if J >= 6 else 0) <= 31)
    prefer2 = J <= 7 or L <= 8  # jw_modwt_wave2.hpp inv_prefer2 (both contracts)
    if env == "wg":
        return "modwt_inv_fast"
    if wave2 and (env == "wave2" or (env not in ("wave", "wave1") and (prefer2 or not wave1))):
        return "modwt_inv_wave2"
    return "modwt_inv_wave" if wave1 else "modwt_inv_fast"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="signals per GPU")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="modwt strong scaling (BASELINE configs[4]): this many signals in total, "
                         "split over the ranks and processed in resident chunks of --chunk")
    ap.add_argument("--chunk", type=int, default=1024, help="signals per launch (--global-batch)")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--levels", type=int, default=8)
    ap.add_argument("--wavelet", default="Daubechies4")
    ap.add_argument("--arith", choices=["strict", "fma"], default="fma",
                    help="headline arithmetic; the other contract is timed too and reported")
    ap.add_argument("--no-alt", action="store_true", help="skip timing the other arith mode")
    ap.add_argument("--workload", choices=["modwt", "cwt", "fwt2d"], default="modwt",
                    help="modwt: the headline metric (BASELINE configs[1]); cwt: configs[2]")
    ap.add_argument("--scales", type=int, default=64, help="cwt: number of log scales 2..1024")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--launch-check", action="store_true",
                    help="print each rank's identity and batch shard, then exit (no GPU work)")
    return ap.parse_args()


CORES_REASON = ("threads = OMP_NUM_THREADS when set: the GPU box allots each GPU a share of 16 "
                "host CPUs (OMP_NUM_THREADS=16 there) although affinity shows the whole "
                "machine; BASELINE.md's 'all host cores' would oversubscribe the other GPUs' "
                "shares, so the baseline is stated per 16-CPU share (scale by affinity_cpus/16 "
                "for a whole-host estimate)")


def cpu_baseline(wname, n, J):
    """Oracle (C restatement of JWave's CPU path) on a bounded sample, signals split by
    ForkJoin-style recursive halving (ParallelTransform.java:222-335)."""
    import oracle as orc
    from jwave.transforms import wavelets as W
    threads, host = host_cpu()
    wv = W.by_name(wname)
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    # AUTO-faithful: at N=2^20 JWave's default performConvolution picks the FFT path for
    # every level (N*M_j > 4096, MODWTTransform.java:653) -- recurrence-twiddle radix-2 FFT.
    ns = 2 * threads  # two signals per thread: ~10-15 s of CPU work on the box
    xs = orc.fill_uniform(ns * n, 42).reshape(ns, n)
    t0 = time.perf_counter()
    orc.modwt_fwdinv_batch(xs, J, g, h, use_fft=True, threads=threads)
    t_auto = time.perf_counter() - t0
    # DIRECT-faithful (every up-sampled tap incl. zeros, floorMod) on quarter-length signals;
    # its cost per sample does not depend on N.
    nd = n // 4
    t0 = time.perf_counter()
    orc.modwt_fwdinv_batch(xs[:threads, :nd].copy(), J, g, h, use_fft=False, threads=threads)
    t_direct = time.perf_counter() - t0
    return dict({
        "value": ns * n / t_auto / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{ns} signals x N={n} {wname} J={J} fwd+inv, AUTO path as JWave runs it "
                   f"(FFT convolution, MODWTTransform.java:653), ForkJoin halving over signals on "
                   f"{threads} threads: {t_auto:.2f} s; DIRECT-faithful on {threads} x N={nd}: "
                   f"{threads * nd / t_direct / 1e6:.3f} Msamples/s"),
        "cores_reason": CORES_REASON,
        "direct_value": threads * nd / t_direct / 1e6,
    }, **host)


def main_cwt(args, dev, rank, world):
    """BASELINE configs[2]: ContinuousWaveletTransform(Morlet omega0=6).transformFFT, 64 log
    scales 2..1024, N=2^18, batch 256 per GPU, fs=1, SYMMETRIC padding (N is a power of 2, so
    no padding occurs).  One step = one jw_cwt_fft call over the batch (all FFT passes)."""
    import math
    import oracle as orc
    from jwave import ContinuousWaveletTransform as CWT, _native
    B = args.batch if args.batch != 1024 else 256
    n = args.n if args.n != (1 << 20) else (1 << 18)
    ns = args.scales
    fb, fc = 1.0, 6.0 / (2 * math.pi)
    scales = CWT.generateLogScales(2.0, 1024.0, ns)
    lib = _native.lib()
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)
    x = torch.empty((B, n), dtype=torch.float64, device=dev)
    out = torch.empty((B, ns, n, 2), dtype=torch.float64, device=dev)
    generate_inputs(lambda: _native.check(
        lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 7 + rank * B, sptr)))
    prm = (ctypes.c_double * 2)(fb, fc)
    sc = np.ascontiguousarray(scales)
    # the engine's own scale split for this call (jw_cwt_fft_paths: the rule jw_cwt_fft runs)
    split = [ctypes.c_int(0) for _ in range(3)]
    _native.check(lib.jw_cwt_fft_paths(_native.JW_CWT_MORLET, prm, n,
                                       sc.ctypes.data_as(ctypes.c_void_p), ns, 1.0,
                                       *[ctypes.byref(v) for v in split]))
    n_two, n_band, n_coarse = (v.value for v in split)

    def call():
        _native.check(lib.jw_cwt_fft(_native.JW_CWT_MORLET, prm, ctypes.c_void_p(x.data_ptr()), n,
                                     sc.ctypes.data_as(ctypes.c_void_p), ns, 1.0,
                                     _native.JW_PAD_SYMMETRIC, ctypes.c_void_p(out.data_ptr()), B,
                                     _native.JW_DEVICE, sptr))

    for _ in range(args.warmup):
        call()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        call()
    e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        from jwave import distributed as jdist
        elapsed = jdist.max_over_ranks(elapsed, device=dev)
    ms = e0.elapsed_time(e1) / args.steps
    value = world * B * n * args.steps / elapsed / 1e6
    per_call = (8 + ns * 16) * B * n  # read the signal, write ns complex coefficients
    res = None
    if rank == 0 and not args.no_check:
        x0 = x[0].cpu().numpy()
        got = out[0].cpu().numpy()
        got = got[..., 0] + 1j * got[..., 1]
        ex = orc.cwt_fft(x0, scales, 1.0, "morlet", (fb, fc), 1, exact=True)
        jw = orc.cwt_fft(x0, scales, 1.0, "morlet", (fb, fc), 1, exact=False)
        res = {"vs_exact_twiddles": float(np.max(np.abs(got - ex)) / np.max(np.abs(ex))),
               "vs_jwave_recurrence": float(np.max(np.abs(got - jw)) / np.max(np.abs(jw)))}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # transformFFTParallel (ContinuousWaveletTransform.java:511-565) per signal, signals in
        # the outer ForkJoin pool, recurrence-twiddle FFT as the reference
        threads, host = host_cpu()
        nsig = threads
        xs = np.stack([orc.fill_uniform(n, 7 + b) for b in range(nsig)])
        t0 = time.perf_counter()
        orc.cwt_fft_parallel_batch(xs, scales, 1.0, "morlet", (fb, fc), 1, threads=threads)
        tc = time.perf_counter() - t0
        cpu = dict({"value": nsig * n / tc / 1e6, "unit": "Msamples/s", "cores": threads,
                    "kind": "port",
                    "sample": f"{nsig} signals x N={n}, {ns} scales, oracle transformFFTParallel "
                              f"(scales in parallel per signal, signals in the outer pool, "
                              f"recurrence-twiddle radix-2 FFT like FastFourierTransform.java), "
                              f"{threads} threads: {tc:.2f} s", "cores_reason": CORES_REASON}, **host)
    if rank == 0:
        ach = per_call / (ms * 1e-3) / 1e9
        print(json.dumps({
            "metric": f"Msamples/s CWT Morlet(omega0=6) transformFFT, {ns} scales, N=2^18",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (java.util.Random(7+signal).nextDouble()*2-1, generated in HBM)",
            "config": {"workload": f"ContinuousWaveletTransform(Morlet fb=1 fc=6/2pi) transformFFT,"
                                   f" {ns} log scales 2..1024, N={n}, batch={B} per GPU "
                                   f"(BASELINE configs[2])", "batch_per_gpu": B, "n": n},
            "parity": res,
            "roofline": {"bound": "hbm", "kernel": "jw_cwt_fft (all passes, one call)",
                         "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": step_traffic("cwt", (B, n, ns) == (256, 1 << 18, 64)),
                         "algorithmic_bytes_per_launch": per_call,
                         "note": "one launch = one jw_cwt_fft call over the batch (all FFT "
                                 "passes); traffic = rocprofv3 FETCH_SIZE*2 + WRITE_SIZE per call "
                                 f"({os.path.relpath(TRAFFIC_STEP_FILE, ROOT)}): the A workspace round "
                                 f"trip of the {n_two} two-pass scales is the excess over "
                                 f"algorithmic; the {n_coarse} scales whose band fits a coarse grid "
                                 "of N/P points (P >= 4) run as an M-point inverse DFT "
                                 "(cwt_band512 on the coarse grid) plus a Kaiser-Bessel "
                                 "interpolation (cwt_interp) that writes each coefficient once, "
                                 f"and {n_band} through the one-pass band kernel (DESIGN.md 5.4; "
                                 "split from jw_cwt_fft_paths)",
                         "scale_split": {"two_pass": n_two, "band": n_band, "coarse_grid": n_coarse}},
            "cpu_baseline": cpu, **REHEARSAL}), flush=True)


def main_fwt2d(args, dev, rank, world):
    """BASELINE configs[3]: FastWaveletTransform(Daubechies8) 2-D forward + reverse on 4096 x
    4096 images, batch 64 per GPU, full levels (getExponent = 12 per axis).  One step = one
    jw_fwt2d_forward + one jw_fwt2d_reverse over the batch."""
    import oracle as orc
    from jwave import _native
    from jwave.transforms import wavelets as W
    B = args.batch if args.batch != 1024 else 64
    R = 4096
    lvl = 12
    wv = W.Daubechies8()
    lib = _native.lib()
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)
    plan = ctypes.c_void_p()
    arr = lambda v: (ctypes.c_double * len(v))(*v)  # noqa: E731
    arith = _native.JW_ARITH_FMA if args.arith == "fma" else _native.JW_ARITH_STRICT
    _native.check(lib.jw_fwt_plan_create(
        ctypes.byref(plan), arr(wv.getScalingDeComposition()), arr(wv.getWaveletDeComposition()),
        arr(wv.getScalingReConstruction()), arr(wv.getWaveletReConstruction()),
        wv.getMotherWavelength(), wv.getTransformWavelength(), getattr(wv, "kind", 0), arith))
    x = torch.empty((B, R, R), dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    xr = torch.empty_like(x)
    generate_inputs(lambda: _native.check(
        lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), R * R, B, 11 + rank * B, sptr)))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def fwd():
        _native.check(lib.jw_fwt2d_forward(plan, P(x), P(y), R, R, lvl, lvl, B,
                                           _native.JW_DEVICE, sptr))

    def rev():
        _native.check(lib.jw_fwt2d_reverse(plan, P(y), P(xr), R, R, lvl, lvl, B,
                                           _native.JW_DEVICE, sptr))

    for _ in range(args.warmup):
        fwd()
        rev()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t0 = time.perf_counter()
    fms = rms_ = 0.0
    for _ in range(args.steps):
        ev[0].record(stream)
        fwd()
        ev[1].record(stream)
        rev()
        ev[2].record(stream)
        torch.cuda.synchronize()
        fms += ev[0].elapsed_time(ev[1])
        rms_ += ev[1].elapsed_time(ev[2])
    elapsed = time.perf_counter() - t0
    if world > 1:
        from jwave import distributed as jdist
        elapsed = jdist.max_over_ranks(elapsed, device=dev)
    fms /= args.steps
    rms_ /= args.steps
    value = world * B * R * R * args.steps / elapsed / 1e6
    err = ((xr - x).abs().max() / x.abs().max()).item()
    check = None
    if rank == 0 and not args.no_check:
        ref = orc.fwt2d_forward(x[0].cpu().numpy(), lvl, lvl, wv)
        got = y[0].cpu().numpy()
        check = "bit-exact" if np.array_equal(ref, got) else \
            f"normwise {np.max(np.abs(ref - got)) / np.max(np.abs(ref)):.3g}"
    lib.jw_fwt_plan_destroy(plan)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # ParallelTransform 2-D (ParallelTransform.java:70-126): per image, rows task then
        # columns task forward, columns then rows reverse, leaves of <= 16 lines
        threads, host = host_cpu()
        nimg = 4
        xs = np.stack([orc.fill_uniform(R * R, 11 + b).reshape(R, R) for b in range(nimg)])
        t0 = time.perf_counter()
        orc.fwt2d_fwdrev_parallel(xs, lvl, lvl, wv, threads=threads)
        tc = time.perf_counter() - t0
        cpu = dict({"value": nimg * R * R / tc / 1e6, "unit": "Mpixels/s", "cores": threads,
                    "kind": "port",
                    "sample": f"{nimg} images {R}x{R} Daubechies8 12x12 levels forward+reverse, "
                              f"oracle ParallelTransform pattern (rows task -> columns task) on "
                              f"{threads} threads: {tc:.2f} s", "cores_reason": CORES_REASON}, **host)
    if rank == 0:
        per = 64 * B * R * R  # 2 passes x (read + write) x 8 B, forward + reverse
        ach = per / ((fms + rms_) * 1e-3) / 1e9
        print(json.dumps({
            "metric": "Mpixels/s FWT Daubechies8 2-D forward+reverse (4096x4096, 12x12 levels)",
            "value": round(value, 2), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (java.util.Random(11+image).nextDouble()*2-1, generated in HBM)",
            "config": {"workload": f"FastWaveletTransform(Daubechies8) 2-D fwd+rev, 4096x4096, "
                                   f"batch={B} per GPU (BASELINE configs[3])", "arith": args.arith},
            "max_recon_error": err, "spot_check_vs_oracle": check,
            "roofline": {"bound": "hbm", "kernel": "jw_fwt2d_forward + jw_fwt2d_reverse",
                         "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": step_traffic("fwt2d", B == 64),
                         "algorithmic_bytes_per_step": per, "fwd_ms": round(fms, 3),
                         "rev_ms": round(rms_, 3)},
            "cpu_baseline": cpu, **REHEARSAL}), flush=True)


def launch_check(args, rank, local_rank, world):
    """--launch-check: each rank reports who it is and which signals it owns (no GPU)."""
    from jwave import distributed as jdist
    if world > 1:
        jdist.init_from_env("gloo")
    total = args.global_batch if args.global_batch > 0 else args.batch * world
    start, count = jdist.shard_range(total, rank, world)
    print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world,
                      "dist_world": dist.get_world_size() if world > 1 else 1,
                      "global_batch": total, "shard_start": start, "shard_count": count,
                      "seed_first": (42 if args.workload == "modwt" else 0) + start}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        return launch_check(args, rank, local_rank, world)
    # JW_BENCH_SHARE_GPU=1 (rehearsal of the multi-rank path on a box with fewer GPUs than
    # ranks; never set by the driver): rank r runs on GPU r mod count, over gloo (RCCL takes
    # one rank per GPU), and the JSON line says so -- a check that the ranks shard, time and
    # reduce correctly on hardware, not a scaling number
    share = os.environ.get("JW_BENCH_SHARE_GPU") == "1"
    if share:
        local_rank %= torch.cuda.device_count()
        REHEARSAL["shared_gpu_rehearsal"] = {
            "ranks": world, "gpus": torch.cuda.device_count(), "backend": "gloo",
            "note": "ranks share GPUs: checks sharding, timing and reductions, not scaling"}
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        from jwave import distributed as jdist
        jdist.init_from_env("gloo" if share else "nccl", device=None if share else dev)
        world = dist.get_world_size()  # the RCCL communicator's size (echoed as n_gpus)
    if args.workload == "cwt":
        return main_cwt(args, dev, rank, world)
    if args.workload == "fwt2d":
        return main_fwt2d(args, dev, rank, world)

    from jwave import MODWTTransform, _native
    from jwave.transforms import wavelets as W

    n, J = args.n, args.levels
    strong = args.global_batch > 0
    if strong:  # configs[4]: a fixed total batch, sharded contiguously over the ranks
        assert args.global_batch % world == 0, "--global-batch must divide over the ranks"
        Bl = args.global_batch // world
    else:       # weak scaling: every rank owns --batch signals
        Bl = args.batch
    B = min(Bl, args.chunk) if strong else Bl  # signals per launch
    assert Bl % B == 0, "--chunk must divide the per-rank batch"
    chunks = Bl // B
    wv = W.by_name(args.wavelet)
    lib = _native.lib()
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)

    # inputs and reconstructions of the whole local batch stay resident; the coefficients
    # of one launch's chunk are reused (sym8 J=6, 8192 signals on 1 GPU: 64 + 64 + 56 GB)
    x = torch.empty((Bl, n), dtype=torch.float64, device=dev)
    c = torch.empty((B, J + 1, n), dtype=torch.float64, device=dev)
    xr = torch.empty((Bl, n), dtype=torch.float64, device=dev)
    seed0 = 42 + rank * Bl  # rank r owns global signals [r*Bl, (r+1)*Bl), seed 42 + g
    generate_inputs(lambda: _native.check(
        lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, Bl, seed0, sptr)))

    def run(arith, steps, warmup):
        """Time `steps` fwd+inv steps; returns (elapsed_s max over ranks, fwd_ms, inv_ms)."""
        m = MODWTTransform(wv, arith=arith)
        m.setConvolutionMethod(MODWTTransform.ConvolutionMethod.DIRECT)
        plan = m.initializeFilterCache()

        def fwd(q):
            _native.check(lib.jw_modwt_forward(plan, ctypes.c_void_p(x[q * B].data_ptr()),
                                               ctypes.c_void_p(c.data_ptr()), n, J, B,
                                               _native.JW_CONV_DIRECT, _native.JW_DEVICE, sptr))

        def inv(q):
            _native.check(lib.jw_modwt_inverse(plan, ctypes.c_void_p(c.data_ptr()),
                                               ctypes.c_void_p(xr[q * B].data_ptr()), n, J, B,
                                               _native.JW_CONV_DIRECT, _native.JW_DEVICE, sptr))

        for _ in range(warmup):
            for q in range(chunks):
                fwd(q)
                inv(q)
        torch.cuda.synchronize()
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
              for _ in range(steps * chunks)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            for q in range(chunks):  # one step = the whole local batch, chunk by chunk
                e = ev[k * chunks + q]
                e[0].record(stream)
                fwd(q)
                e[1].record(stream)
                inv(q)
                e[2].record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            from jwave import distributed as jdist
            elapsed = jdist.max_over_ranks(elapsed, device=dev)
        # per launch (one chunk) averages
        fwd_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev)
        inv_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / len(ev)
        return elapsed, fwd_ms, inv_ms

    def spot_check(arith):
        """One signal's coefficients against the oracle (bit-exact for strict)."""
        import numpy as np
        import oracle as orc
        g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        sig = min(1, B - 1)  # of the last chunk, whose coefficients c still holds
        ref = orc.modwt_forward(orc.fill_uniform(n, seed0 + (chunks - 1) * B + sig), J, g, h,
                                "direct_nz")
        got = c[sig].cpu().numpy()
        if arith == "strict":
            return "bit-exact" if np.array_equal(got.view(np.uint64), ref.view(np.uint64)) else \
                f"MISMATCH max {float(np.max(np.abs(got - ref)))}"
        return f"normwise {float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))):.2e}"

    def auto_strict_bytes(nsig, L, threshold=4096):
        """HBM bytes one jw_modwt_forward + jw_modwt_inverse of JWave's default path (AUTO,
        JW_ARITH_STRICT) must move with the engine's kernel structure (jw_jfft.hip
        forward_cols / inverse_cols, power-of-two n > 4096): every kernel reads its inputs and
        writes its outputs once.  Per FFT level, forward: [kp1 of V_{j-1}: 8n in, 16n out, unless
        the previous level fused it] + kp2p (two items: 2 x 16n in, 2 x 16n out) + kp2r for W_j
        (16n in, 8n out) + kp2r for V_j (16n in; 16n out fused into the next FFT level's pass 1,
        else 8n); inverse: [kp1 of V_j unless fused] + kp1 of W_j (8n in, 16n out) + kp2p (2 x 16n
        in and out) + kp2r of both (2 x 16n in; 16n out fused, else 8n).  DIRECT levels: the
        per-level direct kernels (forward 8n in, 16n out; inverse 16n in, 8n out)."""
        import numpy as np  # noqa: F401
        if n <= 4096 or n & (n - 1):
            return None
        def fft_level(j):  # MODWTTransform.java:653, int32 product
            m = (L - 1) * (1 << (j - 1)) + 1
            prod = (n * m) & 0xffffffff
            prod = prod - (1 << 32) if prod >= (1 << 31) else prod
            return prod > threshold
        f = [None] + [fft_level(j) for j in range(1, J + 1)]
        total, fused = 0, False
        for j in range(1, J + 1):  # forward
            if not f[j]:
                total += 24 * n
                fused = False
                continue
            nxt = j < J and f[j + 1]
            total += (0 if fused else 24 * n) + 64 * n + 24 * n + (32 if nxt else 24) * n
            fused = nxt
        fused = False
        for j in range(J, 0, -1):  # inverse
            if not f[j]:
                total += 24 * n
                fused = False
                continue
            nxt = j > 1 and f[j - 1]
            total += (0 if fused else 24 * n) + 24 * n + 64 * n + (48 if nxt else 40) * n
            fused = nxt
        return total * nsig

    def extra_paths(nb=16, reps=3, nb_auto=128):
        """Secondary figures on a 16-signal sub-batch (never the headline):
        * JW_HOST: host double[] in, host double[] out -- what a JNI caller passing Java arrays
          gets, PCIe staging included;
        * AUTO under JW_ARITH_STRICT: the reference's default ConvolutionMethod, which at this N
          takes the FFT path at every level (MODWTTransform.java:653), run as the reference runs
          it (its own FFT, level by level): bit-exactness against the oracle's restatement of
          that path (one signal) and throughput;
        * FFT under JW_ARITH_FMA: the exact-twiddle frequency-domain pyramid (the fast FFT
          option) and its deviation from the reference's FFT path and from DIRECT."""
        import numpy as np
        import oracle as orc
        P = lambda a: ctypes.c_void_p(a.ctypes.data if isinstance(a, np.ndarray)  # noqa: E731
                                      else a.data_ptr())
        xh = np.ascontiguousarray(x[:nb].cpu().numpy())
        ch = np.empty((nb, J + 1, n))
        xrh = np.empty((nb, n))
        hxf = MODWTTransform(wv, arith=args.arith)  # owns its plan: keep it referenced
        hplan = hxf.initializeFilterCache()

        def host_step():
            _native.check(lib.jw_modwt_forward(hplan, P(xh), P(ch), n, J, nb, _native.JW_CONV_DIRECT,
                                               _native.JW_HOST, None))
            _native.check(lib.jw_modwt_inverse(hplan, P(ch), P(xrh), n, J, nb, _native.JW_CONV_DIRECT,
                                               _native.JW_HOST, None))

        host_step()  # the staging buffers grow once
        t0 = time.perf_counter()
        for _ in range(reps):
            host_step()
        th = (time.perf_counter() - t0) / reps
        host = {"value": round(nb * n / th / 1e6, 1), "unit": "Msamples/s", "signals": nb,
                "ms_per_call_pair": round(th * 1e3, 2),
                "note": "jw_modwt_forward + jw_modwt_inverse with where=JW_HOST (host arrays "
                        "in and out, DIRECT), PCIe staging included; never the headline value",
                "recon_max_abs": float(np.max(np.abs(xrh - xh)))}
        # the reference API's own unit (MODWTTransform.java:256,337; the JNI nForward/nInverse):
        # one signal per call, host arrays in and out
        x1, c1, xr1 = xh[:1].copy(), np.empty((1, J + 1, n)), np.empty((1, n))

        def one_step():
            _native.check(lib.jw_modwt_forward(hplan, P(x1), P(c1), n, J, 1, _native.JW_CONV_DIRECT,
                                               _native.JW_HOST, None))
            _native.check(lib.jw_modwt_inverse(hplan, P(c1), P(xr1), n, J, 1, _native.JW_CONV_DIRECT,
                                               _native.JW_HOST, None))

        one_step()
        t0 = time.perf_counter()
        for _ in range(4 * reps):
            one_step()
        t1 = (time.perf_counter() - t0) / (4 * reps)
        host["one_signal"] = {"value": round(n / t1 / 1e6, 1), "unit": "Msamples/s",
                              "ms_per_call_pair": round(t1 * 1e3, 3),
                              "note": "batch 1 per call (the reference API's unit; JNI nForward + "
                                      "nInverse), host arrays, PCIe staging included"}
        nb = min(nb_auto, Bl)  # AUTO / FFT legs: a batch that fills the chip
        ca = torch.empty((nb, J + 1, n), dtype=torch.float64, device=dev)
        xra = torch.empty((nb, n), dtype=torch.float64, device=dev)

        def timed(arith, method):
            xf = MODWTTransform(wv, arith=arith)  # owns its plan: keep it referenced
            plan = xf.initializeFilterCache()

            def step():
                _native.check(lib.jw_modwt_forward(plan, P(x), P(ca), n, J, nb, method,
                                                   _native.JW_DEVICE, sptr))
                _native.check(lib.jw_modwt_inverse(plan, P(ca), P(xra), n, J, nb, method,
                                                   _native.JW_DEVICE, sptr))
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                step()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps

        g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        jw_auto = orc.modwt_forward(xh[0], J, g, h, "auto")  # = "fft" wherever N*M_j > 4096
        exact = orc.modwt_forward(xh[0], J, g, h, "direct_nz")
        dev_rows = lambda a, b: max(float(np.max(np.abs(a[r] - b[r])) / np.max(np.abs(b[r])))  # noqa: E731
                                    for r in range(J + 1))
        ta = timed("strict", _native.JW_CONV_AUTO)
        got = ca[0].cpu().numpy()
        auto = {"method": "AUTO, JW_ARITH_STRICT (JWave's default): every level whose N*M_j > 4096 "
                          "(MODWTTransform.java:653) through the reference's own FFT convolution",
                "value": round(nb * n / ta / 1e6, 1), "unit": "Msamples/s", "signals": nb,
                "ms_per_signal_fwd_inv": round(ta * 1e3 / nb, 3),
                "bit_exact_vs_reference_path": bool(np.array_equal(got.view(np.uint64),
                                                                   jw_auto.view(np.uint64))),
                "max_abs_vs_reference_path": float(np.max(np.abs(got - jw_auto))),
                "reference_path_vs_exact_direct": dev_rows(jw_auto, exact),
                "recon_max_abs": (xra - x[:nb]).abs().max().item()}
        ab = auto_strict_bytes(nb, len(wv.getScalingDeComposition()))
        if ab:
            auto["roofline"] = {
                "bound": "hbm", "achieved": round(ab / ta / 1e9, 1), "peak": 8000.0,
                "unit": "GB/s", "frac": round(ab / ta / 8e12, 4),
                "bytes_per_sample": ab / (nb * n),
                "note": "bytes = what the AUTO STRICT kernel chain must move, every kernel reading "
                        "its inputs and writing its outputs once (bench.py auto_strict_bytes: the "
                        "three FFT-sized complex transforms per forward level, four per inverse "
                        "level, each two column passes through HBM) / forward+inverse time"}
        tp = timed("fma", _native.JW_CONV_FFT)
        got = ca[0].cpu().numpy()
        auto["fft_pyramid_fma"] = {
            "method": "FFT, JW_ARITH_FMA: exact-twiddle frequency-domain pyramid (fast option)",
            "value": round(nb * n / tp / 1e6, 1), "unit": "Msamples/s",
            "max_row_normwise_vs_reference_fft_path": dev_rows(got, jw_auto),
            "max_row_normwise_vs_exact_direct": dev_rows(got, exact),
            "recon_max_abs": (xra - x[:nb]).abs().max().item()}
        return host, auto

    alt_arith = "strict" if args.arith == "fma" else "fma"
    alt = None
    if not args.no_alt:
        a_el, a_f, a_i = run(alt_arith, max(2, args.steps // 2), 1)
        alt = {"arith": alt_arith, "value": round(Bl * n * world / (a_el / max(2, args.steps // 2)) / 1e6, 1),
               "fwd_ms": round(a_f, 3), "inv_ms": round(a_i, 3)}
        if rank == 0 and not args.no_check:
            alt["spot_check_vs_oracle"] = spot_check(alt_arith)

    elapsed, fwd_ms, inv_ms = run(args.arith, args.steps, args.warmup)
    ms_per_step = elapsed * 1e3 / args.steps
    total_samples = Bl * n * world
    value = total_samples / (elapsed / args.steps) / 1e6

    # Reconstruction error over the whole local batch (max over ranks).
    # chunkwise: a whole-batch temporary would not fit beside the resident buffers
    dmax = xmax = ssq = 0.0
    for q in range(chunks):
        d = xr[q * B:(q + 1) * B] - x[q * B:(q + 1) * B]
        dmax = max(dmax, d.abs().amax().item())
        xmax = max(xmax, x[q * B:(q + 1) * B].abs().amax().item())
        ssq += torch.sum(d * d).item()
        del d
    err = dmax / xmax
    rms = (ssq / (Bl * n)) ** 0.5
    if world > 1:
        from jwave import distributed as jdist
        err = jdist.max_over_ranks(err, device=dev)
        rms = jdist.max_over_ranks(rms, device=dev)

    if rank == 0:
        # Roofline of the dominant kernel: algorithmic bytes per launch / average launch time.
        # forward: read x (8 B) + write J+1 rows (8(J+1) B) per sample; inverse the mirror.
        bytes_per_sample = 8 * (1 + (J + 1))
        per_launch = bytes_per_sample * B * n
        L = len(wv.getScalingDeComposition())
        name, ms = ((inv_kernel_name(L, J, n, args.arith), inv_ms) if inv_ms >= fwd_ms
                    else ("modwt_fwd_fast", fwd_ms))
        achieved = per_launch / (ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(TRAFFIC_FILE):
            try:
                tr = json.load(open(TRAFFIC_FILE))
                key = f"{args.wavelet}/J{J}/N{n}/B{B}/{args.arith}"
                traffic = tr.get(key, {}).get(name)
            except Exception:
                traffic = None
        check = None if args.no_check else spot_check(args.arith)
        out = {
            "metric": METRIC if (args.wavelet, J, n) == ("Daubechies4", 8, 1 << 20) else
            (f"Msamples/s forward+inverse MODWT ({args.wavelet}, {J} levels, N={n}); "
             f"max recon error"),
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "dist_world_size": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (java.util.Random(42+signal).nextDouble()*2-1, generated in HBM)",
            "config": {
                "workload": (f"MODWTTransform({args.wavelet}) forwardMODWT+inverseMODWT, J={J}, "
                             + (f"N={n}, {args.global_batch} signals over {world} GPU(s) in "
                                f"chunks of {B}, DIRECT convolution (BASELINE configs[4])"
                                if strong else
                                f"N={n}, batch={B} per GPU, DIRECT convolution (BASELINE configs[1])")),
                "wavelet": args.wavelet, "levels": J, "n": n, "batch_per_gpu": Bl,
                "signals_per_launch": B, "global_batch": Bl * world, "arith": args.arith,
                "parallelism": f"dp{world} (batch sharded, no data-path collective)",
            },
            "max_recon_error": err,
            "recon_rms": rms,
            "recon_error_note": ("max_recon_error = max |x - inverse(forward(x))| over every sample "
                                 "of the step (absolute; inputs uniform in [-1, 1)); recon_rms = "
                                 "its root mean square. The STRICT contract reproduces JWave's "
                                 "DIRECT forward (other_arith.spot_check_vs_oracle) and inverse "
                                 "(tests/test_modwt_gpu.py) bit for bit, so JWave's own "
                                 "reconstruction at this configuration has the same error class"),
            "spot_check_vs_oracle": check,
            "roofline": {
                "bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": per_launch,
                "fwd_ms": round(fwd_ms, 3), "inv_ms": round(inv_ms, 3),
                "step_achieved": round(2 * per_launch / ((fwd_ms + inv_ms) * 1e-3) / 1e9, 1),
                "step_frac": round(2 * per_launch / ((fwd_ms + inv_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "note": ("achieved = algorithmic bytes per launch (8*(1+(J+1)) B/sample x B*N) / "
                         "average launch time from HIP events on the launch stream; traffic = "
                         "rocprofv3 FETCH_SIZE*2 + WRITE_SIZE per launch (profiles/)"),
            },
            "cpu_baseline": None,
            "other_arith": alt,
        }
        if world == 1 and not args.no_check:
            out["host_path"], out["auto_path"] = extra_paths()
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.wavelet, n, J)
        out.update(REHEARSAL)
        print(json.dumps(out), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
