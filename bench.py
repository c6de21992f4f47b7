"""WAM attribution throughput bench on MI355X (the BASELINE.json metric and its five configs).

    python bench.py [--config c2] [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workloads (BASELINE.json `configs`; synthetic data, random-init weights -- no
network). One STEP = one explainer call on the config's whole batch:
  c1  WAM-2D haar J=3 SmoothGrad n=25, ResNet-18 fp32, 1 image (the elephant crop fixture),
      numpy noise, legacy frame: the reference's own CPU-runnable case (CPU cross-check).
  c2  WAM-2D db4 J=3 SmoothGrad n=25, ResNet-50 (bf16, BN folded), batch 64 of 224^2, Philox
      noise, native frame E1 (the reference cannot run db4 SmoothGrad at 224).
      THE metric's config and the default.
  c3  WAM-1D db6 J=5 SmoothGrad n=25, FtEx audio CNN (fp32) on the mel front-end, batch 256 clips
      of 5 s at 16 kHz, Philox noise.
  c4  WAM-2D sym8 J=5 Integrated Gradients, 64 path steps, ResNet-50 (fp32, BN folded), batch 128
      of 512^2, native frame E2.
  c5  WAM-3D haar J=2 SmoothGrad n=25 (symmetric), Voxel3D CNN (fp32), batch 16 of 128^3, Philox
      noise, legacy in-loop averaging.
  c3-c5 state no reduced model precision, so their credited value runs the model in fp32 (the
  reference's); the bf16 model is reported beside it as variants.bf16_model.
Multi-GPU (one process per GPU, RCCL): the explainer itself shards ONE call of the batch with
dist=True -- c2 over the batch (each rank a contiguous image range, the per-sample batch-global
maxima combined by an all-reduce MAX, the rows gathered), c4 over the IG path steps as BASELINE
configs[3] names it (trapezoid partials summed by one fp32 all-reduce), c3/c5 over the noise
samples (partial accumulators summed by an all-reduce) -- so "scaling" is "strong" and value =
the call's attributions / max-over-ranks time. N > 1 also reports the collectives' time and a
weak-scaling figure (each rank its own batch, no collective) as secondary fields.

The JSON line also carries
  roofline      the dominant WAM kernel (largest total time), timed live with HIP events that
                libwam_hip.so records on the launch stream: SURVEY 8(d) algorithmic bytes per
                launch / mean launch time vs the 8 TB/s HBM peak; traffic = HBM bytes per launch
                from rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes that this run
                starts itself before it touches the GPU (one call of the same config with a stand-in
                model, so the WAM kernels see the same shapes), else null;
  cpu_baseline  the reference algorithm (oracle/wam_ref.py: per-sample loop, torch-CPU ptwt
                restatement, numpy legacy noise, numpy mosaic; fp32 model) on a bounded sample on
                the host cores, rank 0 at N=1 only;
  c2 extras     parity (GPU fp32 map vs that CPU reference map on the same images; bf16 + folded
                model vs fp32; Philox vs numpy noise), variant throughputs (fp32 model, model run
                as is under autocast), DWT->IDWT round-trip error, a measured copy ceiling.
"""
import argparse
import csv
import datetime
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

# MIOpen picks the bf16 model's convolution solvers by timing them on a process's first use (about
# a minute of warm-up on a fresh box). The bench starts from the find database of an
# MI355X run instead (wam_amd/data/miopen: MIOpen's own records, copied to a scratch directory it may
# update, removed at exit); this saves the solver timing, it does not remove the model's run-to-run
# spread (605-628 attr/s at c2 with or without it). A caller's MIOPEN_USER_DB_PATH wins.
if "MIOPEN_USER_DB_PATH" not in os.environ:
    _fdb = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wam_amd", "data", "miopen")
    if os.path.isdir(_fdb):
        import atexit
        _udb = tempfile.mkdtemp(prefix="wam_miopen_")
        for _f in os.listdir(_fdb):
            shutil.copy(os.path.join(_fdb, _f), _udb)
        os.environ["MIOPEN_USER_DB_PATH"] = _udb
        atexit.register(shutil.rmtree, _udb, True)

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    sys.stderr.write("[bench %6.1fs] %s\n" % (time.time() - _T0, msg))
    sys.stderr.flush()


def heartbeat(period=45.0):
    """A daemon thread that reports every `period` s, so long phases (MIOpen searches, profiler
    passes, the CPU baseline) are never mistaken for a hang."""
    import threading

    def run():
        while True:
            time.sleep(period)
            log("alive")
    threading.Thread(target=run, daemon=True).start()


# ============================================================================ configurations
class Workload:
    """One BASELINE config: inputs, model, explainer kwargs, units and algorithmic bytes."""

    def __init__(self, name, dim, metric, unit, n, n_steps, make_x, make_y, model, kw, model_dtype,
                 describe, dist_axis):
        self.name, self.dim, self.metric, self.unit = name, dim, metric, unit
        self.n, self.n_steps = n, n_steps          # batch items, noise samples / IG steps per item
        self.make_x, self.make_y, self.model, self.kw = make_x, make_y, model, kw
        self.model_dtype, self.describe, self.dist_axis = model_dtype, describe, dist_axis


def _elephant():
    crop = np.load(os.path.join(REPO, "tests", "golden", "elephant_224.npz"))["crop"].astype(np.float32) / 255.0
    mean = np.array([0.485, 0.456, 0.406], dtype=np.float32)[:, None, None]
    std = np.array([0.229, 0.224, 0.225], dtype=np.float32)[:, None, None]
    return torch.tensor(((crop.transpose(2, 0, 1) - mean) / std)[None])


def workload(name):
    import testmodels
    if name == "c1":
        return Workload("c1", 2, "WAM-2D attributions/sec @224^2 n_samples=25 (haar J=3 SmoothGrad, ResNet-18, 1 image)",
                        "attributions/s", 1, 25, _elephant, None, lambda: testmodels.resnet18(seed=0),
                        dict(wavelet="haar", J=3, method="smooth", mode="reflect", n_samples=25), "fp32",
                        "c1: WAM-2D haar J=3 SmoothGrad n=25, ResNet-18 (random init), 1 image 224x224 (elephant "
                        "crop), numpy legacy noise, legacy frame", "samples")
    if name == "c2":
        return Workload("c2", 2, "WAM-2D attributions/sec @224^2 n_samples=25 (db4 J=3 SmoothGrad, ResNet-50)",
                        "attributions/s", 64, 25,
                        lambda: torch.tensor(np.random.RandomState(1).standard_normal((64, 3, 224, 224))
                                             .astype(np.float32)),
                        lambda: [int(v) for v in np.random.RandomState(2).randint(0, 1000, 64)],
                        lambda: testmodels.resnet50(seed=0),
                        dict(wavelet="db4", J=3, method="smooth", mode="reflect", n_samples=25, noise="philox",
                             frame="native"), "bf16",
                        "c2: WAM-2D db4 J=3 SmoothGrad n_samples=25, batch 64 x 224x224, ResNet-50", "images")
    if name == "c3":
        return Workload("c3", 1, "WAM-1D attributions/sec, 5 s 16 kHz clips n_samples=25 (db6 J=5 SmoothGrad, FtEx)",
                        "attributions/s", 256, 25, lambda: testmodels.audio_clips(256),
                        lambda: [int(v) for v in np.random.RandomState(6).randint(0, 50, 256)],
                        lambda: testmodels.FtEx(seed=0),
                        dict(wavelet="db6", J=5, method="smooth", mode="reflect", n_samples=25, sample_rate=16000,
                             noise="philox"), "fp32",
                        "c3: WAM-1D db6 J=5 SmoothGrad n_samples=25, batch 256 x 80000 samples, FtEx audio CNN",
                        "samples")
    if name == "c4":
        return Workload("c4", 2, "WAM-2D attributions/sec @512^2 (sym8 J=5 Integrated Gradients, 64 steps, ResNet-50)",
                        "attributions/s", 128, 64,
                        lambda: torch.tensor(np.random.RandomState(4).standard_normal((128, 3, 512, 512))
                                             .astype(np.float32)),
                        lambda: [int(v) for v in np.random.RandomState(7).randint(0, 1000, 128)],
                        lambda: testmodels.resnet50(seed=0),
                        dict(wavelet="sym8", J=5, method="integratedgrad", mode="reflect", n_samples=64,
                             frame="native"), "fp32",
                        "c4: WAM-2D sym8 J=5 Integrated Gradients (64 path steps), batch 128 x 512x512, ResNet-50",
                        "samples")  # BASELINE configs[3]: path steps sharded, one fp32 all-reduce SUM
    if name == "c5":
        return Workload("c5", 3, "WAM-3D attributions/sec @128^3 n_samples=25 (haar J=2 SmoothGrad, Voxel3D)",
                        "attributions/s", 16, 25, lambda: testmodels.voxel_volumes(16),
                        lambda: [int(v) for v in np.random.RandomState(8).randint(0, 10, 16)],
                        lambda: testmodels.Voxel3D(seed=0),
                        dict(wavelet="haar", J=2, method="smooth", mode="symmetric", n_samples=25,
                             noise="philox"), "fp32",
                        "c5: WAM-3D haar J=2 SmoothGrad n_samples=25, batch 16 x 128^3, Voxel3D CNN", "samples")
    raise ValueError(name)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model-dtype", default=None, choices=["bf16", "fp32"], help="default: the config's")
    ap.add_argument("--sample-batch", type=int, default=None,
                    help="noise samples / IG steps per model call (default: ~832 images per call for c2/c4)")
    ap.add_argument("--no-bf16-handoff", action="store_true",
                    help="2D: fp32 model hand-off (cast / layout passes) instead of bf16 NHWC (A/B)")
    ap.add_argument("--no-optimize-model", action="store_true",
                    help="run the model as is under autocast instead of the BN-folded copy (model_opt.py)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"])
    ap.add_argument("--extras", default="auto", choices=["auto", "off"], help="c2 parity / variants / ceilings")
    ap.add_argument("--dist-axis", default=None, choices=["auto", "samples", "images"])
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds a collective may wait before the rank aborts (N > 1)")
    ap.add_argument("--rank-slice", default=None, metavar="N[,N...]",
                    help="one GPU: time the slice ONE rank of an N-GPU run would process, on the images and the "
                         "samples axis, and print the projected strong-scaling efficiency per N (no bench line)")
    ap.add_argument("--link-GBps", type=float, default=50.0,
                    help="--rank-slice: bus bandwidth assumed for the collectives' projection")
    ap.add_argument("--wam-probe", action="store_true", help=argparse.SUPPRESS)  # PMC child run
    # test-only: the process group's backend and every rank on cuda:0 (rehearsing the N > 1 path on
    # a one-GPU box); the driver's runs use the defaults (RCCL, one GPU per rank)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    ap.add_argument("--single-device", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def self_launch(args, argv):
    """`bench.py --gpus N` (N > 1) without a torch.distributed launcher: start one process per GPU
    with torch.distributed.run as a CHILD process -- before this process touches the GPU -- relay
    rank 0's JSON line and exit with the launcher's status."""
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd[1:])))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE)
    out = p.stdout.decode(errors="replace")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if lines:
        print(lines[-1])
        sys.stdout.flush()
    return p.returncode if lines or p.returncode else 1


# ============================================================================ explainer
def build_explainer(wl, dev, args, model=None, dist_on=False, model_dtype=None, optimize=None, noise=None,
                    n_local=None, axis=None):
    import wam_amd
    model_dtype = model_dtype or args.model_dtype or wl.model_dtype
    model = (model if model is not None else wl.model()).to(dev).eval()
    for p in model.parameters():
        p.requires_grad_(False)
    kw = dict(wl.kw)
    if noise is not None:
        kw["noise"] = noise
    ac = torch.bfloat16 if model_dtype == "bf16" else None
    if wl.dim == 2:
        opt = (not args.no_optimize_model) if optimize is None else optimize
        opt = opt and wl.name != "c1"
        cl = wl.name != "c1"
        if cl:
            model = model.to(memory_format=torch.channels_last)
        sb = args.sample_batch or _auto_sample_batch(wl, n_local or wl.n)
        return wam_amd.WaveletAttribution2D(model, sample_batch=sb, autocast_dtype=ac, channels_last=cl,
                                            optimize_model=opt, dist=True if dist_on else None,
                                            dist_axis=axis or args.dist_axis or wl.dist_axis,
                                            bf16_handoff=not args.no_bf16_handoff, **kw)
    if wl.dim == 1:
        return wam_amd.WaveletAttribution1D(model, sample_batch=args.sample_batch or 5, autocast_dtype=ac,
                                            dist=True if dist_on else None, **kw)
    return wam_amd.WaveletAttribution3D(model, sample_batch=args.sample_batch or 2, autocast_dtype=ac,
                                        dist=True if dist_on else None, **kw)


def _auto_sample_batch(wl, n_local):
    """~832 images per model call (the measured sweet spot for ResNet-50 at 224^2; 512^2 images
    count 5.2x), split evenly over the calls."""
    per = 832 if wl.name != "c4" else 160
    sb = max(1, min(wl.n_steps, -(-per // max(1, n_local))))
    calls = -(-wl.n_steps // sb)
    return -(-wl.n_steps // calls)


# ============================================================================ timing helpers
def kernel_table(records, steps):
    kern = {}
    for name, ms, nb in records:
        k = kern.setdefault(name, {"launches": 0, "total_ms": 0.0, "bytes": 0.0})
        k["launches"] += 1
        k["total_ms"] += ms
        k["bytes"] += nb
    for k in kern.values():
        k["mean_us"] = k["total_ms"] * 1e3 / k["launches"]
        k["GBps"] = k["bytes"] / (k["total_ms"] * 1e-3) / 1e9 if k["total_ms"] > 0 else 0.0
        k["bytes_per_launch"] = k["bytes"] / k["launches"]
    return kern


def unit_bytes(wl, kname, units_per_launch, lib_bytes, n_items):
    """SURVEY 8(d) algorithmic bytes of one launch where they differ from the library's own count:
    the fused noisy analyses (k_*<noise>) read the clean input once for all their samples, while
    8(d) counts 4 (P + K) per (item x sample) unit, as the reference materialises each noisy input.
    A kernel that covers only part of each item (the 1D interior / boundary tiles) keeps its share:
    the library's bytes over the whole-item library count."""
    from wam_amd import plan as P
    if wl.name == "c2" and kname.split("<")[0] in ("k_plane_syn", "k_plane_maps"):
        K = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda").coeff_numel
        px = 2 if "bf16" in kname else 4  # the bf16 hand-off forms move 2 B per pixel
        per_unit = {"k_plane_syn": 3 * (4 * K + px * 224 * 224),
                    "k_plane_maps": px * 3 * 224 * 224 + 4 * K}[kname.split("<")[0]]
        return per_unit * units_per_launch
    if not kname.endswith("<noise>"):
        return None
    geo = {"c1": (2, (224, 224), 3, "haar", "reflect", 3), "c2": (2, (224, 224), 3, "db4", "reflect", 3),
           "c3": (1, (80000,), 5, "db6", "reflect", 1), "c5": (3, (128, 128, 128), 2, "haar", "symmetric", 1)}
    if wl.name not in geo:
        return None
    nd, shape, J, wav, mode, C = geo[wl.name]
    K = P.get_plan(nd, shape, J, wav, mode, "cuda").coeff_numel * C  # per item (all channels)
    Pn = int(np.prod(shape)) * C
    whole = 4.0 * (n_items * Pn + units_per_launch * K)                # the library's whole-item count
    return lib_bytes / whole * 4.0 * units_per_launch * (Pn + K)


# FFT front-end kernels (wam_amd/csrc/melspec.hip): VALU / LDS bound by construction (two to three
# 512-point FFTs per 4 KB frame), reported beside the HBM roofline rather than as its kernel, on
# their own compute roofline (mel_roofline)
VALU_BOUND = ("k_mel_fwd", "k_mel_adj", "k_mel_fold")
FP32_PEAK_TFLOPS = 157.3          # MI355X vector fp32 (MI355X_MICROARCH.md)
LDS_PEAK_TBS = 128 * 256 * 2.4e9 / 1e12   # 128 B/clk/CU (ds_read_b32 / mixed rate) x 256 CUs x 2.4 GHz


def mel_frame_model(n_fft, n_mels, nnz, adjoint):
    """FLOPs and LDS bytes per frame of the mel kernels (the model the report prices them on):
    an M = n_fft / 2 point complex FFT = 5 M log2 M flops in ceil(log2 M / 3) radix-8 Stockham
    stages, each reading and writing M complex values (8 B) plus 7/8 M table twiddles after the first;
    the real-spectrum unpack 10 flops and 3 LDS reads per bin, |X|^2 3 flops per bin, the band sums
    2 flops and 12 B per filterbank nonzero; the adjoint adds the second FFT, the by-bin sums, the
    A = 2 dL/dP X products (4 flops per bin) and the Hermitian pack (10 flops, 2 reads per point)."""
    M = n_fft // 2
    lg = int(np.log2(M))
    stages = -(-lg // 3)
    fft_flops = 5.0 * M * lg
    fft_lds = stages * 16.0 * M + (stages - 1) * 7.0 * M
    bins = M + 1
    flops = n_fft + fft_flops + 13.0 * bins + 2.0 * nnz + 2.0 * n_mels
    lds = 8.0 * M + fft_lds + 24.0 * bins + 4.0 * bins + 12.0 * nnz
    if adjoint:
        flops += fft_flops + 2.0 * nnz + 4.0 * bins + 10.0 * M + n_fft + 4.0 * n_mels
        lds += fft_lds + 12.0 * nnz + 8.0 * bins + 16.0 * M + 8.0 * M + 4.0 * n_mels
    return flops, lds


def mel_roofline(wl, kern):
    """compute roofline of the mel kernels at c3: FLOPs / frame (model above), achieved TFLOP/s vs the
    fp32 vector peak and LDS bytes / s vs the LDS array rate"""
    if wl.name != "c3":
        return None
    from wam_amd.melspec import MelTables
    n_fft, n_mels, T = 1024, 128, 80000
    F = T // (n_fft // 2) + 1
    nnz = MelTables.get(n_fft, n_mels, 16000, "cpu").nnz
    out = {}
    for n in ("k_mel_fwd", "k_mel_adj"):
        if n not in kern:
            continue
        k = kern[n]
        per_item = 4.0 * T * (2 if n == "k_mel_adj" else 1) + 4.0 * F * n_mels   # the library's bytes per clip
        frames = k["bytes_per_launch"] / per_item * F
        fl, lb = mel_frame_model(n_fft, n_mels, nnz, n == "k_mel_adj")
        sec = k["mean_us"] * 1e-6
        out[n] = {"frames_per_launch": round(frames), "flops_per_frame": round(fl), "lds_bytes_per_frame": round(lb),
                  "mean_us": round(k["mean_us"], 2), "achieved_tflops": round(frames * fl / sec / 1e12, 2),
                  "fp32_peak_tflops": FP32_PEAK_TFLOPS,
                  "frac_fp32": round(frames * fl / sec / 1e12 / FP32_PEAK_TFLOPS, 4),
                  "lds_tbs": round(frames * lb / sec / 1e12, 2), "lds_peak_tbs": round(LDS_PEAK_TBS, 1),
                  "frac_lds": round(frames * lb / sec / 1e12 / LDS_PEAK_TBS, 4)}
    if "k_mel_fold" in kern:
        out["k_mel_fold"] = {"mean_us": round(kern["k_mel_fold"]["mean_us"], 2),
                             "note": "frames 0 and F-1 of every clip recomputed for the reflect folds"}
    return out or None


def traffic_table(kern, traffic):
    """per kernel: PMC HBM bytes per launch vs the library's algorithmic bytes per launch"""
    out = {}
    for n, k in kern.items():
        pc = (traffic or {}).get("per_call_bytes", {}).get(n)
        if pc is None or not k.get("bytes_per_launch"):
            continue
        out[n] = {"pmc_bytes": pc, "algorithmic_bytes": round(k["bytes_per_launch"]),
                  "ratio": round(pc / k["bytes_per_launch"], 3)}
    return out or None


def roofline(wl, kern, steps, units_per_step, traffic, n_items):
    hbm = {n: k for n, k in kern.items() if n not in VALU_BOUND} or kern
    dom = max(hbm, key=lambda n: hbm[n]["total_ms"])
    kd = kern[dom]
    units_per_launch = units_per_step * steps / kd["launches"]
    ub = unit_bytes(wl, dom, units_per_launch, kd["bytes_per_launch"], n_items)
    bpl = ub if ub else kd["bytes_per_launch"]
    achieved = bpl / (kd["mean_us"] * 1e-6) / 1e9
    tr = None
    if traffic and dom in traffic.get("per_call_bytes", {}):
        tr = traffic["per_call_bytes"][dom]
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr,
            "traffic_per_launch_detail": (traffic or {}).get("per_call", {}).get(dom),
            "traffic_source": (traffic or {}).get("source"),
            "bytes_per_launch": round(bpl), "units_per_launch": units_per_launch,
            "bytes_basis": "SURVEY 8(d) per (item x sample) unit" if ub else "library algorithmic bytes (4 (in + out))",
            "library_bytes_per_launch": round(kd["bytes_per_launch"]), "library_GBps": round(kd["GBps"], 1),
            "mean_us": round(kd["mean_us"], 2),
            "wam_ms_per_step": round(sum(k["total_ms"] for k in kern.values()) / steps, 3),
            "valu_bound_kernels": mel_roofline(wl, kern),
            "traffic_by_kernel": traffic_table(kern, traffic),
            "kernels": {n: {kk: round(vv, 3) for kk, vv in k.items()} for n, k in
                        sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"])}}


def timed(fn, steps, warmup, world, dev):
    from wam_amd import plan as P
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    P.timing_drain()
    P.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    P.timing_enable(False)
    records = P.timing_drain()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    return dt, records, out


# ============================================================================ live PMC traffic
def _short_kernel(name):
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from pmc_summary import short
    return short(name)


def _pmc_pass(counter, config, outdir, extra=()):
    exe = shutil.which("rocprofv3")
    log("rocprofv3 --pmc %s pass (child run of %s)" % (counter, config))
    cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", counter, "--kernel-include-regex", "k_[a-z0-9_]+",
           "--output-format", "csv", "-d", outdir, "-o", "run", "--", sys.executable, os.path.join(REPO, "bench.py"),
           "--config", config, "--wam-probe"] + list(extra)
    env = dict(os.environ, TMPDIR="/tmp")
    p = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=200)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    log("rocprofv3 --pmc %s pass done (rc %d)" % (counter, p.returncode))
    if p.returncode != 0 or not files:
        raise RuntimeError("rocprofv3 --pmc %s failed (rc %d): %s" % (counter, p.returncode,
                                                                       p.stdout.decode(errors="replace")[-600:]))
    acc = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = _short_kernel(row["Kernel_Name"])
            if k is None:
                continue
            a = acc.setdefault(k, {})
            d = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(a))
            a[d] = a.get(d, 0.0) + float(row["Counter_Value"]) * 1024.0  # KiB, summed over dimensions
    return {k: (len(v), sum(v.values())) for k, v in acc.items()}


def live_pmc(config, extra=()):
    """HBM traffic per WAM-kernel launch: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; they
    do not fit one pass) over one call of this config with a stand-in model, started before this
    process touches the GPU. FETCH_SIZE is doubled (gfx950 counts 16-B-per-lane streaming reads at
    half, MI355X_MICROARCH.md HBM section); WRITE_SIZE is taken as is."""
    if not shutil.which("rocprofv3") or not shutil.which("timeout"):
        return None
    tmp = tempfile.mkdtemp(prefix="wam_pmc_", dir="/tmp")
    try:
        fetch = _pmc_pass("FETCH_SIZE", config, os.path.join(tmp, "f"), extra)
        write = _pmc_pass("WRITE_SIZE", config, os.path.join(tmp, "w"), extra)
    except Exception as e:  # profiler unavailable / refused: report null traffic, say why
        return {"error": str(e)[:400]}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    out = {"source": "live rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE passes over one %s call "
                     "(stand-in model)" % config, "per_call_bytes": {}, "per_call": {}}
    for k in sorted(set(fetch) | set(write)):
        nf, bf = fetch.get(k, (0, 0.0))
        nw, bw = write.get(k, (0, 0.0))
        rd, wr = 2.0 * bf / max(nf, 1), bw / max(nw, 1)
        out["per_call"][k] = {"launches": max(nf, nw), "read_bytes": round(rd), "write_bytes": round(wr)}
        out["per_call_bytes"][k] = round(rd + wr)
    return out


class _StandIn(torch.nn.Module):
    """Tiny model with the config's input/output shapes (PMC child runs: WAM kernels only)."""

    def __init__(self, dim, n_classes):
        super().__init__()
        conv = {1: torch.nn.Conv2d, 2: torch.nn.Conv2d, 3: torch.nn.Conv3d}[dim]
        self.conv = conv(1 if dim != 2 else 3, 4, 3, 2, 1)
        self.fc = torch.nn.Linear(4, n_classes)

    def forward(self, x):
        h = torch.tanh(self.conv(x))
        return self.fc(h.flatten(2).mean(-1))


def wam_probe(args):
    wl = workload(args.config)
    dev = torch.device("cuda", 0)
    x, y = wl.make_x(), (wl.make_y() if wl.make_y else 0)
    model = _StandIn(wl.dim, 1000 if wl.dim == 2 else 50)
    if wl.name == "c2":  # the headline's model precision and execution: the bf16 NHWC hand-off kernels
        ex = build_explainer(wl, dev, args, model=model)
    else:
        ex = build_explainer(wl, dev, args, model=model, model_dtype="fp32", optimize=False)
    ex(x.to(dev), y)
    torch.cuda.synchronize()


# ============================================================================ CPU baseline
def _cpu_threads():
    cores = len(os.sched_getaffinity(0))
    return min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))


def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        return "unknown CPU"


def cpu_baseline(wl, seconds, x, y):
    """The reference algorithm (oracle/wam_ref.py) on the host cores on a bounded sample of the
    workload, extrapolated per attribution. Returns (record, (items, samples, cpu map) or None)."""
    from oracle import wam_ref
    cores = _cpu_threads()
    torch.set_num_threads(cores)
    model = wl.model().eval()
    kw = {k: v for k, v in wl.kw.items() if k not in ("method", "noise", "n_samples")}
    if wl.dim == 2:
        fn = wam_ref.smooth_2d if wl.kw["method"] == "smooth" else wam_ref.ig_2d
        if wl.kw["method"] != "smooth":
            kw = {k: v for k, v in kw.items() if k in ("wavelet", "J", "mode", "frame")}
    elif wl.dim == 1:
        fn = wam_ref.smooth_1d
    else:
        fn = wam_ref.smooth_3d
    run = lambda n_img, n_s: fn(model, x[:n_img], y[:n_img] if isinstance(y, list) else y, n_samples=n_s, **kw)
    for _ in range(2):  # the first call pays one-time CPU start-up costs
        t0 = time.perf_counter()
        run(1, 1 if wl.kw["method"] == "smooth" else 2)
        per = max(time.perf_counter() - t0, 1e-3)
    if wl.kw["method"] != "smooth":
        per /= 2
    n_s = wl.n_steps if seconds / per >= wl.n_steps else int(max(2, seconds / per))
    n_img = int(max(1, min(wl.n, seconds / per / n_s)))
    t0 = time.perf_counter()
    out = run(n_img, n_s)
    dt = time.perf_counter() - t0
    per = dt / (n_img * n_s)   # seconds per (item x sample / step) unit
    rec = {"value": n_img * n_s / dt / wl.n_steps, "unit": wl.unit, "cores": cores, "kind": "port",
           "sample": "oracle/wam_ref (reference glue restated on torch-CPU ptwt, numpy legacy noise), fp32 model, "
                     "%d item(s) x %d %s of the %s workload in %.1f s on %d thread(s) of %s%s" % (
                         n_img, n_s, "noise samples" if wl.kw["method"] == "smooth" else "path steps", wl.name, dt,
                         cores, _cpu_model_name(),
                         "" if n_s == wl.n_steps else ", extrapolated to %d per attribution" % wl.n_steps)}
    return rec, (n_img, n_s, out, per, run)


# ============================================================================ c2 extras
def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(1e-30, np.linalg.norm(b)))


def _top_iou(a, b, frac=0.10):
    out = []
    for u, v in zip(a.reshape(a.shape[0], -1), b.reshape(b.shape[0], -1)):
        k = max(1, int(frac * u.size))
        su, sv = set(np.argsort(-u)[:k].tolist()), set(np.argsort(-v)[:k].tolist())
        out.append(len(su & sv) / len(su | sv))
    return float(np.mean(out))


def _cmp(a, b, what):
    """a vs the reference b: relative L2, max |a - b| (unrounded) and the same over max |b|, top-10 %
    IoU of the per-item rankings"""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    mx = float(np.abs(a - b).max())
    return {"what": what, "rel_l2": float("%.4g" % _rel_l2(a, b)), "max_abs": float("%.4g" % mx),
            "max_abs_over_max_ref": float("%.4g" % (mx / max(1e-300, float(np.abs(b).max())))),
            "top10_iou": round(_top_iou(a, b), 4), "items": int(a.shape[0])}


def _main_map(o):
    """the attribution map of a call's output (1D: (mel maps, coefficient maps) -> the mel maps)"""
    return np.asarray(o[0] if isinstance(o, tuple) else o)


# parity blocks cover at least this many items; when the cpu_baseline sample holds fewer, the CPU
# reference runs again on that many items with fewer noise samples / path steps (same algorithm)
PARITY_MIN_ITEMS = {"c3": 4, "c4": 4, "c5": 2}


def parity_extras(wl, dev, args, ex, x, y, cpu_ref):
    """c3 / c4 / c5: the GPU path (fp32 model as is, the reference's numpy noise for SmoothGrad) vs
    the CPU reference path's own output (cpu_baseline) on the same items, samples / path steps and
    weights; where the headline model runs in bf16, the headline map vs that fp32 map too."""
    n_img, n_s, ref, per, run = cpu_ref
    want = min(wl.n, PARITY_MIN_ITEMS.get(wl.name, 1))
    if n_img < want:
        n_img = want
        n_s = int(max(2, min(wl.n_steps, args.cpu_seconds * 1.5 / per / want)))
        log("%s parity: CPU reference on %d items x %d %s" % (wl.name, n_img, n_s,
                                                              "samples" if wl.kw["method"] == "smooth" else "steps"))
        ref = run(n_img, n_s)
    yy = y[:n_img] if isinstance(y, list) else y
    smooth = wl.kw.get("method", "smooth") == "smooth"
    ex32 = build_explainer(wl, dev, args, model_dtype="fp32", optimize=False, noise="numpy" if smooth else None)
    ex32.n_samples = n_s
    got = ex32(x[:n_img], yy)
    par = {"gpu_fp32_vs_cpu_reference": _cmp(_main_map(got), _main_map(ref),
                                             "GPU (fp32 model as is%s) vs the CPU reference path (cpu_baseline's own "
                                             "output), same items / weights / %s" % (
                                                 ", numpy noise" if smooth else "",
                                                 "noise" if smooth else "path steps"))}
    par["gpu_fp32_vs_cpu_reference"]["n_samples"] = n_s
    head_dtype = args.model_dtype or wl.model_dtype
    runs = []
    if head_dtype == "bf16" or wl.dim == 2:   # c3 / c5 headline at fp32 = the fp32 run above
        runs.append(("headline_vs_fp32_as_is", {}, "headline model (%s%s)" % (
            head_dtype, ", BN-folded" if wl.dim == 2 else "")))
    if head_dtype != "bf16":
        runs.append(("bf16_variant_vs_fp32_as_is", {"model_dtype": "bf16"}, "bf16 variant model (%s)" % (
            "BN-folded" if wl.dim == 2 else "autocast")))
    for tag, kw, what in runs:
        hd = build_explainer(wl, dev, args, noise="numpy" if smooth else None, **kw)
        hd.n_samples = n_s
        par[tag] = _cmp(_main_map(hd(x[:n_img], yy)), _main_map(got),
                        "%s vs fp32 model as is, same items and %s: model precision / folding only" % (
                            what, "noise" if smooth else "path steps"))
        del hd
    del ex32
    torch.cuda.empty_cache()
    return par


def c2_extras(wl, dev, args, ex, x, y, cpu_ref):
    """Parity numbers on the headline configuration, variant throughputs and ceilings."""
    import wam_amd
    from wam_amd import plan as P
    extras = {}
    n_sub = 8
    xs, ys = x[:n_sub], y[:n_sub]
    # the headline map (bf16, folded model, Philox) on the subset
    head = ex(xs, ys)
    fp32_philox = build_explainer(wl, dev, args, model_dtype="fp32", optimize=False)
    b = fp32_philox(xs, ys)
    fp32_numpy = build_explainer(wl, dev, args, model_dtype="fp32", optimize=False, noise="numpy")
    c = fp32_numpy(xs, ys)
    par = {"bf16_folded_vs_fp32": _cmp(head, b, "headline map (bf16, BN-folded model, Philox) vs fp32 model as is, "
                                              "same Philox noise: model precision / folding only"),
           "philox_vs_numpy_noise": _cmp(b, c, "fp32 model, Philox vs numpy legacy noise: Monte-Carlo spread of "
                                              "two 25-sample SmoothGrad estimates (context, not an error)")}
    if cpu_ref is not None:
        n_img, n_s, ref = cpu_ref[:3]
        ex_ref = build_explainer(wl, dev, args, model_dtype="fp32", optimize=False, noise="numpy")
        ex_ref.n_samples = n_s
        got = ex_ref(x[:n_img], y[:n_img])
        par["gpu_fp32_vs_cpu_reference"] = _cmp(got, ref, "GPU (fp32 model, numpy noise) vs the CPU reference path "
                                                          "(cpu_baseline's own output), same images / noise / "
                                                          "weights; bar rel L2 <= 2e-2, max-abs <= 5e-2")
        par["gpu_fp32_vs_cpu_reference"]["n_samples"] = n_s
    extras["parity"] = par
    del fp32_philox, fp32_numpy
    torch.cuda.empty_cache()
    # variant throughputs (short runs of the full call)
    if args.extras == "auto":
        var = {}
        for tag, kw in (("fp32_model_folded", dict(model_dtype="fp32")),
                        ("bf16_autocast_model_as_is", dict(model_dtype="bf16", optimize=False))):
            log("variant %s" % tag)
            e = build_explainer(wl, dev, args, **kw)
            dt, _, _ = timed(lambda: e(x, y), 2, 1, 1, dev)
            var[tag] = {"value": round(wl.n * 2 / dt, 3), "ms_per_step": round(dt / 2 * 1e3, 2), "steps": 2}
            del e
            torch.cuda.empty_cache()
        extras["variants"] = var
    # DWT -> IDWT round trip at the c2 geometry (north_star: "also reported")
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", dev)
    xd = x.to(dev).reshape(-1, 224, 224)
    r = p.waverec(p.wavedec(xd), xd.shape[0])[0][:, :224, :224]
    extras["roundtrip"] = {"max_abs": float((r - xd).abs().max()), "max_abs_input": float(xd.abs().max()),
                           "what": "db4 J=3 reflect wavedec2 -> waverec2 of the 64x3 input planes (fp32)"}
    # copy ceiling: libwam_hip.so's streaming copy (16-B loads / stores) and torch's, 2 GiB each
    from wam_amd._lib import check as _check, lib as _lib, ptr as _ptr, stream_of as _stream_of
    a = torch.empty(512 << 20, dtype=torch.float32, device=dev)
    bb = torch.empty_like(a)
    nbytes = a.numel() * 4
    ceil = {}
    for tag, fn in (("k_copy", lambda: _check(_lib.wam_copy(nbytes, _ptr(a), _ptr(bb), _stream_of(dev)))),
                    ("torch_copy", lambda: bb.copy_(a))):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        ceil[tag + "_GBps"] = round(2 * nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9, 1)
    extras["copy_ceiling"] = dict(ceil, bytes=2 * nbytes, what="2 GiB device copy (read + write), mean of 10")
    del a, bb
    return extras


def collectives_timing(wl, dev, world, axis):
    """The sharded call's collectives alone, at its sizes (20 reps after one warm-up)."""
    from wam_amd import engine, plan as P
    shard = engine.Shard(True)
    ops = []
    if axis == "images":
        H = 224 if wl.name != "c4" else 512
        nb = 3 * wl.kw["J"] + 1
        lo, hi = shard.range(wl.n)
        t = torch.rand(wl.n_steps, nb, device=dev)
        rows = torch.zeros(hi - lo, H * H, dtype=torch.float64, device=dev)
        ops.append(("all_reduce_max_band_maxima", lambda: shard.all_reduce_max(t)))
        ops.append(("all_gather_frame_rows", lambda: shard.all_gather_rows(rows, wl.n)))
        out_bytes = {"all_reduce_max_band_maxima_bytes": int(t.numel() * 4),
                     "all_gather_frame_rows_bytes": int(-(-wl.n // world) * world * H * H * 8)}
    else:
        if wl.dim == 1:
            p = P.get_plan(1, (80000,), wl.kw["J"], wl.kw["wavelet"], wl.kw["mode"], dev)
            numel = wl.n * (p.coeff_numel + (80000 // 512 + 1) * 128)
            dt = torch.float32
        elif wl.dim == 3:
            numel, dt = wl.n * 128 ** 3, torch.float32
        elif wl.name == "c4":  # IG: the fp32 trapezoid accumulator of the whole batch
            numel, dt = wl.n * 512 * 512, torch.float32
        else:
            numel, dt = wl.n * 224 * 224, torch.float64
        acc = torch.zeros(numel, dtype=dt, device=dev)
        ops.append(("all_reduce_sum_accumulators", lambda: shard.all_reduce_sum(acc)))
        out_bytes = {"all_reduce_sum_accumulators_bytes": int(numel * acc.element_size())}
    out = dict(out_bytes)
    for tag, fn in ops:
        fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize(dev)
        out[tag + "_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
    return out


# The sharding axis per (config, world size) that the single-GPU rank-slice projection measured
# faster (bench.py --rank-slice); other N use the config's default axis
MEASURED_AXIS = {
    "c2": {2: "samples", 4: "images", 8: "images"},   # profiles/r06e_rank_slice_c2.log
}


# ============================================================================ rank-slice projection
def _slice_workload(wl, n_img, n_steps):
    """wl restricted to its first n_img items and n_steps noise samples / IG steps."""
    import copy
    w = copy.copy(wl)
    w.n, w.n_steps = n_img, n_steps
    w.kw = dict(wl.kw, n_samples=n_steps)
    return w


def _collective_bytes(wl, axis, world):
    """Bytes each rank's collectives move per call (ring algorithms: all-gather (N-1)/N of the
    whole, all-reduce 2 (N-1)/N), the sizes of collectives_timing / DESIGN.md section 6."""
    f = (world - 1) / world
    if axis == "images":
        H = 224 if wl.name != "c4" else 512
        rows = -(-wl.n // world) * world * H * H * 8           # fp64 frame rows, all-gathered
        return f * rows + 2 * f * wl.n_steps * (3 * wl.kw["J"] + 1) * 4
    if wl.dim == 1:
        numel = wl.n * (80052 + 157 * 128)
        return 2 * f * numel * 4
    if wl.dim == 3:
        return 2 * f * wl.n * 128 ** 3 * 4
    if wl.name == "c4":
        return 2 * f * wl.n * 512 * 512 * 4
    return 2 * f * wl.n * 224 * 224 * 8


def rank_slice(args, wl):
    """Single-GPU strong-scaling projection: for every N the slice the busiest
    rank processes -- images axis: ceil(n / N) items x all samples; samples axis: all items x
    ceil(S / N) samples -- timed alone on this GPU with its own model batch; projected N-GPU step =
    slice time + the collectives' bytes at --link-GBps; efficiency = T_1 / (N * T_N)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import wam_amd  # noqa: F401
    x, y = wl.make_x(), (wl.make_y() if wl.make_y else None)
    xd = x.to(dev)
    steps, warm = args.steps, args.warmup

    def run(w, n_img):
        ex = build_explainer(w, dev, args, n_local=n_img)
        yy = y[:n_img] if isinstance(y, list) else y
        dt, _, _ = timed(lambda: ex(xd[:n_img], yy), steps, warm, 1, dev)
        sb = getattr(ex, "sample_batch", None)
        del ex
        torch.cuda.empty_cache()
        return dt / steps, sb

    t1, sb1 = run(wl, wl.n)
    rows = []
    axes = ["images", "samples"] if wl.dim == 2 else ["samples"]
    for N in [int(v) for v in args.rank_slice.split(",")]:
        for axis in axes:
            if axis == "images":
                w = _slice_workload(wl, -(-wl.n // N), wl.n_steps)
            else:
                w = _slice_workload(wl, wl.n, -(-wl.n_steps // N))
            log("rank slice N=%d %s axis: %d items x %d samples" % (N, axis, w.n, w.n_steps))
            ts, sb = run(w, w.n)
            cb = _collective_bytes(wl, axis, N)
            tc = cb / (args.link_GBps * 1e9)
            tn = ts + tc
            rows.append({"n_gpus": N, "axis": axis, "slice_items": w.n, "slice_samples": w.n_steps,
                         "model_batch": (sb or 0) * w.n, "slice_ms": round(ts * 1e3, 2),
                         "collective_MB": round(cb / 1e6, 2), "collective_ms_model": round(tc * 1e3, 3),
                         "projected_value": round(wl.n / tn, 3),
                         "projected_efficiency": round(t1 / (N * tn), 4)})
    best = {}
    for r in rows:
        if r["n_gpus"] not in best or r["projected_value"] > best[r["n_gpus"]]["projected_value"]:
            best[r["n_gpus"]] = r
    print(json.dumps({"config": wl.name, "metric": wl.metric, "one_gpu": {"ms_per_step": round(t1 * 1e3, 2),
                      "value": round(wl.n / t1, 3), "model_batch": (sb1 or 0) * wl.n},
                      "link_GBps_assumed": args.link_GBps, "steps": steps, "warmup": warm, "slices": rows,
                      "best_axis": {str(k): v["axis"] for k, v in sorted(best.items())}}))
    return 0


# ============================================================================ main
def main():
    args = parse()
    if args.wam_probe:
        return wam_probe(args)
    heartbeat()
    if args.rank_slice:
        return rank_slice(args, workload(args.config))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return self_launch(args, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch one process per GPU)" % (args.gpus, world))
    if args.single_device:
        local = 0
    wl = workload(args.config)
    traffic = None
    if rank == 0 and world == 1 and args.pmc == "auto":
        # child processes, BEFORE this process touches the GPU
        traffic = live_pmc(args.config, ["--no-bf16-handoff"] if args.no_bf16_handoff else [])
    if world > 1:
        torch.cuda.set_device(local)
        # a collective that does not complete within the timeout aborts the rank with the
        # collective's name (RCCL watchdog) instead of hanging until the driver kills the run
        tmo = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group("gloo", timeout=tmo)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import wam_amd  # noqa: F401  (fails loudly without libwam_hip.so)
    from wam_amd import engine

    x, y = wl.make_x(), (wl.make_y() if wl.make_y else None)
    if y is None:  # c1: the model's own top class (as the reference demo does)
        with torch.no_grad():
            y = int(wl.model()(x).argmax().item())
    xd = x.to(dev)
    shard_on = world > 1
    axis = args.dist_axis or MEASURED_AXIS.get(wl.name, {}).get(world) or wl.dist_axis
    if wl.dim != 2 or axis == "auto":
        axis = "images" if (wl.dim == 2 and wl.n >= world) else "samples"
    n_local, s_local = wl.n, wl.n_steps
    if shard_on:
        lo, hi = engine.Shard.range_of(rank, world, wl.n if axis == "images" else wl.n_steps)
        if axis == "images":
            n_local = hi - lo
        else:
            s_local = hi - lo
    # the sample batch is sized from the largest rank's image count, the same on every rank
    ex = build_explainer(wl, dev, args, dist_on=shard_on, n_local=-(-wl.n // world) if axis == "images" else wl.n,
                         axis=axis)
    log("%s: %d warm-up + %d timed steps on %d GPU(s)" % (wl.name, args.warmup, args.steps, world))
    dt, records, out = timed(lambda: ex(xd, y), args.steps, args.warmup, world, dev)
    assert out is not None
    first = out[0] if isinstance(out, tuple) else out
    assert np.isfinite(np.asarray(first)).all()
    kern = kernel_table(records, args.steps)
    units_per_step = n_local * s_local  # (item x sample) units this rank's launches processed
    roof = roofline(wl, kern, args.steps, units_per_step, traffic, n_local)
    if traffic and "error" in traffic:
        roof["traffic_error"] = traffic["error"]

    log("timed: %.1f ms per step" % (dt / args.steps * 1e3))
    secondary = {}
    # the drop-in caller hands the explainer a host tensor (lib/wam_2D.py:392,114); the class moves
    # it once per call. The timed steps start from an HBM-resident x; the host -> device copy of the
    # same (pageable) tensor is timed here and reported beside the value, never folded into it.
    h2d = []
    for _ in range(5):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        x.to(dev)
        torch.cuda.synchronize(dev)
        h2d.append(time.perf_counter() - t0)
    h2d_s = sorted(h2d)[2]
    secondary["h2d_input"] = {
        "ms": round(h2d_s * 1e3, 3), "bytes": int(x.numel() * x.element_size()),
        "GB_per_s": round(x.numel() * x.element_size() / h2d_s / 1e9, 2),
        "value_including_h2d": round(n_local / (dt / args.steps + h2d_s), 3),
        "what": "median of 5 host->device copies of the call's (pageable) input, as the drop-in caller passes it; "
                "value_including_h2d = this rank's items / (ms_per_step + that copy)"}
    if wl.kw.get("noise", "numpy") == "numpy" and wl.kw.get("method") == "smooth":
        # parity-mode noise: the legacy numpy stream is drawn on the host once per (seed, shape,
        # batch) and replayed from the device afterwards (engine.LegacyNoise); a first ("cold")
        # call pays the host generation
        engine.clear_noise_cache()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ex(xd, y)
        torch.cuda.synchronize(dev)
        secondary["noise_cache"] = {
            "cold_call_ms": round((time.perf_counter() - t0) * 1e3, 2), "warm_call_ms": round(dt / args.steps * 1e3, 2),
            "what": "timed calls replay the reference's legacy numpy noise stream from the device (drawn once per "
                    "seed / shape / batch, scaled per call, bit-exact); cold_call_ms = one call after clearing it"}
    if wl.dim == 2:
        log(".scales host copy")
        # .scales (lib/wam_2D.py:413,457): the reprojection kernel runs inside every timed call;
        # its float64 host copy is made on first access -- its cost, outside the timed region:
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        sc = ex.scales
        secondary["scales_host_copy"] = {
            "ms": round((time.perf_counter() - t0) * 1e3, 2), "bytes": int(sc.nbytes),
            "what": ".scales reprojection (k_reproject) runs in every timed call on the device; this is the one-off "
                    "device -> host float64 copy on first access of ex.scales, not in the timed region"}
        del sc
    if world > 1:
        log("collectives timing")
        secondary["collectives"] = collectives_timing(wl, dev, world, axis)
    if world > 1 and args.extras == "auto":
        log("weak scaling: each rank its own %d-item batch" % wl.n)
        exw = build_explainer(wl, dev, args, dist_on=False)  # each rank its own batch, no collective
        dtw, _, _ = timed(lambda: exw(xd, y), 2, 1, world, dev)
        secondary["weak_scaling"] = {"value": round(wl.n * 2 * world / dtw, 3), "ms_per_step": round(dtw / 2 * 1e3, 2),
                                     "what": "each rank explains its own %d-item batch (no collective), 2 steps"
                                             % wl.n}

    cpu, cpu_ref = None, None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        log("cpu baseline (~%.0f s)" % args.cpu_seconds)
        cpu, cpu_ref = cpu_baseline(wl, args.cpu_seconds, x, y)
    extras = {}
    if rank == 0 and world == 1 and wl.name == "c2" and args.extras == "auto":
        log("c2 extras: parity, variants, round trip, copy ceiling")
        extras = c2_extras(wl, dev, args, ex, xd, y, cpu_ref)
    elif cpu_ref is not None and wl.name in ("c1",):
        n_img, n_s, ref = cpu_ref[:3]
        extras["parity"] = {"gpu_vs_cpu_reference": _cmp(out[:n_img], ref, "GPU vs CPU reference path, same input, "
                                                                            "weights and numpy noise")}
    elif cpu_ref is not None and args.extras == "auto":
        log("%s extras: parity" % wl.name)
        extras["parity"] = parity_extras(wl, dev, args, ex, xd, y, cpu_ref)
    if rank == 0 and world == 1 and wl.name in ("c3", "c4", "c5") and args.extras == "auto" and \
            (args.model_dtype or wl.model_dtype) == "fp32":
        log("%s variant: bf16 model" % wl.name)
        e = build_explainer(wl, dev, args, model_dtype="bf16")
        dtv, _, _ = timed(lambda: e(xd, y), 2, 1, 1, dev)
        extras["variants"] = {"bf16_model": {
            "value": round(wl.n * 2 / dtv, 3), "ms_per_step": round(dtv / 2 * 1e3, 2), "steps": 2,
            "what": "the same call with the model in bf16 (%s): not the credited value, the reference runs fp32"
                    % ("BN-folded" if wl.dim == 2 else "autocast")}}
        del e
        torch.cuda.empty_cache()

    model_dtype = args.model_dtype or wl.model_dtype
    total = wl.n * args.steps
    if rank == 0:
        line = {
            "metric": wl.metric, "value": round(total / dt, 3), "unit": wl.unit, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong" if world > 1 else "weak", "vs_baseline": None,
            "dtype": "fp32", "data": "synthetic inputs, random-init weights (no network)",
            "config": {"workload": wl.describe, "model_dtype": model_dtype, "global_batch": wl.n,
                       "seq_len": None, "parallelism": ("dp%d (%s axis)" % (world, axis))
                       if world > 1 else "dp1",
                       "sample_batch": getattr(ex, "sample_batch", None),
                       "model_exec": "as is" if (args.no_optimize_model or wl.dim != 2 or wl.name == "c1") else
                       "optimize_model (BN folded, polyphase stem input-gradient, fused epilogues)",
                       "wam_arith": "fp32"},
            "roofline": roof, "cpu_baseline": cpu}
        line.update(secondary)
        line.update(extras)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
