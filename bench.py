"""WAM-2D throughput bench on MI355X (the BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[1], the metric's config): WAM-2D SmoothGrad, db4, J=3,
n_samples=25, batch 64 of synthetic 224x224 images (RandomState(1) N(0,1), ImageNet-normalised
scale), labels RandomState(2).randint(0, 1000, 64) as a list, random-init ResNet-50 (no network:
synthetic data, random weights). One STEP = one explainer call on the 64-image batch = 64
attributions, 1600 model forward/backward passes. The reference cannot run db4 SmoothGrad at 224
(its hard-coded 224 canvas vs a 230 mosaic); the native frame (E1: crop to the
input size) is used, identical to the reference wherever the reference runs.
Multi-GPU: one process per GPU, each rank explains its own 64-image batch (independent
attributions, no data-path collective) -> "scaling": "weak"; value = all ranks' attributions /
max-over-ranks time.

The JSON line also carries
  roofline      the dominant WAM transform (largest total time) measured live with HIP events on
                the stream the kernels run on: SURVEY 8(d) algorithmic bytes per launch (4 (P+K)
                per image-sample x image-samples per launch) / mean launch time vs the 8 TB/s HBM
                peak; fused_min_* = the fused kernel's own minimum bytes (clean input read once);
                traffic = PMC HBM bytes per launch from profiles/*_pmc.json when a matching
                rocprofv3 --pmc capture is committed (else null);
  cpu_baseline  the reference algorithm (oracle/wam_ref.py: per-sample loop, torch-CPU ptwt
                restatement, numpy legacy noise, numpy mosaic; fp32 ResNet-50) on a bounded
                sample on the host cores, rank 0 at N=1 only.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
N_IMAGES = 64
N_SAMPLES = 25


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model-dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--sample-batch", type=int, default=13, help="noise samples per model call (x64 images)")
    ap.add_argument("--channels-last", dest="channels_last", action="store_true", default=True,
                    help="NHWC model execution (default; faster than NCHW for the BN-folded bf16 model)")
    ap.add_argument("--no-channels-last", dest="channels_last", action="store_false")
    ap.add_argument("--no-optimize-model", action="store_true",
                    help="run the model as is under autocast instead of the BN-folded bf16 copy (model_opt.py)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    return ap.parse_args()


def make_inputs():
    x = torch.tensor(np.random.RandomState(1).standard_normal((N_IMAGES, 3, 224, 224)).astype(np.float32))
    y = [int(v) for v in np.random.RandomState(2).randint(0, 1000, N_IMAGES)]
    return x, y


def cpu_baseline(seconds):
    """Reference algorithm on the host cores, bounded sample (images x noise samples)."""
    import testmodels
    from oracle import wam_ref
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    model = testmodels.resnet50(seed=0)
    x, y = make_inputs()
    # calibrate on one image x one sample, then size the sample to ~`seconds` of CPU work
    for _ in range(2):  # the first call pays one-time CPU start-up costs
        t0 = time.perf_counter()
        wam_ref.smooth_2d(model, x[:2], y[:2], wavelet="db4", J=3, mode="reflect", n_samples=1, frame="native")
        t1 = (time.perf_counter() - t0) / 2
    per = max(t1, 1e-3)
    # images x samples sized to ~`seconds` of CPU work: all 25 samples of as many images as fit
    n_s = N_SAMPLES if seconds / per >= N_SAMPLES else int(max(1, seconds / per))
    n_img = int(max(1, min(N_IMAGES, seconds / per / n_s)))
    t0 = time.perf_counter()
    wam_ref.smooth_2d(model, x[:n_img], y[:n_img], wavelet="db4", J=3, mode="reflect", n_samples=n_s, frame="native")
    dt = time.perf_counter() - t0
    image_samples_per_s = n_img * n_s / dt
    cpu_model = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": image_samples_per_s / N_SAMPLES, "unit": "attributions/s", "cores": cores,
            "kind": "port",
            "sample": "oracle/wam_ref.smooth_2d (reference glue restated on torch-CPU ptwt, numpy legacy noise), "
                      "fp32 ResNet-50, %d image(s) x %d noise sample(s) of the c2 workload in %.1f s on %d "
                      "thread(s) of %s, extrapolated to 25 samples per attribution" % (n_img, n_s, dt, cores,
                                                                                       cpu_model)}


def load_traffic(op_kernel):
    """PMC HBM bytes per call of the dominant op from the newest committed profiles/*_pmc.json."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        return d.get("per_call_bytes", {}).get(op_kernel)
    except Exception:
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import testmodels
    from wam_amd import plan as P
    from wam_amd.wam_2D import WaveletAttribution2D

    model = testmodels.resnet50(seed=0).to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    for p in model.parameters():
        p.requires_grad_(False)
    x, y = make_inputs()
    x = x.to(dev)
    ex = WaveletAttribution2D(model, wavelet="db4", J=3, method="smooth", mode="reflect", n_samples=N_SAMPLES,
                              noise="philox", frame="native", sample_batch=args.sample_batch,
                              autocast_dtype=torch.bfloat16 if args.model_dtype == "bf16" else None,
                              channels_last=args.channels_last, optimize_model=not args.no_optimize_model)

    def step():
        return ex(x, y)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    P.timing_drain()
    P.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
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
    assert out.shape == (N_IMAGES, 224, 224) and np.isfinite(out).all()

    # live per-launch timing: HIP events recorded by libwam_hip.so around every launch, on the
    # stream the kernel runs on; bytes = algorithmic (each input read once, each output written once)
    kern = {}
    for name, ms, nb in records:
        k = kern.setdefault(name, {"launches": 0, "total_ms": 0.0, "bytes": 0.0})
        k["launches"] += 1
        k["total_ms"] += ms
        k["bytes"] += nb
    for k in kern.values():
        k["mean_us"] = k["total_ms"] * 1e3 / k["launches"]
        k["GBps"] = k["bytes"] / (k["total_ms"] * 1e-3) / 1e9
        k["bytes_per_launch"] = k["bytes"] / k["launches"]
    dom = max(kern, key=lambda n: kern[n]["total_ms"])
    # achieved = SURVEY.md section 8(d)'s per-unit algorithmic bytes x the units one launch
    # processes. The unit is one (image x noise sample); per unit the analysis moves 4 (P + K)
    # bytes (P = C*H*W input values, K = C * coefficients per plane), the input of every sample
    # counted as the reference materialises each noisy image. The fused noisy analysis reads the
    # clean image once for all its samples, so it moves fewer bytes than that: its own minimum
    # (clean input once + every sample's coefficients) is reported as fused_min_*.
    kd = kern[dom]
    units_per_launch = N_IMAGES * N_SAMPLES * args.steps / kd["launches"]
    coeff_plane = P.get_plan(2, (224, 224), 3, "db4", "reflect", dev).coeff_numel
    unit_bytes = {"k_plane_ana<noise>": 4 * 3 * (224 * 224 + coeff_plane),
                  "k_plane_syn": 4 * 3 * (coeff_plane + 224 * 224),
                  "k_plane_maps": 4 * (3 * 224 * 224 + coeff_plane)}.get(dom)
    bpl = unit_bytes * units_per_launch if unit_bytes else kd["bytes_per_launch"]
    achieved = bpl / (kd["mean_us"] * 1e-6) / 1e9
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(dom),
                "bytes_per_launch": round(bpl), "units_per_launch": units_per_launch,
                "bytes_basis": "SURVEY 8(d): 4(P+K) per image-sample" if unit_bytes else "library algorithmic bytes",
                "fused_min_bytes_per_launch": round(kd["bytes_per_launch"]), "fused_min_GBps": round(kd["GBps"], 1),
                "mean_us": round(kd["mean_us"], 2),
                "wam_ms_per_step": round(sum(k["total_ms"] for k in kern.values()) / args.steps, 3),
                "kernels": {n: {kk: round(vv, 3) for kk, vv in k.items()} for n, k in
                            sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"])}}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(args.cpu_seconds)

    total_attr = N_IMAGES * args.steps * world
    if rank == 0:
        line = {
            "metric": "WAM-2D attributions/sec @224^2 n_samples=25 (db4 J=3 SmoothGrad, ResNet-50)",
            "value": round(total_attr / dt, 3), "unit": "attributions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (RandomState(1) N(0,1) images, random-init ResNet-50)",
            "config": {"workload": "c2: WAM-2D db4 J=3 SmoothGrad n_samples=25, batch 64 x 224x224, ResNet-50",
                       "model_dtype": args.model_dtype, "global_batch": N_IMAGES * world, "seq_len": None,
                       "parallelism": "dp%d" % world, "noise": "philox", "frame": "native(E1)",
                       "sample_batch": args.sample_batch, "channels_last": args.channels_last,
                       "model_exec": "autocast" if args.no_optimize_model else
                       "optimize_model (BN folded into convs, polyphase stem input-gradient, bf16 weights)"},
            "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
