"""k_mel_fwd / k_mel_adj at c3 group size (1280 clips x 80000 samples, n_fft 1024, 128 mels,
16 kHz) vs the torch.stft restatement (stft -> |.|^2 -> mel matmul -> dB, autograd backward)
on the same device. Prints per-call times (HIP events on the current stream)."""
import argparse
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=1280)
    ap.add_argument("--samples", type=int, default=80000)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from wam_amd import melspec as M
    x = torch.randn(a.items, a.samples, device="cuda")
    F = a.samples // 512 + 1
    g = torch.randn(a.items, F, 128, device="cuda")
    t_f = timed(lambda: M.mel_forward(x, 1024, 16000, 128), a.iters)
    t_a = timed(lambda: M.mel_adjoint(x, g, 1024, 16000, 128), a.iters)

    def torch_path():
        xl = x.detach().requires_grad_(True)
        db = M._torch_melspec(xl, 1024, 16000, 128, True)
        torch.autograd.grad(db, xl, grad_outputs=g)

    t_t = timed(torch_path, a.iters)
    gb = 4.0 * a.items * a.samples / 1e9
    print("k_mel_fwd  %8.1f us  (%.0f GB/s on the waveform read)" % (1e3 * t_f, gb / (t_f * 1e-3)))
    print("k_mel_adj  %8.1f us  (%.0f GB/s on waveform read + gradient write)" % (1e3 * t_a, 2 * gb / (t_a * 1e-3)))
    print("kernels fwd+adj %8.1f us ; torch stft path fwd+bwd %8.1f us ; speedup %.1fx"
          % (1e3 * (t_f + t_a), 1e3 * t_t, t_t / (t_f + t_a)))


if __name__ == "__main__":
    main()
