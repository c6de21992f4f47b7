// The 1D mel front-end (lib/wam_1D.py:194-219: torchaudio MelSpectrogram(sample_rate, n_fft,
// n_mels) + AmplitudeToDB() per waveform) and its adjoint, one wave per frame.
//
// Frame f of a [T] waveform covers samples (f - 1) * hop + n, n < N (N = n_fft, hop = N / 2,
// center=True, reflect padding), F = T / hop + 1 frames. Per frame:
//   z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1]   (periodic Hann w; the real frame packed in M = N/2
//                                               complex points)
//   Z = FFT_M(z)                              (in-place Stockham in the wave's LDS, radix 8 stages
//                                               plus one radix 2/4 stage, table twiddles)
//   X[k] = (Z[k] + conj Z[M-k]) / 2 - i/2 e^{-2 pi i k/N} (Z[k] - conj Z[M-k]),  k = 0..M
//   P[k] = |X[k]|^2,  mel[m] = sum_k P[k] fb[k][m] (band-sparse),  db = 10 log10(max(mel, 1e-10))
// The adjoint (what torch autograd does through stft -> abs -> pow -> matmul -> clamp -> log10)
// recomputes the frame, forms G[k] = 2 dL/dP[k] X[k] and evaluates
//   g_frame[n] = w[n] Re(sum_{k=0..M} G[k] e^{+2 pi i k n/N})
// with one inverse M-point FFT of the Hermitian-packed spectrum; the reflect padding is folded
// back when the frames are overlap-added. A wave owns a run of hop-blocks of the output and streams
// its frames in order, keeping the previous frame's second half in registers, so every output sample
// is written once, in a fixed order (k_mel_adj_run); the reflect folds follow (k_mel_fold).
//
// tables (device, float): window[N] | twiddle[2N] (cos, sin of -2 pi m / N) | band_w[nnz] | bin_w[nnz]
// index  (device, int32): band_ptr[n_mels+1] | band_bin[nnz] | bin_ptr[N/2+2] | bin_band[nnz]
// (the filterbank's nonzeros by band and by bin, built on the host from torchaudio's HTK
// filterbank: wam_amd/melspec.py).
#include "kernels.hpp"

#include <algorithm>
#include <mutex>
#include <set>

namespace {

constexpr int kWavesF = 4;  // forward: waves per workgroup, each streaming frames (one frame per wave at a time)

struct MelGeom {
  int64_t items, T;
  int F, hop, n_mels, nnz;
  int to_db;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
// v * (S i)
template <int S>
__device__ __forceinline__ float2 muls(float2 v) {
  return S < 0 ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
}

// LDS index padding: breaks the stride-R writes of the first stages across banks
__host__ __device__ __forceinline__ int pad(int i) { return i + (i >> 4); }

template <int S>
__device__ __forceinline__ void dft2(float2* a) {
  const float2 t = a[0];
  a[0] = cadd(t, a[1]);
  a[1] = csub(t, a[1]);
}

template <int S>
__device__ __forceinline__ void dft4(float2* a) {
  const float2 c0 = cadd(a[0], a[2]), c2 = csub(a[0], a[2]);
  const float2 c1 = cadd(a[1], a[3]), c3 = muls<S>(csub(a[1], a[3]));
  a[0] = cadd(c0, c1);
  a[1] = cadd(c2, c3);
  a[2] = csub(c0, c1);
  a[3] = csub(c2, c3);
}

template <int S>
__device__ __forceinline__ void dft8(float2* a) {
  constexpr float c = 0.70710678118654752f;
  float2 b[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    b[q] = cadd(a[q], a[q + 4]);
    b[q + 4] = csub(a[q], a[q + 4]);
  }
  b[5] = cmul(b[5], make_float2(c, S * c));
  b[6] = muls<S>(b[6]);
  b[7] = cmul(b[7], make_float2(-c, S * c));
  const float2 c0 = cadd(b[0], b[2]), c2 = csub(b[0], b[2]);
  const float2 c1 = cadd(b[1], b[3]), c3 = muls<S>(csub(b[1], b[3]));
  a[0] = cadd(c0, c1);
  a[4] = csub(c0, c1);
  a[2] = cadd(c2, c3);
  a[6] = csub(c2, c3);
  const float2 d0 = cadd(b[4], b[6]), d2 = csub(b[4], b[6]);
  const float2 d1 = cadd(b[5], b[7]), d3 = muls<S>(csub(b[5], b[7]));
  a[1] = cadd(d0, d1);
  a[5] = csub(d0, d1);
  a[3] = cadd(d2, d3);
  a[7] = csub(d2, d3);
}

// stage plan of an M = 2^LOGM point FFT: one radix 2^(LOGM % 3) stage first (if any), then radix 8
template <int LOGM>
struct Plan {
  static constexpr int first = LOGM % 3;  // log2 radix of the optional first stage
  static constexpr int stages = LOGM / 3 + (first ? 1 : 0);
  static constexpr int log_radix(int st) { return (first && st == 0) ? first : 3; }
  static constexpr int log_ns(int st) { return st == 0 ? 0 : log_ns(st - 1) + log_radix(st - 1); }
};

// one in-place Stockham stage: all of a lane's butterflies are loaded before any is written back
template <int LOGN, int ST, int S>
__device__ __forceinline__ void fft_stage(float2* buf, const float2* __restrict__ tw, int lane) {
  constexpr int LOGM = LOGN - 1, M = 1 << LOGM;
  constexpr int LR = Plan<LOGM>::log_radix(ST), R = 1 << LR;
  constexpr int LNS = Plan<LOGM>::log_ns(ST), Ns = 1 << LNS;
  constexpr int B = M / R, NB = (B + 63) / 64;
  float2 v[NB][R];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = lane + 64 * b;
    if (B % 64 == 0 || j < B) {
      const int k = j & (Ns - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float2 x = buf[pad(j + r * B)];
        if (Ns > 1 && r > 0) {
          float2 t = tw[(r * k) << (LOGN - LNS - LR)];
          if (S > 0) t = cconj(t);
          x = cmul(x, t);
        }
        v[b][r] = x;
      }
      if (R == 8) dft8<S>(v[b]);
      else if (R == 4) dft4<S>(v[b]);
      else dft2<S>(v[b]);
    }
  }
  wave_sync();
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = lane + 64 * b;
    if (B % 64 == 0 || j < B) {
      const int k = j & (Ns - 1);
      const int idx = ((j >> LNS) << (LNS + LR)) + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[pad(idx + r * Ns)] = v[b][r];
    }
  }
  wave_sync();
}

// Register-fed / register-draining forms of a stage for the M = 512 transforms (three radix-8
// stages of 64 butterflies, one per lane): stage 0 reads elements lane + 64 r, which are the
// frame's samples a lane already holds (IN = 1) or the Hermitian pack of the adjoint spectrum
// computed on the load from A (IN = 2: Z''[k] = (A_k + conj A_(M-k)) + i (A_k - conj A_(M-k))
// e^(+2 pi i k / N)); the last stage writes elements lane + 64 r, which stay in registers
// (OUT = 1). Same arithmetic as fft_stage, fewer LDS round trips.
template <int LOGN, int ST, int S, int IN, bool OUT>
__device__ __forceinline__ void fft_stage_io(float2* buf, const float2* __restrict__ tw, int lane,
                                             const float2* vin, float2* vout) {
  constexpr int LOGM = LOGN - 1, M = 1 << LOGM;
  constexpr int LR = Plan<LOGM>::log_radix(ST), R = 1 << LR;
  constexpr int LNS = Plan<LOGM>::log_ns(ST), Ns = 1 << LNS;
  constexpr int B = M / R;
  static_assert(R == 8 && B == 64, "the register forms are for 512-point stages");
  static_assert(IN == 0 || ST == 0, "register input: first stage only");
  static_assert(!OUT || LNS + LR == LOGM, "register output: last stage only");
  const int j = lane, k = j & (Ns - 1);
  float2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float2 x;
    if constexpr (IN == 1) {
      x = vin[r];
    } else if constexpr (IN == 2) {
      const int q = j + r * B;
      const float2 ak = buf[pad(q)], ac = cconj(buf[pad(M - q)]);
      const float2 d = cmul(csub(ak, ac), cconj(tw[q]));
      const float2 sm = cadd(ak, ac);
      x = make_float2(sm.x - d.y, sm.y + d.x);
    } else {
      x = buf[pad(j + r * B)];
    }
    if (Ns > 1 && r > 0) {
      float2 t = tw[(r * k) << (LOGN - LNS - LR)];
      if (S > 0) t = cconj(t);
      x = cmul(x, t);
    }
    v[r] = x;
  }
  dft8<S>(v);
  if constexpr (OUT) {
#pragma unroll
    for (int r = 0; r < R; ++r) vout[r] = v[r];  // element j + r Ns = j + 64 r
  } else {
    wave_sync();
    const int idx = ((j >> LNS) << (LNS + LR)) + k;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[pad(idx + r * Ns)] = v[r];
    wave_sync();
  }
}

template <int LOGN, int ST, int S>
__device__ __forceinline__ void fft_stages(float2* buf, const float2* __restrict__ tw, int lane) {
  if constexpr (ST < Plan<LOGN - 1>::stages) {
    fft_stage<LOGN, ST, S>(buf, tw, lane);
    fft_stages<LOGN, ST + 1, S>(buf, tw, lane);
  }
}

// the kernels' constant tables: staged in LDS once per workgroup (n_fft <= 1024), else read from
// global memory (L1/L2-resident)
struct Tabs {
  const float* win;
  const float2* tw;
  const float* band_w;
  const float* bin_w;
  const int* band_ptr;
  const int* band_bin;
  const int* bin_ptr;
  const int* bin_band;
};

__host__ __device__ inline int tab_floats(int N, int n_mels, int nnz, bool adj) {
  const int nf = 3 * N + nnz * (adj ? 2 : 1);
  const int ni = n_mels + 1 + nnz + (adj ? N / 2 + 2 + nnz : 0);
  return (nf + ni + 3) & ~3;  // float4-aligned end
}

template <bool STAGE>
__device__ __forceinline__ Tabs stage_tables(const MelGeom& g, int N, const float* __restrict__ tables,
                                             const int* __restrict__ index, float* lds, bool adj) {
  const int nf = 3 * N + g.nnz * (adj ? 2 : 1);
  const int ni = g.n_mels + 1 + g.nnz + (adj ? N / 2 + 2 + g.nnz : 0);
  const float* tf = tables;
  const int* ti = index;
  if (STAGE) {
    for (int i = threadIdx.x; i < nf; i += blockDim.x) lds[i] = tables[i];
    int* li = reinterpret_cast<int*>(lds + nf);
    for (int i = threadIdx.x; i < ni; i += blockDim.x) li[i] = index[i];
    __syncthreads();
    tf = lds;
    ti = li;
  }
  Tabs t;
  t.win = tf;
  t.tw = reinterpret_cast<const float2*>(tf + N);
  t.band_w = tf + 3 * N;
  t.bin_w = t.band_w + g.nnz;
  t.band_ptr = ti;
  t.band_bin = ti + g.n_mels + 1;
  t.bin_ptr = t.band_bin + g.nnz;
  t.bin_band = t.bin_ptr + N / 2 + 2;
  return t;
}

// a frame's samples held in registers: fetched one frame ahead, stored (windowed) into the
// wave's LDS buffer when its turn comes
template <int LOGN>
struct FrameIn {
  static constexpr int M = 1 << (LOGN - 1), KM = (M + 63) / 64;
  float a[KM], b[KM];

  __device__ __forceinline__ void fetch(const float* __restrict__ x, int64_t T, int f, int hop, int F, int lane) {
    const int64_t s0 = (int64_t)(f - 1) * hop;
    if (f > 0 && f < F - 1) {
      if ((reinterpret_cast<uintptr_t>(x) & 7) == 0) {  // s0 is even: aligned float2 pairs
        const float2* x2 = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
        for (int i = 0; i < KM; ++i) {
          const int n = lane + 64 * i;
          if (M % 64 == 0 || n < M) {
            const float2 v = x2[n];
            a[i] = v.x;
            b[i] = v.y;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < KM; ++i) {
          const int n = lane + 64 * i;
          if (M % 64 == 0 || n < M) {
            a[i] = x[s0 + 2 * n];
            b[i] = x[s0 + 2 * n + 1];
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        const int n = lane + 64 * i;
        if (M % 64 == 0 || n < M) {
          int64_t s = s0 + 2 * n, t = s + 1;
          s = s < 0 ? -s : (s >= T ? 2 * (T - 1) - s : s);
          t = t < 0 ? -t : (t >= T ? 2 * (T - 1) - t : t);
          a[i] = x[s];
          b[i] = x[t];
        }
      }
    }
  }

  __device__ __forceinline__ void store(const float* win, float2* buf, int lane) const {
#pragma unroll
    for (int i = 0; i < KM; ++i) {
      const int n = lane + 64 * i;
      if (M % 64 == 0 || n < M) buf[pad(n)] = make_float2(a[i] * win[2 * n], b[i] * win[2 * n + 1]);
    }
  }
};

// X[k] of bin k (k <= M) from the packed spectrum in buf
template <int LOGN>
__device__ __forceinline__ float2 unpack_bin(const float2* buf, const float2* tw, int k) {
  constexpr int M = 1 << (LOGN - 1);
  const float2 zk = buf[pad(k & (M - 1))], zc = cconj(buf[pad((M - k) & (M - 1))]);
  const float2 e = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
  const float2 d = csub(zk, zc);
  const float2 o = make_float2(0.5f * d.y, -0.5f * d.x);  // -i/2 (zk - zc)
  return cadd(e, cmul(tw[k], o));
}

// FFT of the stored frame, then P[k] = |X[k]|^2 into buf (as floats, k <= M); X kept if asked
template <int LOGN, bool KEEP>
__device__ __forceinline__ void frame_unpack_power(const Tabs& t, float2* buf, float2* X, int lane) {
  constexpr int M = 1 << (LOGN - 1), KI = M / 64 + 1;
  float p[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    if (k <= M) {
      const float2 x = unpack_bin<LOGN>(buf, t.tw, k);
      if (KEEP) X[i] = x;
      p[i] = x.x * x.x + x.y * x.y;
    }
  }
  wave_sync();
  float* P = reinterpret_cast<float*>(buf);
#pragma unroll
  for (int i = 0; i < KI; ++i)
    if (lane + 64 * i <= M) P[lane + 64 * i] = p[i];
  wave_sync();
}

template <int LOGN, bool KEEP>
__device__ __forceinline__ void frame_power(const Tabs& t, float2* buf, float2* X, int lane) {
  fft_stages<LOGN, 0, -1>(buf, t.tw, lane);
  frame_unpack_power<LOGN, KEEP>(t, buf, X, lane);
}

__device__ __forceinline__ float band_sum(const Tabs& t, const float* P, int m) {
  float acc = 0.f;
  const int e0 = t.band_ptr[m], e1 = t.band_ptr[m + 1];
  if (e1 > e0 && t.band_bin[e1 - 1] - t.band_bin[e0] == e1 - 1 - e0) {
    // a triangular band's bins are consecutive: the P and weight loads do not wait on an index
    // load (same terms, same order)
    const float* pb = P + (t.band_bin[e0] - e0);
#pragma unroll 4
    for (int e = e0; e < e1; ++e) acc = fmaf(pb[e], t.band_w[e], acc);
    return acc;
  }
#pragma unroll 4
  for (int e = e0; e < e1; ++e) acc = fmaf(P[t.band_bin[e]], t.band_w[e], acc);
  return acc;
}

template <int LOGN, bool STAGE>
__global__ void __launch_bounds__(64 * kWavesF) k_mel_fwd(MelGeom g, const float* __restrict__ wave,
                                                          const float* __restrict__ tables,
                                                          const int* __restrict__ index, float* __restrict__ out) {
  constexpr int N = 1 << LOGN, M = N / 2;
  extern __shared__ float4 lds_raw[];
  float* lf = reinterpret_cast<float*>(lds_raw);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const Tabs t = stage_tables<STAGE>(g, N, tables, index, lf, false);
  float2* buf = reinterpret_cast<float2*>(lf + (STAGE ? tab_floats(N, g.n_mels, g.nnz, false) : 0)) + w * (pad(M) + 2);
  const int64_t frames = g.items * g.F, stride = (int64_t)gridDim.x * kWavesF;
  // XCD-aware: logically consecutive workgroups (consecutive frames, which share half a frame of
  // samples) run on one XCD, so the shared half comes from its L2 instead of a second HBM read
  int64_t q = wam_xcd_block(blockIdx.x, gridDim.x) * kWavesF + w;
  FrameIn<LOGN> in;
  if (q < frames) in.fetch(wave + (q / g.F) * g.T, g.T, (int)(q % g.F), g.hop, g.F, lane);
  for (; q < frames; q += stride) {
    const int64_t qn = q + stride;
    if constexpr (LOGN == 10) {  // 512-point transform: the first stage fed from registers
      float2 z0[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = lane + 64 * i;
        z0[i] = make_float2(in.a[i] * t.win[2 * n], in.b[i] * t.win[2 * n + 1]);
      }
      fft_stage_io<LOGN, 0, -1, 1, false>(buf, t.tw, lane, z0, nullptr);
      if (qn < frames) in.fetch(wave + (qn / g.F) * g.T, g.T, (int)(qn % g.F), g.hop, g.F, lane);
      fft_stages<LOGN, 1, -1>(buf, t.tw, lane);
      frame_unpack_power<LOGN, false>(t, buf, nullptr, lane);
    } else {
      in.store(t.win, buf, lane);
      if (qn < frames) in.fetch(wave + (qn / g.F) * g.T, g.T, (int)(qn % g.F), g.hop, g.F, lane);
      wave_sync();
      frame_power<LOGN, false>(t, buf, nullptr, lane);
    }
    const float* P = reinterpret_cast<const float*>(buf);
    float* o = out + q * g.n_mels;
    for (int m = lane; m < g.n_mels; m += 64) {
      const float acc = band_sum(t, P, m);
      o[m] = g.to_db ? 10.f * log10f(fmaxf(acc, 1e-10f)) : acc;
    }
    wave_sync();
  }
}

// one frame's adjoint chain (see header) up to the inverse FFT, whose output z stays in buf: the
// frame's gradient is g[2n] = w[2n] z[n].x / 2, g[2n+1] = w[2n+1] z[n].y / 2; the frame's samples are
// in `in`, which is refilled with frame f_next (if >= 0) meanwhile
template <int LOGN>
__device__ __forceinline__ void frame_adjoint_buf(const MelGeom& g, const Tabs& t, FrameIn<LOGN>& in,
                                                  const float* __restrict__ x, int f, int f_next,
                                                  const float* __restrict__ gdb, float2* buf, float* gmel, int lane,
                                                  float2* zout = nullptr) {
  constexpr int M = 1 << (LOGN - 1), KI = M / 64 + 1;
  constexpr int kMelRegs = 4;  // bands lane + 64 j, j < 4, held in registers (n_mels <= 256)
  constexpr bool FAST = LOGN == 10;  // 512-point transforms: register-fed first / last stages
  float gq[kMelRegs];
  const float* gf = gdb + (int64_t)f * g.n_mels;
#pragma unroll
  for (int j = 0; j < kMelRegs; ++j) gq[j] = lane + 64 * j < g.n_mels ? gf[lane + 64 * j] : 0.f;
  float2 X[KI];
  if constexpr (FAST) {
    // stage 0 straight from the windowed samples in registers (no store + reload of the frame)
    float2 z0[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = lane + 64 * i;
      z0[i] = make_float2(in.a[i] * t.win[2 * n], in.b[i] * t.win[2 * n + 1]);
    }
    fft_stage_io<LOGN, 0, -1, 1, false>(buf, t.tw, lane, z0, nullptr);
    if (f_next >= 0) in.fetch(x, g.T, f_next, g.hop, g.F, lane);
    fft_stages<LOGN, 1, -1>(buf, t.tw, lane);
    frame_unpack_power<LOGN, true>(t, buf, X, lane);
  } else {
    in.store(t.win, buf, lane);
    if (f_next >= 0) in.fetch(x, g.T, f_next, g.hop, g.F, lane);
    wave_sync();
    frame_power<LOGN, true>(t, buf, X, lane);
  }
  const float* P = reinterpret_cast<const float*>(buf);
  // d db / d mel: mul(10) -> log10 -> clamp(min=1e-10), in torch's order
#pragma unroll
  for (int j = 0; j < kMelRegs; ++j) {
    const int m = lane + 64 * j;
    if (m < g.n_mels) {
      const float acc = band_sum(t, P, m);
      float gm = gq[j];
      if (g.to_db) {
        const float gl = gm * 10.f;
        gm = acc >= 1e-10f ? gl / (fmaxf(acc, 1e-10f) * 2.302585092994046f) : 0.f;
      }
      gmel[m] = gm;
    }
  }
  wave_sync();
  // A[k] = 2 dL/dP[k] X[k] (real at k = 0, M: doubled real part, the Hermitian pair folded)
  float2 A[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    if (k <= M) {
      float gp = 0.f;
      const int e1 = t.bin_ptr[k + 1];
      for (int e = t.bin_ptr[k]; e < e1; ++e) gp = fmaf(gmel[t.bin_band[e]], t.bin_w[e], gp);
      A[i] = make_float2(2.f * gp * X[i].x, 2.f * gp * X[i].y);
      if (k == 0 || k == M) A[i] = make_float2(2.f * A[i].x, 0.f);
    }
  }
  wave_sync();  // gmel may live in buf's tail (the run kernel): all reads before A overwrites it
#pragma unroll
  for (int i = 0; i < KI; ++i)
    if (lane + 64 * i <= M) buf[pad(lane + 64 * i)] = A[i];
  wave_sync();
  if constexpr (FAST) {
    // the Hermitian pack computed on the first inverse stage's load; the last stage's output
    // (z[lane + 64 r]) stays in registers or goes back to buf
    fft_stage_io<LOGN, 0, 1, 2, false>(buf, t.tw, lane, nullptr, nullptr);
    fft_stage_io<LOGN, 1, 1, 0, false>(buf, t.tw, lane, nullptr, nullptr);
    if (zout) fft_stage_io<LOGN, 2, 1, 0, true>(buf, t.tw, lane, nullptr, zout);
    else fft_stage_io<LOGN, 2, 1, 0, false>(buf, t.tw, lane, nullptr, nullptr);
    return;
  }
  // Z''[k] = (A_k + conj A_{M-k}) + i (A_k - conj A_{M-k}) e^{+2 pi i k/N},  k < M
  float2 Zp[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    if (k < M) {
      const float2 ak = buf[pad(k)], ac = cconj(buf[pad(M - k)]);
      const float2 d = cmul(csub(ak, ac), cconj(t.tw[k]));
      const float2 s = cadd(ak, ac);
      Zp[i] = make_float2(s.x - d.y, s.y + d.x);
    }
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < KI; ++i)
    if (lane + 64 * i < M) buf[pad(lane + 64 * i)] = Zp[i];
  wave_sync();
  fft_stages<LOGN, 0, 1>(buf, t.tw, lane);
}

// ------------------------------------------------------------------------------------------------
// Run-streaming adjoint (the default). A wave owns a run of consecutive hop-blocks [b0, b1) of one
// waveform and computes the frames b0 .. min(b1, F - 1) in order; frame f's gradient leaves the
// inverse FFT as samples 2n, 2n + 1 of lane n mod 64 (n = lane + 64 j), so its second half stays
// in registers (`carry`) and block f - 1 = carry + the next frame's first half is written straight
// to HBM with coalesced float2 stores, once, in the slot kernel's summation order. No frame slots
// and no workgroup barrier after the table staging: the LDS per wave is its FFT buffer (P and the
// band gradients reuse it), so 4-wave workgroups fit three to a CU (12 waves) where the slot kernel
// (138 KB of LDS) fit one 8-wave workgroup. The reflect folds (frame 0 onto samples [1, hop],
// frame F - 1 onto [2T - 1 - F hop, T - 2]) are added afterwards by k_mel_fold.
constexpr int kWavesR = 4;

struct RunGeom {
  int runs_per_item;
  int64_t runs;  // items * runs_per_item
};

__host__ __device__ inline int run_gmel_off(int M) { return (M + 1 + 3) & ~3; }
__host__ __device__ inline int run_wave_floats(int M, int n_mels) {
  const int a = 2 * (pad(M) + 2), b = run_gmel_off(M) + n_mels;
  return ((a > b ? a : b) + 3) & ~3;
}

// the frame's windowed gradient pairs (g[2n], g[2n+1]), n = lane + 64 j, from buf
template <int LOGN, int KJ>
__device__ __forceinline__ void frame_pairs(const float* __restrict__ win, const float2* buf, float2 (&gp)[KJ],
                                            int lane) {
  constexpr int M = 1 << (LOGN - 1);
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int n = lane + 64 * j;
    if (M % 64 == 0 || n < M) {
      const float2 z = buf[pad(n)];
      gp[j] = make_float2(win[2 * n] * (0.5f * z.x), win[2 * n + 1] * (0.5f * z.y));
    }
  }
}

template <int LOGN, bool STAGE>
__global__ void __launch_bounds__(64 * kWavesR) __attribute__((amdgpu_waves_per_eu(3, 8)))
    k_mel_adj_run(MelGeom g, RunGeom rg, const float* __restrict__ wave, const float* __restrict__ gdb,
                  const float* __restrict__ tables, const int* __restrict__ index, float* __restrict__ gwave) {
  constexpr int N = 1 << LOGN, M = N / 2, KJ = M / 64 > 0 ? M / 64 : 1, KH = KJ / 2 > 0 ? KJ / 2 : 1;
  extern __shared__ float4 lds_raw[];
  float* lf = reinterpret_cast<float*>(lds_raw);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Tabs t = stage_tables<STAGE>(g, N, tables, index, lf, true);
  float* wbase = lf + (STAGE ? tab_floats(N, g.n_mels, g.nnz, true) : 0) + w * run_wave_floats(M, g.n_mels);
  float2* buf = reinterpret_cast<float2*>(wbase);
  float* gmel = wbase + run_gmel_off(M);
  const int hop = g.hop, F = g.F;
  const int64_t T = g.T;
  const int nb = (int)((T + hop - 1) / hop);
  const int64_t stride = (int64_t)gridDim.x * kWavesR;
  for (int64_t run = (int64_t)blockIdx.x * kWavesR + w; run < rg.runs; run += stride) {
    const int64_t it = run / rg.runs_per_item;
    const int r = (int)(run - it * rg.runs_per_item);
    const int b0 = (int)((int64_t)r * nb / rg.runs_per_item), b1 = (int)((int64_t)(r + 1) * nb / rg.runs_per_item);
    const int fe = min(b1, F - 1);
    const float* x = wave + it * T;
    const float* gd = gdb + it * (int64_t)F * g.n_mels;
    float* o = gwave + it * T;
    const bool vec = ((it * T) & 1) == 0;  // float2 stores stay 8-byte aligned
    // block b (samples b hop + 2n + e, n = lane + 64 j, j < KH) = a (+ bsec)
    auto put_block = [&](int b, const float2 (&a)[KH], const float2* bsec) {
      const int64_t s0 = (int64_t)b * hop;
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        const int n = lane + 64 * j;
        if (2 * n < hop) {
          float2 v = a[j];
          if (bsec) v = make_float2(v.x + bsec[j].x, v.y + bsec[j].y);
          const int64_t s = s0 + 2 * n;
          if (vec && s + 1 < T) {
            *reinterpret_cast<float2*>(o + s) = v;
          } else {
            if (s < T) o[s] = v.x;
            if (s + 1 < T) o[s + 1] = v.y;
          }
        }
      }
    };
    FrameIn<LOGN> in;
    in.fetch(x, T, b0, hop, F, lane);
    float2 carry[KH];
    for (int f = b0; f <= fe; ++f) {
      float2 gp[KJ];
      if constexpr (LOGN == 10) {  // the last inverse stage's output straight from registers
        float2 z[8];
        frame_adjoint_buf<LOGN>(g, t, in, x, f, f < fe ? f + 1 : -1, gd, buf, gmel, lane, z);
#pragma unroll
        for (int j = 0; j < KJ; ++j) {
          const int n = lane + 64 * j;
          gp[j] = make_float2(t.win[2 * n] * (0.5f * z[j].x), t.win[2 * n + 1] * (0.5f * z[j].y));
        }
      } else {
        frame_adjoint_buf<LOGN>(g, t, in, x, f, f < fe ? f + 1 : -1, gd, buf, gmel, lane);
        frame_pairs<LOGN, KJ>(t.win, buf, gp, lane);
      }
      if (f > b0) put_block(f - 1, carry, gp);  // frame f - 1's second half + frame f's first half
      if constexpr (KJ >= 2) {
#pragma unroll
        for (int j = 0; j < KH; ++j) carry[j] = gp[KH + j];
      } else {  // M <= 64: the second half is lanes M/2 .. M-1
        carry[0] = make_float2(__shfl(gp[0].x, (lane + M / 2) & 63, 64), __shfl(gp[0].y, (lane + M / 2) & 63, 64));
      }
      wave_sync();
    }
    if (fe == F - 1 && fe < b1) put_block(fe, carry, nullptr);  // the last block: no next frame
  }
}

// The reflect folds, after k_mel_adj_run: wave 2 i recomputes frame 0 of waveform i and adds it
// onto samples [1, min(hop, T - 1)], wave 2 i + 1 frame F - 1 onto [2T - 1 - F hop, T - 2] (the
// slot kernel's order: regular frames, then frame 0, then frame F - 1; the two run in sequence
// inside one wave when the regions overlap, T < 2 hop)
template <int LOGN, bool STAGE>
__global__ void __launch_bounds__(64 * kWavesR) __attribute__((amdgpu_waves_per_eu(3, 8)))
    k_mel_fold(MelGeom g, const float* __restrict__ wave, const float* __restrict__ gdb,
               const float* __restrict__ tables, const int* __restrict__ index, float* __restrict__ gwave) {
  constexpr int N = 1 << LOGN, M = N / 2;
  extern __shared__ float4 lds_raw[];
  float* lf = reinterpret_cast<float*>(lds_raw);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Tabs t = stage_tables<STAGE>(g, N, tables, index, lf, true);
  float* wbase = lf + (STAGE ? tab_floats(N, g.n_mels, g.nnz, true) : 0) + w * run_wave_floats(M, g.n_mels);
  float2* buf = reinterpret_cast<float2*>(wbase);
  float* gmel = wbase + run_gmel_off(M);
  const int hop = g.hop, F = g.F;
  const int64_t T = g.T;
  const int64_t r_lo = 2 * T - 1 - (int64_t)F * hop;
  const bool overlap = r_lo <= hop;  // both folds touch a sample: one wave does both, in order
  const int64_t q = (int64_t)blockIdx.x * kWavesR + w;
  if (q >= 2 * g.items) return;
  const int64_t it = q >> 1;
  const int side = (int)(q & 1);
  if (overlap && side) return;
  const float* x = wave + it * T;
  const float* gd = gdb + it * (int64_t)F * g.n_mels;
  float* o = gwave + it * T;
  FrameIn<LOGN> in;
  for (int k = side; k < (overlap ? 2 : side + 1); ++k) {
    const int f = k ? F - 1 : 0;
    in.fetch(x, T, f, hop, F, lane);
    frame_adjoint_buf<LOGN>(g, t, in, x, f, -1, gd, buf, gmel, lane);
    auto at = [&](int n) {  // the frame's windowed gradient at sample n of the frame
      const float2 z = buf[pad(n >> 1)];
      return t.win[n] * (0.5f * ((n & 1) ? z.y : z.x));
    };
    if (k == 0) {
      for (int64_t s = 1 + lane; s <= min((int64_t)hop, T - 1); s += 64) o[s] += at((int)(hop - s));
    } else {
      for (int64_t s = max(r_lo, (int64_t)0) + lane; s <= T - 2; s += 64)
        o[s] += at((int)(2 * (T - 1) - s - (int64_t)(F - 2) * hop));
    }
    wave_sync();
  }
}

constexpr int kMaxLds = 160 * 1024;

int lds_fwd(int log_n, int n_mels, int nnz) {
  const int N = 1 << log_n, M = N / 2;
  return (log_n <= 10 ? tab_floats(N, n_mels, nnz, false) * 4 : 0) + kWavesF * (M + (M >> 4) + 2) * 8;
}

int lds_opt_in_mel(const void* kern, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  if (bytes <= 64 * 1024) return WAM_OK;
  int dev = 0;
  WAM_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({kern, dev})) return WAM_OK;
  WAM_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({kern, dev});
  return WAM_OK;
}

int check_args(int64_t items, int64_t samples, int n_fft, int n_mels, int nnz, int* log_n) {
  if (items < 0 || n_mels < 1 || nnz < 0) return WAM_ERR_INVALID_ARG;
  int l = 0;
  while ((1 << l) < n_fft) ++l;
  if ((1 << l) != n_fft || l < 6 || l > 11 || n_mels > 256) return WAM_ERR_UNSUPPORTED;
  if (nnz > 2 * (n_fft / 2 + 1)) return WAM_ERR_INVALID_ARG;  // a triangular bank: <= 2 bands per bin
  if (samples <= n_fft / 2) return WAM_ERR_SHAPE;              // reflect pad needs T > n_fft / 2
  *log_n = l;
  return WAM_OK;
}

}  // namespace

extern "C" int wam_melspec(int64_t items, int64_t samples, int n_fft, int n_mels, int nnz, int to_db,
                           const float* wave, const float* tables, const int* index, float* out, void* stream) {
  int log_n = 0;
  if (int rc = check_args(items, samples, n_fft, n_mels, nnz, &log_n)) return rc;
  if (items == 0) return WAM_OK;
  if (!wave || !tables || !index || !out) return WAM_ERR_INVALID_ARG;
  MelGeom g{};
  g.items = items;
  g.T = samples;
  g.hop = n_fft / 2;
  g.F = (int)(samples / g.hop + 1);
  g.n_mels = n_mels;
  g.nnz = nnz;
  g.to_db = to_db ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t frames = items * g.F;
  const int lds = lds_fwd(log_n, n_mels, nnz);
  if (lds > kMaxLds) return WAM_ERR_UNSUPPORTED;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  // persistent-ish grid: a few workgroups per CU, each wave streaming frames with one-ahead prefetch
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((frames + kWavesF - 1) / kWavesF, 4 * cus));
  WamTimer tm(st, "k_mel_fwd", 4.0 * (double)items * samples + 4.0 * (double)frames * n_mels);
  switch (log_n) {
#define WAM_MELF(L)                                                                                           \
  case L:                                                                                                     \
    if (int rc = lds_opt_in_mel((const void*)k_mel_fwd<L, (L <= 10)>, lds)) return rc;                        \
    hipLaunchKernelGGL((k_mel_fwd<L, (L <= 10)>), dim3(grid), dim3(64 * kWavesF), lds, st, g, wave, tables, index, \
                       out);                                                                                  \
    break;
    WAM_MELF(6) WAM_MELF(7) WAM_MELF(8) WAM_MELF(9) WAM_MELF(10) WAM_MELF(11)
#undef WAM_MELF
    default: return WAM_ERR_UNSUPPORTED;
  }
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

extern "C" int wam_melspec_adjoint(int64_t items, int64_t samples, int n_fft, int n_mels, int nnz, int to_db,
                                   const float* wave, const float* grad_out, const float* tables, const int* index,
                                   float* grad_wave, void* stream) {
  int log_n = 0;
  if (int rc = check_args(items, samples, n_fft, n_mels, nnz, &log_n)) return rc;
  if (items == 0) return WAM_OK;
  if (!wave || !grad_out || !tables || !index || !grad_wave) return WAM_ERR_INVALID_ARG;
  MelGeom g{};
  g.items = items;
  g.T = samples;
  g.hop = n_fft / 2;
  g.F = (int)(samples / g.hop + 1);
  g.n_mels = n_mels;
  g.nnz = nnz;
  g.to_db = to_db ? 1 : 0;
  const int nb = (int)((samples + g.hop - 1) / g.hop);
  hipStream_t st = (hipStream_t)stream;
  const int M = n_fft / 2;
  const int lds = ((log_n <= 10 ? tab_floats(n_fft, n_mels, nnz, true) : 0) + kWavesR * run_wave_floats(M, n_mels)) * 4;
  if (lds > kMaxLds) return WAM_ERR_UNSUPPORTED;
  const void* kern = nullptr;
  const void* kfold = nullptr;
  switch (log_n) {
#define WAM_MELR(L)                                     \
  case L:                                               \
    kern = (const void*)k_mel_adj_run<L, (L <= 10)>;    \
    kfold = (const void*)k_mel_fold<L, (L <= 10)>;      \
    break;
    WAM_MELR(6) WAM_MELR(7) WAM_MELR(8) WAM_MELR(9) WAM_MELR(10) WAM_MELR(11)
#undef WAM_MELR
    default: return WAM_ERR_UNSUPPORTED;
  }
  if (int rc = lds_opt_in_mel(kern, lds)) return rc;
  if (int rc = lds_opt_in_mel(kfold, lds)) return rc;
  int dev = 0, cus = 256, per_cu = 1;
  WAM_HIP_CHECK(hipGetDevice(&dev));
  WAM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kWavesR, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  // runs of about 16 hop-blocks (one extra frame each), their count rounded to whole rounds of the
  // resident waves (the runs cost the same)
  const int64_t resident = (int64_t)per_cu * cus * kWavesR;
  const int64_t want = std::max<int64_t>(1, (items * nb + 8 * resident) / (16 * resident)) * resident;
  RunGeom rg{};
  rg.runs_per_item = (int)std::max<int64_t>(1, std::min<int64_t>(nb, (want + items / 2) / items));
  rg.runs = items * rg.runs_per_item;
  const int64_t wgs = std::min<int64_t>((rg.runs + kWavesR - 1) / kWavesR, (int64_t)per_cu * cus);
  const unsigned fold_wgs = (unsigned)((2 * items + kWavesR - 1) / kWavesR);
  {
    WamTimer tm(st, "k_mel_adj", 8.0 * (double)items * samples + 4.0 * (double)items * g.F * n_mels);
    switch (log_n) {
#define WAM_MELR(L)                                                                                       \
  case L:                                                                                                 \
    hipLaunchKernelGGL((k_mel_adj_run<L, (L <= 10)>), dim3((unsigned)wgs), dim3(64 * kWavesR), lds, st, g, rg, \
                       wave, grad_out, tables, index, grad_wave);                                         \
    break;
      WAM_MELR(6) WAM_MELR(7) WAM_MELR(8) WAM_MELR(9) WAM_MELR(10) WAM_MELR(11)
#undef WAM_MELR
    }
    WAM_LAUNCH_CHECK();
  }
  // the folds: two frames per waveform recomputed, 2 hop samples read and written
  WamTimer tm(st, "k_mel_fold", 4.0 * (double)items * (2.0 * n_fft + 2.0 * n_mels + 4.0 * g.hop));
  switch (log_n) {
#define WAM_MELR(L)                                                                                            \
  case L:                                                                                                      \
    hipLaunchKernelGGL((k_mel_fold<L, (L <= 10)>), dim3(fold_wgs), dim3(64 * kWavesR), lds, st, g, wave, grad_out, \
                       tables, index, grad_wave);                                                              \
    break;
    WAM_MELR(6) WAM_MELR(7) WAM_MELR(8) WAM_MELR(9) WAM_MELR(10) WAM_MELR(11)
#undef WAM_MELR
  }
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}
