// Row-streaming helpers shared by the row-resident 2D kernels (dwt2_rows.hip) and the
// plane-resident multi-level kernels (dwt2_plane.hip): whole source rows fetched with 16-byte
// loads into registers, committed to a wave-private LDS row whose pad slots carry the boundary
// extension, filtered horizontally from LDS.
#pragma once
#include "kernels.hpp"
#include "rng.hpp"

namespace wam_rows {

constexpr int kMaxRow = 512;
constexpr int kPadL = 24;              // >= p = L - 2 for L <= 20, multiple of 4 (16-byte commits)
constexpr int kRowLds = kPadL + kMaxRow + 32;
constexpr int kWaves = 4;

__device__ __forceinline__ void wsync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || a > b) ? a : b; }

// source row of extended row er (-1 = zero row). Inlined on purpose: an out-of-line call for the
// rare far rows in the row loops forced the call ABI's register split on the whole loop (VGPR
// spills whose scratch reloads drain the row fetches in flight): the noisy plane analysis ran 4 %
// and the c4 row kernels 3-4 % faster without it (r02h A/B)
__device__ __forceinline__ int row_src(int er, int n, int mode) { return wam_ext_index(er, n, mode); }

// One source row in registers: VEC-wide loads, MAXV per lane.
template <int VEC, int MAXV>
struct RowRegs {
  float v[VEC * MAXV];
  bool ok[MAXV];

  // branch-free: out-of-range lanes / rows load a clamped valid address; the zeroing select is
  // deferred to commit() so the load stays in flight until the row is consumed
  __device__ __forceinline__ void fetch(const float* __restrict__ row, int nw, int lane, bool valid) {
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      const int idx = (lane + 64 * q) * VEC;
      ok[q] = valid && idx < nw;
      const int ci = idx < nw ? idx : nw - VEC;
      if constexpr (VEC == 4) {
        float4 t = *reinterpret_cast<const float4*>(row + ci);
        v[4 * q] = t.x;
        v[4 * q + 1] = t.y;
        v[4 * q + 2] = t.z;
        v[4 * q + 3] = t.w;
      } else {
        v[q] = row[ci];
      }
    }
  }

  // commit to the padded LDS row (sample s at lds[kPadL + s]); noise (optional) added here
  __device__ __forceinline__ void commit(float* lds, int lane, const float* nz, float sg = 0.f) const {
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      const int idx = (lane + 64 * q) * VEC;
      if constexpr (VEC == 4) {
        float4 o = ok[q] ? make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3])
                         : make_float4(0.f, 0.f, 0.f, 0.f);
        if (nz) {
          // noisy = fma(sigma, z, x): the same rounding as wam_noise_add
          o.x = fmaf(sg, nz[4 * q], o.x);
          o.y = fmaf(sg, nz[4 * q + 1], o.y);
          o.z = fmaf(sg, nz[4 * q + 2], o.z);
          o.w = fmaf(sg, nz[4 * q + 3], o.w);
        }
        *reinterpret_cast<float4*>(lds + kPadL + idx) = o;
      } else {
        lds[kPadL + idx] = ok[q] ? v[q] : 0.f;
      }
    }
  }
};

// SmoothGrad noise for one fetched row (group g = e / 4 with e = (c*nh + sr)*nw + idx)
template <int MAXV>
__device__ __forceinline__ void make_noise(float (&nz)[4 * MAXV], int nw, int lane, int64_t row_elem0, float sg,
                                           int64_t img, int64_t smp, uint32_t k0, uint32_t k1, bool valid) {
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int idx = (lane + 64 * q) * 4;
    float z[4];
    wam_normal4((row_elem0 + (idx < nw ? idx : 0)) >> 2, img, smp, k0, k1, z);
    const bool ok = valid && idx < nw;
#pragma unroll
    for (int u = 0; u < 4; ++u) nz[4 * q + u] = ok ? z[u] : 0.f;
  }
}

// pad-slot refresh: lane t < npad owns ext column ext_col (left pads t - p, right pads nw + ...)
struct PadLane {
  int dst;   // lds index of the pad slot (or -1: this lane owns none)
  int src;   // lds index of its source sample (or -1: zero)
};

__device__ __forceinline__ PadLane pad_lane(int lane, int nw, int p, int mode, int padl = kPadL) {
  const int npad_r = p + (nw & 1) + 1;  // right pads (one spare)
  PadLane pl{-1, -1};
  int e;
  if (lane < p) e = lane - p;
  else if (lane < p + npad_r) e = nw + (lane - p);
  else return pl;
  pl.dst = padl + e;
  const int s = wam_ext_index(e, nw, mode);
  pl.src = s >= 0 ? padl + s : -1;
  return pl;
}

__device__ __forceinline__ void refresh_pads(float* lds, const PadLane& pl) {
  float v = 0.f;
  if (pl.src >= 0) v = lds[pl.src];
  wsync();
  if (pl.dst >= 0) lds[pl.dst] = v;
}

// Horizontal analysis of output column j from the padded LDS row (ext column 2j - p + k).
template <int L, int PADL = kPadL>
__device__ __forceinline__ void hfilter(const float* lds, int j, int p, const float (&flo)[L], const float (&fhi)[L],
                                        float& lo, float& hi) {
  const float2* s2 = reinterpret_cast<const float2*>(lds + PADL + 2 * j - p);  // even offset (p, PADL even)
  float a = 0.f, d = 0.f;
#pragma unroll
  for (int k = 0; k < L; k += 2) {
    const float2 v = s2[k >> 1];
    a = fmaf(flo[k], v.x, a);
    d = fmaf(fhi[k], v.x, d);
    a = fmaf(flo[k + 1], v.y, a);
    d = fmaf(fhi[k + 1], v.y, d);
  }
  lo = a;
  hi = d;
}

typedef float wam_f2 __attribute__((ext_vector_type(2)));

// hfilter with (lo, hi) as one packed chain: fp[k] = (flo[k], fhi[k]); the same sums
template <int L, int PADL = kPadL>
__device__ __forceinline__ wam_f2 hfilter_pk(const float* lds, int j, int p, const wam_f2 (&fp)[L]) {
  const float2* s2 = reinterpret_cast<const float2*>(lds + PADL + 2 * j - p);
  wam_f2 acc = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < L; k += 2) {
    const float2 v = s2[k >> 1];
    acc = __builtin_elementwise_fma(fp[k], wam_f2{v.x, v.x}, acc);
    acc = __builtin_elementwise_fma(fp[k + 1], wam_f2{v.y, v.y}, acc);
  }
  return acc;
}

// ------------------------------------------------------------------------------------------------
// One level's streaming synthesis (waverec2 level) for (strip, coefficient rows [qbeg, qend)) of
// one wave, shared by the plane-resident synthesis (dwt2_plane.hip) and the per-level kernel
// (dwt2_fused.hip): every lane keeps a ring of the last L/2 coefficient rows of A/H/V/D (scaled on
// entry: sa for A, sd for the details -- the IG alpha), combines them vertically (polyphase, two
// output rows per coefficient row), exchanges the per-column results through the wave's LDS float4
// row and combines horizontally; lanes L/2-1..63 own complete outputs (a strip yields 130 - L output
// columns). Coefficient rows are fetched kSynPF rows ahead with clamped, unconditional loads.
// vec2: output row bases are 8-byte aligned (pairs stored as float2).
constexpr int kSynPF = 4;

// base[idx] with a 32-bit byte offset: a wave-uniform base stays in SGPRs and the access is one
// global load / store with an SGPR base and a VGPR offset (no 64-bit address arithmetic)
__device__ __forceinline__ const float* at32(const float* base, unsigned idx) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + idx * 4u);
}
__device__ __forceinline__ float* at32(float* base, unsigned idx) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(base) + idx * 4u);
}

constexpr int syn_gcd(int a, int b) { return b == 0 ? a : syn_gcd(b, a % b); }
constexpr int syn_lcm(int a, int b) { return a / syn_gcd(a, b) * b; }

// acc += w * (x, x): one v_pk_fma_f32 (PK) or two scalar fmas -- the same sums either way
template <bool PK, class F2>
__device__ __forceinline__ void syn_fma2(F2& acc, F2 w, float x) {
  if constexpr (PK) {
    acc = __builtin_elementwise_fma(w, F2{x, x}, acc);
  } else {
    acc.x = fmaf(w.x, x, acc.x);
    acc.y = fmaf(w.y, x, acc.y);
  }
}

// PK (long filters, where the level synthesis is VALU-bound): packed fp32 FMAs over a static
// register ring, lcm(H2, PF) rows per iteration (sym8 at 512^2: 444 -> 353 us per 2-alpha finest
// level). Short filters keep scalar chains and a shifted ring: the memory-bound plane synthesis
// measured 447 vs 439 us in the static-ring form (profiles/r03j_kbench_syn_ab.log)
// Output sinks of syn_stream: where the reconstructed pixels of a level go (element index idx =
// row * ow + column of the level's output plane).
struct SynOutF32 {  // fp32 plane, row-major (HBM or LDS); a pixel pair as one 8-byte store
  float* dst;
  __device__ __forceinline__ void pair(unsigned idx, float a, float b) const {
    *reinterpret_cast<float2*>(at32(dst, idx)) = make_float2(a, b);
  }
  __device__ __forceinline__ void one(unsigned idx, float a) const { *at32(dst, idx) = a; }
};

// fp32 -> bf16, round to nearest even, NaN -> 0x7FC0: torch's float -> BFloat16 conversion bit for bit
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return f != f ? (uint16_t)0x7FC0u : (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// bf16 channel-interleaved plane (NHWC with C channels): pixel idx of this channel at dst[idx * C]
// (dst = image base + channel). The C channel planes of an image are reconstructed by C
// neighbouring workgroups of one XCD, so their partial-line stores meet in that XCD's L2.
template <int C>
struct SynOutBf16 {
  uint16_t* dst;
  __device__ __forceinline__ void one(unsigned idx, float a) const {
    *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(dst) + 2u * C * idx) = bf16_rne(a);
  }
  __device__ __forceinline__ void pair(unsigned idx, float a, float b) const {
    one(idx, a);
    one(idx + 1, b);
  }
};

template <int L, int PF = kSynPF, bool PK = (L >= 12), class Out = SynOutF32>
__device__ __forceinline__ void syn_stream_to(const float* __restrict__ pA, float sa, const float* __restrict__ pH,
                                              const float* __restrict__ pV, const float* __restrict__ pD, float sd,
                                              int mh, int mw, const Out dst, int oh, int ow, int strip,
                                              int qbeg, int qend, float4* xch, const float (&rlo)[L],
                                              const float (&rhi)[L], int lane, bool vec2 = true) {
  constexpr int p = L - 2;
  constexpr int H2 = L / 2;
  constexpr int OUTQ = 65 - H2;
  const int qs = p >> 1;
  const int jj = qs + strip * OUTQ - (H2 - 1) + lane;
  const bool colv = jj >= 0 && jj < mw;
  const int jc = min(max(jj, 0), mw - 1);
  const bool producer = lane >= H2 - 1;
  const int ucol = 2 * (jj - qs);
  // raw fetched rows (a, h, v, d) + validity; scaled / zeroed when they enter the ring
  float fa[PF], fh[PF], fv[PF], fd[PF];
  bool fok[PF];
  auto fetch = [&](int u, int q) {
    fok[u] = colv && q >= 0 && q < mh;
    // unsigned 32-bit element offsets from the (wave-uniform) band bases: SGPR-base loads, no
    // 64-bit address arithmetic per row
    const unsigned o = (unsigned)(min(max(q, 0), mh - 1) * mw + jc);
    fa[u] = *at32(pA, o);
    fh[u] = *at32(pH, o);
    fv[u] = *at32(pV, o);
    fd[u] = *at32(pD, o);
  };
  if constexpr (PK) {
    // filter pairs (taps 2 i2, 2 i2 + 1): the two outputs of a phase pair as one (packed) chain
    // pair, every output keeping the scalar chain's tap order (same sums)
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 flo2[H2], fhi2[H2];
  #pragma unroll
    for (int i2 = 0; i2 < H2; ++i2) {
      flo2[i2] = f2{rlo[2 * i2], rlo[2 * i2 + 1]};
      fhi2[i2] = f2{rhi[2 * i2], rhi[2 * i2 + 1]};
    }
    // ring of the last H2 coefficient rows in static slots: row qbeg - (H2 - 1) + k in slot k mod H2
    float ra[H2], rh[H2], rv[H2], rd[H2];
  #pragma unroll
    for (int k = 0; k < H2 - 1; ++k) {
      fetch(0, qbeg - (H2 - 1) + k);
      ra[k] = fok[0] ? sa * fa[0] : 0.f;
      rh[k] = fok[0] ? sd * fh[0] : 0.f;
      rv[k] = fok[0] ? sd * fv[0] : 0.f;
      rd[k] = fok[0] ? sd * fd[0] : 0.f;
    }
  #pragma unroll
    for (int u = 0; u < PF; ++u) fetch(u, qbeg + u);
    // rows per iteration lcm(H2, PF): ring slots and fetch buffers static across iterations
    constexpr int GR = syn_lcm(H2, PF);
    for (int base = qbeg; base < qend; base += GR) {
  #pragma unroll
      for (int u = 0; u < GR; ++u) {
        const int q = base + u;
        if (q >= qend) break;  // uniform
        const int uf = u % PF;
        const int ns = (H2 - 1 + u) % H2;  // slot of row q
        ra[ns] = fok[uf] ? sa * fa[uf] : 0.f;
        rh[ns] = fok[uf] ? sd * fh[uf] : 0.f;
        rv[ns] = fok[uf] ? sd * fv[uf] : 0.f;
        rd[ns] = fok[uf] ? sd * fd[uf] : 0.f;
        // rows past the chunk are never used: re-fetch the chunk's last row (a cache hit) rather
        // than the next chunk's first rows, which that chunk's wave read long ago (HBM re-reads)
        fetch(uf, min(q + PF, qend - 1));
        f2 lo = {0.f, 0.f}, hi = {0.f, 0.f};  // (lo0, lo1), (hi0, hi1)
  #pragma unroll
        for (int i2 = 0; i2 < H2; ++i2) {
          const int sl = (ns - i2 + H2) % H2;  // row q - i2
          syn_fma2<PK>(lo, flo2[i2], ra[sl]);
          syn_fma2<PK>(lo, fhi2[i2], rh[sl]);
          syn_fma2<PK>(hi, flo2[i2], rv[sl]);
          syn_fma2<PK>(hi, fhi2[i2], rd[sl]);
        }
        xch[lane] = make_float4(lo.x, lo.y, hi.x, hi.y);
        wsync();
        if (producer) {
          f2 o0 = {0.f, 0.f}, o1 = {0.f, 0.f};  // (o00, o01), (o10, o11)
  #pragma unroll
          for (int i2 = 0; i2 < H2; ++i2) {
            const float4 n = xch[lane - i2];
            syn_fma2<PK>(o0, flo2[i2], n.x);
            syn_fma2<PK>(o0, fhi2[i2], n.z);
            syn_fma2<PK>(o1, flo2[i2], n.y);
            syn_fma2<PK>(o1, fhi2[i2], n.w);
          }
          const int r0 = 2 * (q - qs);
          if (ucol >= 0 && ucol < ow) {
            const bool two = ucol + 1 < ow, pair = two && vec2;
            if (pair && r0 + 1 < oh) {
              // the common case in one block: both chains are used by it, so the compiler keeps
              // them interleaved (with a store branch per row it sank each 2 H2-deep dependent
              // chain into its own branch, back to back)
              dst.pair((unsigned)(r0 * ow + ucol), o0.x, o0.y);
              dst.pair((unsigned)((r0 + 1) * ow + ucol), o1.x, o1.y);
            } else {
              if (r0 < oh) {
                const unsigned d0 = (unsigned)(r0 * ow + ucol);
                if (pair) {
                  dst.pair(d0, o0.x, o0.y);
                } else {
                  dst.one(d0, o0.x);
                  if (two) dst.one(d0 + 1, o0.y);
                }
              }
              if (r0 + 1 < oh) {
                const unsigned d1 = (unsigned)((r0 + 1) * ow + ucol);
                if (pair) {
                  dst.pair(d1, o1.x, o1.y);
                } else {
                  dst.one(d1, o1.x);
                  if (two) dst.one(d1 + 1, o1.y);
                }
              }
            }
          }
        }
        wsync();
      }
    }
  } else {  // short filters: scalar chains, ring shifted by register moves
    float ra[H2], rh[H2], rv[H2], rd[H2];
  #pragma unroll
    for (int k = 0; k < H2 - 1; ++k) {
      fetch(0, qbeg - (H2 - 1) + k);
      ra[k] = fok[0] ? sa * fa[0] : 0.f;
      rh[k] = fok[0] ? sd * fh[0] : 0.f;
      rv[k] = fok[0] ? sd * fv[0] : 0.f;
      rd[k] = fok[0] ? sd * fd[0] : 0.f;
    }
  #pragma unroll
    for (int u = 0; u < PF; ++u) fetch(u, qbeg + u);
    for (int base = qbeg; base < qend; base += PF) {
  #pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int q = base + u;
        ra[H2 - 1] = fok[u] ? sa * fa[u] : 0.f;
        rh[H2 - 1] = fok[u] ? sd * fh[u] : 0.f;
        rv[H2 - 1] = fok[u] ? sd * fv[u] : 0.f;
        rd[H2 - 1] = fok[u] ? sd * fd[u] : 0.f;
        fetch(u, min(q + PF, qend - 1));  // past the chunk: the chunk's last row again (see PK)
        float lo0 = 0.f, lo1 = 0.f, hi0 = 0.f, hi1 = 0.f;
  #pragma unroll
        for (int i2 = 0; i2 < H2; ++i2) {
          const int sl = H2 - 1 - i2;
          lo0 = fmaf(rlo[2 * i2], ra[sl], lo0);
          lo0 = fmaf(rhi[2 * i2], rh[sl], lo0);
          lo1 = fmaf(rlo[2 * i2 + 1], ra[sl], lo1);
          lo1 = fmaf(rhi[2 * i2 + 1], rh[sl], lo1);
          hi0 = fmaf(rlo[2 * i2], rv[sl], hi0);
          hi0 = fmaf(rhi[2 * i2], rd[sl], hi0);
          hi1 = fmaf(rlo[2 * i2 + 1], rv[sl], hi1);
          hi1 = fmaf(rhi[2 * i2 + 1], rd[sl], hi1);
        }
        xch[lane] = make_float4(lo0, lo1, hi0, hi1);
        wsync();
        if (producer && q < qend) {
          float o00 = 0.f, o01 = 0.f, o10 = 0.f, o11 = 0.f;
  #pragma unroll
          for (int i2 = 0; i2 < H2; ++i2) {
            const float4 n = xch[lane - i2];
            o00 = fmaf(rlo[2 * i2], n.x, o00);
            o00 = fmaf(rhi[2 * i2], n.z, o00);
            o01 = fmaf(rlo[2 * i2 + 1], n.x, o01);
            o01 = fmaf(rhi[2 * i2 + 1], n.z, o01);
            o10 = fmaf(rlo[2 * i2], n.y, o10);
            o10 = fmaf(rhi[2 * i2], n.w, o10);
            o11 = fmaf(rlo[2 * i2 + 1], n.y, o11);
            o11 = fmaf(rhi[2 * i2 + 1], n.w, o11);
          }
          const int r0 = 2 * (q - qs);
          if (ucol >= 0 && ucol < ow) {
            const bool two = ucol + 1 < ow, pair = two && vec2;
            if (pair && r0 + 1 < oh) {  // the common case in one block (see the PK form)
              dst.pair((unsigned)(r0 * ow + ucol), o00, o01);
              dst.pair((unsigned)((r0 + 1) * ow + ucol), o10, o11);
            } else {
              if (r0 < oh) {
                const unsigned d0 = (unsigned)(r0 * ow + ucol);
                if (pair) {
                  dst.pair(d0, o00, o01);
                } else {
                  dst.one(d0, o00);
                  if (two) dst.one(d0 + 1, o01);
                }
              }
              if (r0 + 1 < oh) {
                const unsigned d1 = (unsigned)((r0 + 1) * ow + ucol);
                if (pair) {
                  dst.pair(d1, o10, o11);
                } else {
                  dst.one(d1, o10);
                  if (two) dst.one(d1 + 1, o11);
                }
              }
            }
          }
        }
        wsync();
  #pragma unroll
        for (int k = 0; k < H2 - 1; ++k) {
          ra[k] = ra[k + 1];
          rh[k] = rh[k + 1];
          rv[k] = rv[k + 1];
          rd[k] = rd[k + 1];
        }
      }
    }
  }
}

template <int L, int PF = kSynPF, bool PK = (L >= 12)>
__device__ __forceinline__ void syn_stream(const float* __restrict__ pA, float sa, const float* __restrict__ pH,
                                           const float* __restrict__ pV, const float* __restrict__ pD, float sd,
                                           int mh, int mw, float* __restrict__ dst, int oh, int ow, int strip,
                                           int qbeg, int qend, float4* xch, const float (&rlo)[L],
                                           const float (&rhi)[L], int lane, bool vec2 = true) {
  syn_stream_to<L, PF, PK>(pA, sa, pH, pV, pD, sd, mh, mw, SynOutF32{dst}, oh, ow, strip, qbeg, qend, xch, rlo, rhi,
                           lane, vec2);
}

}  // namespace wam_rows
