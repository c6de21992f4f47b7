// Counter-based Philox4x32-10 + Box-Muller, shared by the standalone noise kernel and the fused
// noisy analysis so both produce the same stream: counter = (g, (g >> 32) ^ (item << 8),
// sample, item) with g = element index within the item / 4; key = seed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct wam_u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ wam_u4 wam_philox4x32_10(wam_u4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per 32x32->64 product instead of separate mul_hi / mul_lo
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    // three-input xor as one v_bitop3_b32 (truth table 0x96; gfx950) instead of two v_xor_b32
    c = {(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
         (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
    k0 += W0;
    k1 += W1;
    // keep the key schedule as two scalar registers advanced by SALU adds: folded into 20
    // constants it exceeds the SGPR budget of the plane kernels and is spilled to VGPR lanes
    // (one v_readlane + hazard nop per use)
    asm volatile("" : "+s"(k0), "+s"(k1));
  }
  return c;
}

// Box-Muller on the hardware transcendentals (v_log_f32 = log2, v_sqrt_f32, v_sin/v_cos_f32 take
// the angle in revolutions): ~1 ulp each, a handful of instructions instead of the libm paths.
__device__ __forceinline__ void wam_box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float two32inv = 2.3283064365386963e-10f;  // 2^-32
  const float u1 = ((float)a + 1.0f) * two32inv;   // (0, 1]
  const float u2 = (float)b * two32inv;            // [0, 1)
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // sqrt(-2 ln u1)
  z0 = r * __builtin_amdgcn_cosf(u2);
  z1 = r * __builtin_amdgcn_sinf(u2);
}

// Two independent Philox4x32-10 blocks advanced round by round in lockstep: the two dependent
// v_mad_u64_u32 -> v_bitop3 chains interleave, so one wave keeps twice the multiplies in flight.
__device__ __forceinline__ void wam_philox4x32_10_x2(wam_u4& a, wam_u4& b, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t pa0 = (uint64_t)M0 * a.x, pa1 = (uint64_t)M1 * a.z;
    const uint64_t pb0 = (uint64_t)M0 * b.x, pb1 = (uint64_t)M1 * b.z;
    a = {(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(pa1 >> 32), a.y, k0, 0x96), (uint32_t)pa1,
         (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(pa0 >> 32), a.w, k1, 0x96), (uint32_t)pa0};
    b = {(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(pb1 >> 32), b.y, k0, 0x96), (uint32_t)pb1,
         (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(pb0 >> 32), b.w, k1, 0x96), (uint32_t)pb0};
    k0 += W0;
    k1 += W1;
    asm volatile("" : "+s"(k0), "+s"(k1));
  }
}

// four N(0,1) values for element group g of `item` in `sample`
__device__ __forceinline__ void wam_normal4(int64_t g, int64_t item, int64_t sample, uint32_t k0, uint32_t k1,
                                            float z[4]) {
  wam_u4 c = {(uint32_t)g, (uint32_t)(g >> 32) ^ ((uint32_t)item << 8), (uint32_t)sample, (uint32_t)item};
  wam_u4 r = wam_philox4x32_10(c, k0, k1);
  wam_box_muller(r.x, r.y, z[0], z[1]);
  wam_box_muller(r.z, r.w, z[2], z[3]);
}

// wam_normal4 for two element groups ga, gb < 2^32 of the same (item, sample), generated together:
// with g < 2^32 the counter word (g >> 32) ^ (item << 8) is the uniform item << 8, so the stream is
// the same as wam_normal4's.
__device__ __forceinline__ void wam_normal4_x2(uint32_t ga, uint32_t gb, uint32_t item, uint32_t sample, uint32_t k0,
                                               uint32_t k1, float za[4], float zb[4]) {
  wam_u4 a = {ga, item << 8, sample, item}, b = {gb, item << 8, sample, item};
  wam_philox4x32_10_x2(a, b, k0, k1);
  wam_box_muller(a.x, a.y, za[0], za[1]);
  wam_box_muller(a.z, a.w, za[2], za[3]);
  wam_box_muller(b.x, b.y, zb[0], zb[1]);
  wam_box_muller(b.z, b.w, zb[2], zb[3]);
}
