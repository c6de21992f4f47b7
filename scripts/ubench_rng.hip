// Throughput microbench of the SmoothGrad noise generator pieces on one MI355X (not part of the
// library): v_mad_u64_u32 vs 24-bit / 32-bit multiplies, Philox4x32-R rounds, and Philox + Box-Muller
// normals per second with every CU busy. Each lane runs NCH independent chains (ILP) and the result
// is folded into one store per lane so nothing is dead code.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_rng.hip -o scripts/ubench_rng
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../wam_amd/csrc/rng.hpp"

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                      \
    }                                                                \
  } while (0)

constexpr int NCH = 8;

template <int OP>
__global__ void __launch_bounds__(256) k_mul(uint32_t* out, int iters, uint32_t m) {
  uint32_t a[NCH], b[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    a[c] = threadIdx.x * 7u + c;
    b[c] = blockIdx.x + c;
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if constexpr (OP == 0) {  // v_mad_u64_u32
        const uint64_t p = (uint64_t)m * a[c];
        a[c] = (uint32_t)(p >> 32) ^ b[c];
        b[c] = (uint32_t)p;
      } else if constexpr (OP == 1) {  // v_mul_hi_u32 + v_mul_lo_u32
        a[c] = __umulhi(m, a[c]) ^ b[c];
        b[c] = m * b[c];
      } else if constexpr (OP == 2) {  // 24-bit multiplies (full rate)
        a[c] = __umul24(a[c], m) ^ b[c];
        b[c] = (uint32_t)(((uint64_t)(b[c] & 0xFFFFFFu) * (m & 0xFFFFFFu)) >> 32) + a[c];
      } else {  // plain xor/add (baseline)
        a[c] = (a[c] ^ m) + b[c];
        b[c] = b[c] + a[c];
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= a[c] + b[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int ROUNDS>
__device__ __forceinline__ wam_u4 philox_r(wam_u4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    c = {(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
         (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0};
    k0 += W0;
    k1 += W1;
    asm volatile("" : "+s"(k0), "+s"(k1));
  }
  return c;
}

// MODE 0: Philox-R words only; MODE 1: Philox-R + Box-Muller normals
template <int ROUNDS, int MODE, int ILP>
__global__ void __launch_bounds__(256) k_noise(float* out, int iters, uint32_t k0, uint32_t k1) {
  float acc = 0.f;
  uint32_t accu = 0;
  const uint32_t g0 = (blockIdx.x * 256 + threadIdx.x) * (uint32_t)iters * ILP;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < ILP; ++c) {
      wam_u4 ctr = {g0 + i * ILP + c, 0u, 7u, 3u};
      wam_u4 r = philox_r<ROUNDS>(ctr, k0, k1);
      if constexpr (MODE == 0) {
        accu ^= r.x + r.y + r.z + r.w;
      } else {
        float z0, z1, z2, z3;
        wam_box_muller(r.x, r.y, z0, z1);
        wam_box_muller(r.z, r.w, z2, z3);
        acc += (z0 + z1) + (z2 + z3);
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc + (float)accu;
}

template <typename F>
static float time_it(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 16;  // 16 workgroups of 4 waves per CU
  const int threads = 256;
  float* out;
  CK(hipMalloc(&out, sizeof(float) * blocks * threads));
  const int iters = 256;
  const double waves = (double)blocks * threads / 64;
  auto report_mul = [&](const char* name, float ms, int per_iter) {
    const double inst = waves * iters * NCH * per_iter;
    // cycles per wave-instruction per SIMD at 2.4 GHz: SIMD-cycles available / instructions
    printf("%-34s %8.3f ms  %6.2f SIMD-cycles per wave-instruction (2.4 GHz, 1024 SIMDs)\n", name, ms,
           ms * 1e-3 * 2.4e9 * 1024 / inst);
  };
  report_mul("v_mad_u64_u32 (+xor)", time_it([&] { k_mul<0><<<blocks, threads>>>((uint32_t*)out, iters, 0xD2511F53u); }), 2);
  report_mul("v_mul_hi_u32 + v_mul_lo_u32 (+xor)", time_it([&] { k_mul<1><<<blocks, threads>>>((uint32_t*)out, iters, 0xD2511F53u); }), 3);
  report_mul("v_mul_u32_u24 + v_mul_hi_u32_u24", time_it([&] { k_mul<2><<<blocks, threads>>>((uint32_t*)out, iters, 0x511F53u); }), 4);
  report_mul("xor/add baseline", time_it([&] { k_mul<3><<<blocks, threads>>>((uint32_t*)out, iters, 0xD2511F53u); }), 3);
  const int it2 = 64;
  auto report_n = [&](const char* name, float ms, int ilp, int per) {
    const double n = (double)blocks * threads * it2 * ilp * per;
    printf("%-34s %8.3f ms  %8.1f G values/s  %6.1f SIMD-cycles per wave of 64 values\n", name, ms, n / (ms * 1e-3) / 1e9,
           ms * 1e-3 * 2.4e9 * 1024 / (n / 64));
  };
  report_n("philox4x32-10 words", time_it([&] { k_noise<10, 0, 4><<<blocks, threads>>>(out, it2, 1u, 2u); }), 4, 4);
  report_n("philox4x32-7 words", time_it([&] { k_noise<7, 0, 4><<<blocks, threads>>>(out, it2, 1u, 2u); }), 4, 4);
  report_n("philox4x32-10 + BM normals ILP1", time_it([&] { k_noise<10, 1, 1><<<blocks, threads>>>(out, it2, 1u, 2u); }), 1, 4);
  report_n("philox4x32-10 + BM normals ILP2", time_it([&] { k_noise<10, 1, 2><<<blocks, threads>>>(out, it2, 1u, 2u); }), 2, 4);
  report_n("philox4x32-10 + BM normals ILP4", time_it([&] { k_noise<10, 1, 4><<<blocks, threads>>>(out, it2, 1u, 2u); }), 4, 4);
  report_n("philox4x32-7 + BM normals ILP4", time_it([&] { k_noise<7, 1, 4><<<blocks, threads>>>(out, it2, 1u, 2u); }), 4, 4);
  CK(hipFree(out));
  return 0;
}
