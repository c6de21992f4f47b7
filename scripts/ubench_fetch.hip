// FETCH_SIZE / WRITE_SIZE calibration on gfx950 (not part of the library): the same 1 GiB streaming
// copy with 16-byte, 8-byte and 4-byte loads per lane. Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./scripts/ubench_fetch   (and a separate --pmc WRITE_SIZE pass)
// and compare each kernel's counter with its 1 GiB read / 1 GiB write: the guide's x2 correction of
// FETCH_SIZE is documented for 16-B-per-lane reads; the 4-B form is what several WAM kernels use.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_fetch.hip -o scripts/ubench_fetch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <typename T>
__global__ void __launch_bounds__(256) k_copy_w(int64_t n, const T* __restrict__ src, T* __restrict__ dst) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    dst[t] = src[t];
}

int main() {
  const int64_t bytes = 1ll << 30;
  void *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  hipMemset(a, 1, bytes);
  const int grid = 256 * 64;
  for (int rep = 0; rep < 2; ++rep) {
    k_copy_w<float4><<<grid, 256>>>(bytes / 16, (const float4*)a, (float4*)b);
    k_copy_w<float2><<<grid, 256>>>(bytes / 8, (const float2*)a, (float2*)b);
    k_copy_w<float><<<grid, 256>>>(bytes / 4, (const float*)a, (float*)b);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("done: 3 copy widths x 2, 1 GiB each\n");
  return 0;
}
