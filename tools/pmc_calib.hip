// FETCH_SIZE / WRITE_SIZE calibration for the access widths of this repo's kernels
// (MI355X_MICROARCH.md §HBM: the counters read 1/2 of the bytes of 16-B-per-lane streaming
// loads and "other access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern").  Each kernel streams a known byte count (1 GiB, past the 256 MiB Infinity
// Cache) once with one access width; scripts/pmc_calibrate.py divides the counters of
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes of this program by those counts.
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/_bin/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;

template <class T>
__global__ __launch_bounds__(256) void calib_read(const T* __restrict__ src, size_t n,
                                                  uint32_t* __restrict__ sink, uint32_t magic) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = src[i];
    const uint32_t* w = (const uint32_t*)&v;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) >= 4 ? sizeof(T) / 4 : 1); k++)
      acc ^= sizeof(T) >= 4 ? w[k] : (uint32_t)(*(const uint8_t*)&v);
  }
  // never true for the zero buffer, so no stores; `magic` is a kernel argument so the compiler
  // cannot prove the comparison false (a literal above 255 let it delete the whole 1-B loop,
  // which is why round 1 saw FETCH_SIZE = 0 for 1-B loads)
  if (acc == magic) sink[blockIdx.x] = acc;
}

template <class T>
__global__ __launch_bounds__(256) void calib_write(T* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = (T)i;
}

// 16 B per lane (uint4): the staged windows of k_fast_tile / k_cvfast / k_blur
__global__ __launch_bounds__(256) void calib_read16(const uint4* __restrict__ src, size_t n,
                                                    uint32_t* __restrict__ sink, uint32_t magic) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == magic) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void calib_write16(uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = make_uint4((uint32_t)i, 0u, 0u, 0u);
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 65536 * sizeof(uint32_t)));
  CK(hipMemset(buf, 0, kBytes));
  CK(hipDeviceSynchronize());
  const dim3 grid(8192), block(256);
  hipLaunchKernelGGL(calib_read<uint64_t>, grid, block, 0, 0, (const uint64_t*)buf, kBytes / 8, sink, 0x9E3779B9u);
  hipLaunchKernelGGL(calib_read<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, kBytes / 4, sink, 0x9E3779B9u);
  hipLaunchKernelGGL(calib_read<uint8_t>, grid, block, 0, 0, (const uint8_t*)buf, kBytes, sink, 0x9E3779B9u);
  hipLaunchKernelGGL(calib_read16, grid, block, 0, 0, (const uint4*)buf, kBytes / 16, sink, 0x9E3779B9u);
  hipLaunchKernelGGL(calib_write16, grid, block, 0, 0, (uint4*)buf, kBytes / 16);
  hipLaunchKernelGGL(calib_write<uint64_t>, grid, block, 0, 0, (uint64_t*)buf, kBytes / 8);
  hipLaunchKernelGGL(calib_write<uint32_t>, grid, block, 0, 0, (uint32_t*)buf, kBytes / 4);
  hipLaunchKernelGGL(calib_write<uint8_t>, grid, block, 0, 0, (uint8_t*)buf, kBytes);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"bytes_per_kernel\": %zu}\n", kBytes);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
