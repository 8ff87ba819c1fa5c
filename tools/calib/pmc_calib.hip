// FETCH_SIZE / WRITE_SIZE calibration for the access widths the decode kernels use (the guide
// calibrates only 16-byte-per-lane streaming reads): each kernel streams N bytes once, coalesced,
// with 16, 8, 4 or 1 bytes per lane per load, and writes 16 / 4 bytes per lane per store. Run under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); tools/pmc_summary.py divides
// the counters by the known byte counts (tools/pmc_calib.sh).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <class T>
__global__ void rd(const T* __restrict__ in, size_t n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = in[i];
    const unsigned* w = (const unsigned*)&v;
    for (size_t k = 0; k < (sizeof(T) + 3) / 4; k++) acc ^= sizeof(T) >= 4 ? w[k] : (unsigned)((const uint8_t*)&v)[0];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;       // keeps the loads
}
template <class T>
__global__ void wr(T* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v; memset(&v, (int)(i & 0xff), sizeof v);
    out[i] = v;
  }
}

int main() {
  const size_t bytes = (size_t)2 << 30;        // 2 GiB: far past the 256 MiB Infinity Cache
  uint8_t* buf; unsigned* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(buf, 1, bytes);
  hipDeviceSynchronize();
  dim3 g(8192), b(256);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(rd<uint4>, g, b, 0, 0, (const uint4*)buf, bytes / 16, sink);
    hipLaunchKernelGGL(rd<uint2>, g, b, 0, 0, (const uint2*)buf, bytes / 8, sink);
    hipLaunchKernelGGL(rd<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, bytes / 4, sink);
    hipLaunchKernelGGL(rd<uint8_t>, g, b, 0, 0, (const uint8_t*)buf, bytes, sink);
    hipLaunchKernelGGL(wr<uint4>, g, b, 0, 0, (uint4*)buf, bytes / 16);
    hipLaunchKernelGGL(wr<uint32_t>, g, b, 0, 0, (uint32_t*)buf, bytes / 4);
    hipLaunchKernelGGL(wr<uint8_t>, g, b, 0, 0, (uint8_t*)buf, bytes);
  }
  hipDeviceSynchronize();
  printf("bytes per kernel %zu\n", bytes);
  return 0;
}
