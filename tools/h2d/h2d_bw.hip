// H2D bandwidth probe (round 4): pinned host -> HBM by hipMemcpyAsync in 8 MiB pieces over 1-8
// streams, and by a copy kernel reading the pinned buffer directly (zero-copy), 1 GiB each.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <vector>
__global__ void k_copy(uint4* __restrict__ d, const uint4* __restrict__ s, long long n16) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) d[i] = s[i];
}
int main() {
  const size_t N = 1ull << 30, P = 8ull << 20;
  void *h = nullptr, *d = nullptr;
  if (hipHostMalloc(&h, N, hipHostMallocDefault) != hipSuccess || hipMalloc(&d, N) != hipSuccess) { printf("alloc failed\n"); return 1; }
  memset(h, 1, N);
  std::vector<hipStream_t> st(8);
  for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int ns : {1, 2, 4, 8}) {
    for (int rep = 0; rep < 3; rep++) {
      hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (size_t o = 0, k = 0; o < N; o += P, k++) hipMemcpyAsync((char*)d + o, (char*)h + o, P, hipMemcpyHostToDevice, st[k % ns]);
      for (int k = 0; k < ns; k++) hipStreamSynchronize(st[k]);
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rep == 2) printf("memcpyAsync %d streams: %.1f GB/s\n", ns, N / ms / 1e6);
    }
  }
  for (int blocks : {256, 1024, 4096}) {
    for (int rep = 0; rep < 3; rep++) {
      hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, st[0], (uint4*)d, (const uint4*)h, (long long)(N / 16));
      hipStreamSynchronize(st[0]);
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rep == 2) printf("zero-copy kernel %d blocks: %.1f GB/s\n", blocks, N / ms / 1e6);
    }
  }
  // D2H while H2D runs (full duplex?)
  void* h2 = nullptr; hipHostMalloc(&h2, N, hipHostMallocDefault);
  for (int rep = 0; rep < 2; rep++) {
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (size_t o = 0, k = 0; o < N; o += P, k++) {
      hipMemcpyAsync((char*)d + o, (char*)h + o, P, hipMemcpyHostToDevice, st[k % 4]);
      hipMemcpyAsync((char*)h2 + o, (char*)d + o, P / 8, hipMemcpyDeviceToHost, st[4 + k % 4]);
    }
    hipDeviceSynchronize();
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rep == 1) printf("H2D 1 GiB + D2H 128 MiB concurrently: %.1f ms (H2D-equivalent %.1f GB/s)\n", ms, N / ms / 1e6);
  }
  return 0;
}
