// Deletion-vector bitmaps on the GPU (dk_dv_*, include/dkgpu.h).
//
// Reference: DeletionVectorStoredBitmap.load / RoaringBitmapArray.readFrom
// (kernel-api/.../internal/deletionvectors/DeletionVectorStoredBitmap.java:50-116,
// RoaringBitmapArray.java:100-229) over org.roaringbitmap:RoaringBitmap 0.9.25's portable container
// format, and SelectionColumnVector (internal/data/SelectionColumnVector.java) for the per-row test
// Scan.transformPhysicalData applies (Scan.java:176-199). The host validates the stored bytes (size,
// CRC-32, magic, container headers) and lists the containers; the device expands every container of
// every DV into one dense deleted-row bitmap per DV, then answers `contains(rowIndex)` per data row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dk_device.h"

namespace dk {

// one workgroup (64 lanes) per container
__global__ __launch_bounds__(64) void k_dv_expand(const DvCont* __restrict__ conts, const uint8_t* __restrict__ blob,
                                                  unsigned long long* __restrict__ bits) {
  const DvCont c = conts[blockIdx.x];
  const uint8_t* s = blob + c.src;
  unsigned long long* out = bits + c.out_word;
  const int lane = threadIdx.x;
  if (c.type == DV_BITMAP) {             // 1024 little-endian u64 words
    for (int w = lane; w < 1024; w += 64) {
      if (c.word0 + w >= c.nwords) break;
      unsigned long long v = 0;
#pragma unroll
      for (int b = 0; b < 8; b++) v |= (unsigned long long)s[8 * w + b] << (8 * b);
      if (v) out[c.word0 + w] = v;      // each word belongs to this container alone
    }
  } else if (c.type == DV_ARRAY) {       // sorted u16 values
    for (int i = lane; i < c.n; i += 64) {
      const uint32_t v = (uint32_t)s[2 * i] | ((uint32_t)s[2 * i + 1] << 8);
      atomicOr(out + c.word0 + (v >> 6), 1ull << (v & 63));
    }
  } else {                               // runs: (start u16, length - 1 u16)
    for (int r = lane; r < c.n; r += 64) {
      const uint32_t st = (uint32_t)s[2 + 4 * r] | ((uint32_t)s[3 + 4 * r] << 8);
      const uint32_t ln = (uint32_t)s[4 + 4 * r] | ((uint32_t)s[5 + 4 * r] << 8);
      const uint32_t en = st + ln;       // inclusive
      for (uint32_t w = st >> 6; w <= (en >> 6); w++) {
        const uint32_t lo = w == (st >> 6) ? (st & 63) : 0, hi = w == (en >> 6) ? (en & 63) : 63;
        const unsigned long long m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo);
        atomicOr(out + c.word0 + w, m);
      }
    }
  }
}

// sel[k] = row_index[k] is not deleted (SelectionColumnVector.getBoolean: !bitmap.contains(rowIndex))
__global__ __launch_bounds__(256) void k_dv_select(const unsigned long long* __restrict__ bits, long long nbits,
                                                   const long long* __restrict__ rows, long long n,
                                                   uint8_t* __restrict__ sel) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const long long r = rows[k];
  const bool del = r >= 0 && r < nbits && ((bits[r >> 6] >> (r & 63)) & 1);
  sel[k] = del ? 0 : 1;
}

void launch_dv_expand(const DvCont* conts, int n, const uint8_t* blob, unsigned long long* bits, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_dv_expand, dim3(n), dim3(64), 0, s, conts, blob, bits);
}

void launch_dv_select(const unsigned long long* bits, long long nbits, const long long* rows, long long n,
                      uint8_t* sel, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_dv_select, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bits, nbits, rows, n, sel);
}

}  // namespace dk
