// Arrow-style batch buffers for the streaming ParquetHandler reader (dk_reader_*, include/dkgpu.h).
//
// The reference hands a connector ColumnarBatches of at most `parquet.reader.batch-size` rows
// (ParquetFileReader.java:54-147, DefaultColumnarBatch); the engine keeps the decoded columns in HBM
// and ships them to pinned host memory one window of batches at a time. Per leaf and window, one
// launch derives what the decoded layout does not hold directly:
//   validity bits  value i non-null iff its definition level equals the leaf's max_def
//                  (ballot per wave -> one u64 word per 64 values, LSB first)
//   int32 offsets  byte-array offsets and repeated-leaf row offsets, rebased to the window
// Everything else (row_def, entry_def, fixed-width values, chars) is a contiguous slice of the
// decoded column and goes to the host with a plain async copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dk_device.h"

namespace dk {


__global__ __launch_bounds__(256) void k_arrow_window(ArrowWin A) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = A.nv > A.nr ? A.nv : A.nr;
  if (i > n) return;
  // validity: the wave owns 64 consecutive values (word i / 64)
  const bool nn = i < A.nv && A.def[i] == A.max_def;
  const unsigned long long m = __ballot(nn);
  if ((threadIdx.x & 63) == 0 && i < A.nv) A.bits[i >> 6] = m;
  if (A.offs && i <= A.nv) {
    const int64_t v = A.offs[i] - A.offs[0];
    if (v > 0x7fffffffll) *A.overflow = 1;
    A.offs32[i] = (int32_t)v;
  }
  if (A.row_offs && i <= A.nr) {
    const int64_t v = A.row_offs[i] - A.row_offs[0];
    if (v > 0x7fffffffll) *A.overflow = 1;
    A.row_offs32[i] = (int32_t)v;
  }
}

void launch_arrow_window(const ArrowWin& A, hipStream_t s) {
  const int64_t n = (A.nv > A.nr ? A.nv : A.nr) + 1;
  hipLaunchKernelGGL(k_arrow_window, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A);
}

}  // namespace dk
