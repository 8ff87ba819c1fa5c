// Checkpoint Parquet encoder, device half (Table.checkpoint -> ParquetHandler.writeParquetFileAtomically,
// kernel-defaults/.../engine/DefaultParquetHandler.java:110-163 over parquet-mr's ParquetFileWriter,
// kernel-defaults/.../internal/parquet/ParquetFileWriter.java).
//
// Column data of a row group is laid out per leaf as level arrays (def, rep) plus PLAIN value
// material (fixed-width values, or string lengths + chars). Rows that come from the old checkpoint
// are gathered here from its decoded columns by the replay's selection (the bulk: every surviving
// add row); rows built on the host (commit actions, protocol, metaData, ...) are uploaded in the same
// layout. Pages are then encoded in parallel (v1 data pages: RLE/bit-packed hybrid levels written
// as one bit-packed run, PLAIN values) and compressed with snappy, one workgroup per 64 KiB block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dk_device.h"

namespace dk {

constexpr int ENT = 256;

// One leaf of one row group sourced from a decoded checkpoint column: the selected rows (sel_rows,
// in file order) are written in the new file's schema; defmap / emap translate the old file's
// definition levels into the new schema's (0xff: the row violates the new schema -- a required
// field is null).
struct EncSrc {
  const uint8_t* row_def; const int64_t* row_offs; const uint8_t* entry_def;
  const uint8_t* fixed; const int64_t* offs; const uint8_t* chars;
  int32_t width, is_str, repeated, max_def_new;
  int32_t entry_def_old;           // repeated: row_def >= this means the row has entries
  uint8_t defmap[16], emap[16];
};

// per selected row: levels, non-null values, chars (a repeated leaf: one level per entry, or one
// for a null / empty map)
__global__ void k_enc_count(EncSrc S, const int32_t* __restrict__ rows, long long n, long long* __restrict__ nlev,
                            long long* __restrict__ nval, long long* __restrict__ nchr, int* __restrict__ err) {
  for (long long j = (long long)blockIdx.x * ENT + threadIdx.x; j < n; j += (long long)gridDim.x * ENT) {
    const long long r = rows[j];
    long long lv = 1, vv = 0, cc = 0;
    if (S.repeated) {
      const int d = S.row_def[r];
      const long long e0 = S.row_offs[r], e1 = S.row_offs[r + 1];
      if (d >= S.entry_def_old && e1 > e0) {
        lv = e1 - e0;
        for (long long e = e0; e < e1; e++) {
          const uint8_t nd = S.emap[S.entry_def[e]];
          if (nd == 0xff) atomicOr(err, 1);
          else if (nd == S.max_def_new) { vv++; if (S.is_str) cc += S.offs[e + 1] - S.offs[e]; }
        }
      } else if (S.defmap[d] == 0xff) atomicOr(err, 1);
    } else {
      const uint8_t nd = S.defmap[S.row_def[r]];
      if (nd == 0xff) atomicOr(err, 1);
      else if (nd == S.max_def_new) { vv = 1; if (S.is_str) cc = S.offs[r + 1] - S.offs[r]; }
    }
    nlev[j] = lv; nval[j] = vv; if (nchr) nchr[j] = cc;
  }
}

__global__ void k_enc_fill(EncSrc S, const int32_t* __restrict__ rows, long long n, const long long* __restrict__ lbase,
                           const long long* __restrict__ vbase, const long long* __restrict__ cbase,
                           uint8_t* __restrict__ def, uint8_t* __restrict__ rep, uint8_t* __restrict__ vals,
                           int32_t* __restrict__ lens, uint8_t* __restrict__ chars, long long* __restrict__ coff) {
  for (long long j = (long long)blockIdx.x * ENT + threadIdx.x; j < n; j += (long long)gridDim.x * ENT) {
    const long long r = rows[j];
    long long l = lbase[j], v = vbase[j], c = cbase ? cbase[j] : 0;
    auto put = [&](long long src, bool nonnull) {
      if (!nonnull) return;
      if (S.is_str) {
        const long long a = S.offs[src], b = S.offs[src + 1];
        lens[v] = (int32_t)(b - a);
        coff[v] = c;
        for (long long k = a; k < b; k++) chars[c++] = S.chars[k];
      } else {
        for (int k = 0; k < S.width; k++) vals[v * S.width + k] = S.fixed[src * S.width + k];
      }
      v++;
    };
    if (S.repeated) {
      const int d = S.row_def[r];
      const long long e0 = S.row_offs[r], e1 = S.row_offs[r + 1];
      if (d >= S.entry_def_old && e1 > e0) {
        for (long long e = e0; e < e1; e++) {
          const uint8_t nd = S.emap[S.entry_def[e]];
          def[l] = nd; rep[l] = e == e0 ? 0 : 1;
          put(e, nd == S.max_def_new);
          l++;
        }
      } else {
        def[l] = S.defmap[d]; rep[l] = 0;
      }
    } else {
      const uint8_t nd = S.defmap[S.row_def[r]];
      def[l] = nd;
      if (rep) rep[l] = 0;
      put(r, nd == S.max_def_new && S.row_offs == nullptr);
    }
  }
}

// selected rows of a file, in order (sel: one byte per row; pos: exclusive scan of sel)
__global__ void k_enc_sel_rows(const uint8_t* __restrict__ sel, const long long* __restrict__ pos, long long n,
                               int32_t* __restrict__ rows) {
  for (long long r = (long long)blockIdx.x * ENT + threadIdx.x; r < n; r += (long long)gridDim.x * ENT)
    if (sel[r]) rows[pos[r]] = (int32_t)r;
}
__global__ void k_enc_u8_to_i64(const uint8_t* __restrict__ a, long long n, long long* __restrict__ b) {
  for (long long r = (long long)blockIdx.x * ENT + threadIdx.x; r < n; r += (long long)gridDim.x * ENT) b[r] = a[r];
}

// Decoupled-free device exclusive scan of int64 (three passes: block sums, one-block scan of the
// sums, block-local scans plus offsets). Returns the total in *total (device).
constexpr int SCAN_B = 2048;   // elements per block (8 per thread)
__global__ void k_scan_sums(const long long* __restrict__ in, long long n, long long* __restrict__ sums) {
  __shared__ long long red[ENT / 64];
  const long long b0 = (long long)blockIdx.x * SCAN_B;
  long long s = 0;
  for (int k = threadIdx.x; k < SCAN_B; k += ENT) if (b0 + k < n) s += in[b0 + k];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) { long long t = 0; for (int i = 0; i < ENT / 64; i++) t += red[i]; sums[blockIdx.x] = t; }
}
__global__ void k_scan_top(long long* __restrict__ sums, int nb, long long* __restrict__ total) {
  if (threadIdx.x || blockIdx.x) return;
  long long run = 0;
  for (int i = 0; i < nb; i++) { const long long v = sums[i]; sums[i] = run; run += v; }
  *total = run;
}
__global__ void k_scan_down(const long long* __restrict__ in, long long n, const long long* __restrict__ sums,
                            long long* __restrict__ out) {
  __shared__ long long part[ENT];
  const long long b0 = (long long)blockIdx.x * SCAN_B;
  constexpr int PER = SCAN_B / ENT;
  long long v[PER], s = 0;
  for (int k = 0; k < PER; k++) {
    const long long i = b0 + (long long)threadIdx.x * PER + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < ENT; o <<= 1) {
    const long long t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  long long run = sums[blockIdx.x] + part[threadIdx.x] - s;
  for (int k = 0; k < PER; k++) {
    const long long i = b0 + (long long)threadIdx.x * PER + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

// RLE / bit-packed hybrid levels of one page as ONE bit-packed run: varint((groups << 1) | 1), then
// groups of 8 values, bw bits each, LSB first (parquet-format Encodings.md). One thread per group.
__global__ void k_enc_bitpack(const uint8_t* __restrict__ lv, long long n, int bw, uint8_t* __restrict__ out) {
  const long long groups = (n + 7) / 8;
  for (long long g = (long long)blockIdx.x * ENT + threadIdx.x; g < groups; g += (long long)gridDim.x * ENT) {
    uint32_t acc = 0;
    for (int k = 0; k < 8; k++) {
      const long long i = g * 8 + k;
      acc |= (uint32_t)(i < n ? lv[i] : 0) << (bw * k);
    }
    for (int b = 0; b < bw; b++) out[g * bw + b] = (uint8_t)(acc >> (8 * b));
  }
}

// PLAIN BYTE_ARRAY values of a page: per value a 4-byte little-endian length, then its bytes
__global__ void k_enc_plain_str(const int32_t* __restrict__ lens, const long long* __restrict__ coff,
                                const uint8_t* __restrict__ chars, long long v0, long long nv, long long c0,
                                uint8_t* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * ENT + threadIdx.x; i < nv; i += (long long)gridDim.x * ENT) {
    const long long v = v0 + i;
    const long long at = 4 * i + (coff[v] - c0);
    const int32_t L = lens[v];
    out[at] = (uint8_t)L; out[at + 1] = (uint8_t)(L >> 8); out[at + 2] = (uint8_t)(L >> 16); out[at + 3] = (uint8_t)(L >> 24);
    const uint8_t* s = chars + coff[v];
    for (int32_t k = 0; k < L; k++) out[at + 4 + k] = s[k];
  }
}

// Snappy block compressor (the format's 64 KiB blocks, compressed independently, concatenated into
// one stream after the page's varint preamble). One workgroup per block: the block is staged in LDS,
// then one lane runs the greedy parse (a 4096-entry hash table of 4-byte sequences in LDS, minimum
// match 4, copies of <= 64 bytes, literals as they come). The output of block b goes to
// out + b * cap; its length to lens[b].
constexpr int SZ_BLOCK = 65536;
constexpr int SZ_HBITS = 12;
struct SzBlock { long long src; int32_t n; int32_t pad; };

__device__ __forceinline__ uint32_t sz_load32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(64) void k_snappy_compress(const uint8_t* __restrict__ src, const SzBlock* __restrict__ blocks,
                                                        long long cap, uint8_t* __restrict__ out,
                                                        int32_t* __restrict__ lens) {
  __shared__ uint8_t in[SZ_BLOCK + 8];
  __shared__ uint16_t table[1 << SZ_HBITS];
  const SzBlock B = blocks[blockIdx.x];
  const int n = B.n;
  for (int i = threadIdx.x; i < n; i += 64) in[i] = src[B.src + i];
  for (int i = threadIdx.x; i < (1 << SZ_HBITS); i += 64) table[i] = 0xffff;
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint8_t* o = out + (long long)blockIdx.x * cap;
  long long w = 0;
  auto lit = [&](int a, int b) {                    // literal bytes in[a, b)
    while (a < b) {
      const int len = b - a < 65536 ? b - a : 65536;
      const uint32_t l1 = (uint32_t)len - 1;
      if (l1 < 60) o[w++] = (uint8_t)(l1 << 2);
      else if (l1 < 256) { o[w++] = (uint8_t)(60 << 2); o[w++] = (uint8_t)l1; }
      else { o[w++] = (uint8_t)(61 << 2); o[w++] = (uint8_t)l1; o[w++] = (uint8_t)(l1 >> 8); }
      for (int k = 0; k < len; k++) o[w++] = in[a + k];
      a += len;
    }
  };
  auto copy = [&](int off, int len) {               // back reference, split into <= 64-byte copies
    while (len > 0) {
      int l = len > 64 ? 64 : len;
      if (len - l > 0 && len - l < 4) l = len - 4;  // keep every piece >= 4 bytes
      if (l >= 4 && l <= 11 && off < 2048) {
        o[w++] = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5));
        o[w++] = (uint8_t)off;
      } else {
        o[w++] = (uint8_t)(2 | ((l - 1) << 2));
        o[w++] = (uint8_t)off; o[w++] = (uint8_t)(off >> 8);
      }
      len -= l;
    }
  };
  int ip = 0, lit0 = 0;
  while (ip + 4 <= n) {
    const uint32_t v = sz_load32(in + ip);
    const uint32_t h = (v * 0x1e35a7bdu) >> (32 - SZ_HBITS);
    const int cand = table[h];
    table[h] = (uint16_t)ip;
    if (cand != 0xffff && cand < ip && sz_load32(in + cand) == v) {
      int len = 4;
      while (ip + len < n && in[cand + len] == in[ip + len]) len++;
      lit(lit0, ip);
      copy(ip - cand, len);
      ip += len;
      lit0 = ip;
    } else {
      ip++;
    }
  }
  lit(lit0, n);
  lens[blockIdx.x] = (int32_t)w;
}

// ---- launchers ----
static unsigned enc_grid(long long n) {
  const long long want = (n + ENT - 1) / ENT;
  return (unsigned)(want < 4096 ? (want > 0 ? want : 1) : 4096);
}
void enc_exscan(const long long* in, long long n, long long* out, long long* sums, long long* total, hipStream_t s) {
  const int nb = (int)((n + SCAN_B - 1) / SCAN_B);
  if (n <= 0) { hipMemsetAsync(total, 0, 8, s); return; }
  hipLaunchKernelGGL(k_scan_sums, dim3(nb), dim3(ENT), 0, s, in, n, sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(64), 0, s, sums, nb, total);
  hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(ENT), 0, s, in, n, sums, out);
}
long long enc_scan_blocks(long long n) { return (n + SCAN_B - 1) / SCAN_B + 1; }
void enc_sel_rows(const uint8_t* sel, long long n, long long* tmp_i64, long long* pos, long long* sums, long long* total,
                  int32_t* rows, hipStream_t s) {
  if (n <= 0) { hipMemsetAsync(total, 0, 8, s); return; }
  hipLaunchKernelGGL(k_enc_u8_to_i64, dim3(enc_grid(n)), dim3(ENT), 0, s, sel, n, tmp_i64);
  enc_exscan(tmp_i64, n, pos, sums, total, s);
  hipLaunchKernelGGL(k_enc_sel_rows, dim3(enc_grid(n)), dim3(ENT), 0, s, sel, pos, n, rows);
}
void enc_count(const EncSrc& S, const int32_t* rows, long long n, long long* nlev, long long* nval, long long* nchr,
               int* err, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_enc_count, dim3(enc_grid(n)), dim3(ENT), 0, s, S, rows, n, nlev, nval, nchr, err);
}
void enc_fill(const EncSrc& S, const int32_t* rows, long long n, const long long* lb, const long long* vb,
              const long long* cb, uint8_t* def, uint8_t* rep, uint8_t* vals, int32_t* lens, uint8_t* chars,
              long long* coff, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_enc_fill, dim3(enc_grid(n)), dim3(ENT), 0, s, S, rows, n, lb, vb, cb, def, rep, vals, lens, chars,
                       coff);
}
void enc_bitpack(const uint8_t* lv, long long n, int bw, uint8_t* out, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_enc_bitpack, dim3(enc_grid((n + 7) / 8)), dim3(ENT), 0, s, lv, n, bw, out);
}
void enc_plain_str(const int32_t* lens, const long long* coff, const uint8_t* chars, long long v0, long long nv,
                   long long c0, uint8_t* out, hipStream_t s) {
  if (nv > 0) hipLaunchKernelGGL(k_enc_plain_str, dim3(enc_grid(nv)), dim3(ENT), 0, s, lens, coff, chars, v0, nv, c0, out);
}
void enc_snappy(const uint8_t* src, const SzBlock* blocks, int nb, long long cap, uint8_t* out, int32_t* lens,
                hipStream_t s) {
  if (nb > 0) hipLaunchKernelGGL(k_snappy_compress, dim3(nb), dim3(64), 0, s, src, blocks, cap, out, lens);
}

}  // namespace dk
