// Thrift compact-protocol reader shared by host (footer / offset index) and device (page headers).
// Parquet's footer and page headers are Thrift-compact structs (parquet-format, as read by
// parquet-mr 1.12.3 under kernel-defaults' ParquetFileReader.java:54-147).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DK_HD __host__ __device__ __forceinline__
#else
#define DK_HD inline
#endif

namespace dk {

struct TReader {
  const uint8_t* p;
  const uint8_t* e;
  int bad;

  DK_HD uint8_t byte() {
    if (p >= e) { bad = 1; return 0; }
    return *p++;
  }
  DK_HD uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) { bad = 1; return 0; }
      uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    bad = 1;
    return 0;
  }
  DK_HD int64_t zigzag() {
    uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  // Returns field id (0 = STOP); *type gets the compact type nibble.
  DK_HD int field(int* last, int* type) {
    uint8_t h = byte();
    if (bad || h == 0) return 0;
    int d = h >> 4;
    int id = d ? *last + d : (int)zigzag();
    *last = id;
    *type = h & 15;
    return id;
  }
  DK_HD int list_header(int* etype) {
    uint8_t h = byte();
    uint64_t n = h >> 4;
    *etype = h & 15;
    if (n == 15) n = varint();
    return (int)n;
  }
  // Skip without recursion (device-friendly): explicit stack of pending containers.
  DK_HD void skip(int type) {
    // stack entries: kind (0 struct, 1 list-elements remaining, 2 map pairs remaining), counts
    int kind[16];
    int64_t rem[16];
    int et[16], vt[16], half[16];
    int sp = -1;
    int t = type;
    for (;;) {
      if (bad) return;
      switch (t) {
        case 1: case 2: break;
        case 3: byte(); break;
        case 4: case 5: case 6: varint(); break;
        case 7: if (e - p < 8) bad = 1; else p += 8; break;
        // bound-check before advancing: a huge length must not wrap the pointer past the check
        case 8: { uint64_t n = varint(); if (bad || n > (uint64_t)(e - p)) bad = 1; else p += n; break; }
        case 9: case 10: {
          int etp; int n = list_header(&etp);
          if (sp + 1 >= 16) { bad = 1; return; }
          ++sp; kind[sp] = 1; rem[sp] = n; et[sp] = etp;
          break;
        }
        case 11: {
          uint64_t n = varint();
          int kvt = n ? byte() : 0;
          if (sp + 1 >= 16) { bad = 1; return; }
          ++sp; kind[sp] = 2; rem[sp] = (int64_t)n; et[sp] = kvt >> 4; vt[sp] = kvt & 15; half[sp] = 0;
          break;
        }
        case 12: {
          if (sp + 1 >= 16) { bad = 1; return; }
          ++sp; kind[sp] = 0; rem[sp] = 0;
          break;
        }
        default: bad = 1; return;
      }
      // find next item to skip
      for (;;) {
        if (sp < 0) return;
        if (kind[sp] == 0) {
          uint8_t h = byte();
          if (bad) return;
          if (h == 0) { --sp; continue; }
          if ((h >> 4) == 0) zigzag();
          t = h & 15;
          break;
        } else if (kind[sp] == 1) {
          if (rem[sp] == 0) { --sp; continue; }
          rem[sp]--;
          t = et[sp];
          if (t == 1 || t == 2) { byte(); continue; }   // bools in containers are one byte
          break;
        } else {
          if (rem[sp] == 0 && half[sp] == 0) { --sp; continue; }
          if (half[sp] == 0) { t = et[sp]; half[sp] = 1; }
          else { t = vt[sp]; half[sp] = 0; rem[sp]--; }
          if (t == 1 || t == 2) { byte(); continue; }
          break;
        }
      }
    }
  }
};

// Parquet enums (parquet-format)
enum PageType { PAGE_DATA = 0, PAGE_INDEX = 1, PAGE_DICT = 2, PAGE_DATA_V2 = 3 };
enum Encoding { ENC_PLAIN = 0, ENC_PLAIN_DICT = 2, ENC_RLE = 3, ENC_BIT_PACKED = 4, ENC_DELTA_BP = 5,
                ENC_DELTA_LBA = 6, ENC_DELTA_BA = 7, ENC_RLE_DICT = 8 };
enum Phys { PT_BOOLEAN = 0, PT_INT32 = 1, PT_INT64 = 2, PT_INT96 = 3, PT_FLOAT = 4, PT_DOUBLE = 5,
            PT_BYTE_ARRAY = 6, PT_FIXED = 7 };
enum Codec { CODEC_NONE = 0, CODEC_SNAPPY = 1 };

struct PageHeader {
  int32_t type, usize, csize, num_values, enc, dl_enc, rl_enc, dl_len, rl_len, is_comp, hdr_len, ok;
};

// Parse one PageHeader starting at p (end bound e).
DK_HD PageHeader parse_page_header(const uint8_t* p, const uint8_t* e) {
  PageHeader h;
  h.type = -1; h.usize = h.csize = h.num_values = h.enc = 0; h.dl_enc = h.rl_enc = 3;
  h.dl_len = h.rl_len = 0; h.is_comp = 1; h.hdr_len = 0; h.ok = 0;
  TReader t{p, e, 0};
  int last = 0, ty, id;
  while ((id = t.field(&last, &ty))) {
    if (id == 1) h.type = (int32_t)t.zigzag();
    else if (id == 2) h.usize = (int32_t)t.zigzag();
    else if (id == 3) h.csize = (int32_t)t.zigzag();
    else if ((id == 5 || id == 7 || id == 8) && ty == 12) {
      int l2 = 0, t2, i2;
      while ((i2 = t.field(&l2, &t2))) {
        if (id == 5) {          // DataPageHeader
          if (i2 == 1) h.num_values = (int32_t)t.zigzag();
          else if (i2 == 2) h.enc = (int32_t)t.zigzag();
          else if (i2 == 3) h.dl_enc = (int32_t)t.zigzag();
          else if (i2 == 4) h.rl_enc = (int32_t)t.zigzag();
          else t.skip(t2);
        } else if (id == 7) {   // DictionaryPageHeader
          if (i2 == 1) h.num_values = (int32_t)t.zigzag();
          else if (i2 == 2) h.enc = (int32_t)t.zigzag();
          else t.skip(t2);
        } else {                // DataPageHeaderV2
          if (i2 == 1) h.num_values = (int32_t)t.zigzag();
          else if (i2 == 4) h.enc = (int32_t)t.zigzag();
          else if (i2 == 5) h.dl_len = (int32_t)t.zigzag();
          else if (i2 == 6) h.rl_len = (int32_t)t.zigzag();
          else if (i2 == 7) h.is_comp = (t2 == 1);
          else t.skip(t2);
        }
        if (t.bad) return h;
      }
    } else t.skip(ty);
    if (t.bad) return h;
  }
  if (t.bad) return h;
  h.hdr_len = (int32_t)(t.p - p);
  h.ok = 1;
  return h;
}

#ifdef DK_DEVICE_TYPES
// A page header into its DPage, with the checks k_page_headers and the host open share: the parse
// is bounded by 64 KiB and by `end` (large min / max statistics are skipped).
DK_HD void apply_page_header(DPage& pg, const DChunk& ck, const uint8_t* base, const uint8_t* end) {
  const uint8_t* p = base + pg.hdr_off;
  const uint8_t* e = (end && end - p < 65536) ? end : p + 65536;
  PageHeader h = parse_page_header(p, e);
  pg.status = PS_OK;
  if (!h.ok) pg.status = PS_BAD_HEADER;
  pg.ptype = h.type; pg.enc = h.enc; pg.num_values = h.num_values; pg.dl_len = h.dl_len; pg.rl_len = h.rl_len;
  pg.csize = h.csize; pg.usize = h.usize; pg.hdr_len = h.hdr_len; pg.is_comp = h.is_comp;
  pg.data_off = pg.hdr_off + h.hdr_len;
  if (h.ok) {
    bool dict = (pg.flags & PF_DICT) != 0;
    if (dict != (h.type == PAGE_DICT)) pg.status = PS_BAD_HEADER;
    if (!dict && h.type != PAGE_DATA && h.type != PAGE_DATA_V2) pg.status = PS_UNSUPPORTED;
    if (h.type == PAGE_DATA && ((ck.max_def > 0 && h.dl_enc != ENC_RLE) || (ck.max_rep > 0 && h.rl_enc != ENC_RLE)))
      pg.status = PS_UNSUPPORTED;
    if (ck.codec != CODEC_NONE && pg.unc_off < 0 && !(h.type == PAGE_DATA_V2 && !h.is_comp)) pg.status = PS_UNSUPPORTED;
  }
}
#endif

}  // namespace dk
