/*
 * dk_ref — CPU ORACLE for the Delta Kernel snapshot-reconstruction hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / CPU baseline. The product (delta_amd,
 * libdkgpu.so) never links, loads or calls it.
 *
 * Plain scalar C restatement of:
 *  - Parquet decode as performed by parquet-mr 1.12.3 (third-party, absent from /root/reference;
 *    `build.sbt:662`) under kernel-defaults' converters: footer (Thrift compact), page headers,
 *    data page v1/v2, RLE/bit-packed hybrid levels, PLAIN / PLAIN_DICTIONARY / RLE_DICTIONARY /
 *    DELTA_BINARY_PACKED / RLE(boolean), SNAPPY and UNCOMPRESSED codecs. Record assembly follows
 *    kernel/kernel-defaults/src/main/java/io/delta/kernel/defaults/internal/parquet/
 *    RowColumnReader.java:106-131 (struct null iff start() not called, i.e. def < struct level),
 *    RepeatedValueConverter.java:65-81 (map offsets, null vs empty map) and
 *    ParquetColumnReaders.java:155-478 (leaf value / null handling).
 *  - java.net.URI parsing and URI.equals (JDK; call site
 *    kernel/kernel-api/src/main/java/io/delta/kernel/internal/replay/LogReplayUtils.java:83-89),
 *    restated from the JDK's published Parser grammar (RFC 2396 + RFC 2732 deviations).
 *  - Java's UTF-8 decoding with malformed-input replacement (DefaultBinaryVector.getString,
 *    kernel-defaults/.../internal/data/vector/DefaultBinaryVector.java:66-77).
 *  - DeletionVectorDescriptor.getUniqueId (kernel-api/.../internal/actions/
 *    DeletionVectorDescriptor.java:167-174): storageType + pathOrInlineDv + "@Optional[off]".
 *  - The checkpoint-batch half of ActiveAddFilesIterator.prepareNext
 *    (kernel-api/.../internal/replay/ActiveAddFilesIterator.java:192-234): membership probe
 *    against the JSON-derived add / tombstone sets plus ScanMetrics counters.
 *
 * Parity pinning: see tests/test_oracle_golden.py (golden tables of the reference, their known
 * answers from KDT/LogReplaySuite.scala etc.) and tests/test_oracle_vs_pyarrow.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

static __thread char g_err[512];
static void seterr(const char* m) { snprintf(g_err, sizeof g_err, "%s", m); }
EXPORT const char* dkr_errmsg(void) { return g_err; }

/* ------------------------------------------------------------------------------------------ */
/* Thrift compact protocol reader                                                             */
/* ------------------------------------------------------------------------------------------ */
typedef struct { const uint8_t* p; const uint8_t* e; int bad; } TR;

static uint64_t tr_varint(TR* t) {
  uint64_t v = 0; int s = 0;
  while (t->p < t->e) {
    uint8_t b = *t->p++;
    v |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return v;
    s += 7;
    if (s > 63) break;
  }
  t->bad = 1; return 0;
}
static int64_t tr_zz(TR* t) { uint64_t v = tr_varint(t); return (int64_t)(v >> 1) ^ -(int64_t)(v & 1); }
static void tr_skip(TR* t, int type);
static void tr_skip_struct(TR* t) {
  for (;;) {
    if (t->p >= t->e) { t->bad = 1; return; }
    uint8_t h = *t->p++;
    if (h == 0) return;
    if ((h >> 4) == 0) tr_zz(t);
    tr_skip(t, h & 15);
    if (t->bad) return;
  }
}
static void tr_skip(TR* t, int type) {
  switch (type) {
    case 1: case 2: return;                          /* bool in field header */
    case 3: t->p++; return;
    case 4: case 5: case 6: tr_varint(t); return;
    case 7: t->p += 8; return;
    case 8: { uint64_t n = tr_varint(t); t->p += n; return; }
    case 9: case 10: {
      if (t->p >= t->e) { t->bad = 1; return; }
      uint8_t h = *t->p++; uint64_t n = h >> 4; int et = h & 15;
      if (n == 15) n = tr_varint(t);
      for (uint64_t i = 0; i < n && !t->bad; i++) { if (et == 1 || et == 2) t->p++; else tr_skip(t, et); }
      return;
    }
    case 11: {
      uint64_t n = tr_varint(t);
      if (n == 0) return;
      uint8_t kv = *t->p++;
      for (uint64_t i = 0; i < n && !t->bad; i++) { tr_skip(t, kv >> 4); tr_skip(t, kv & 15); }
      return;
    }
    case 12: tr_skip_struct(t); return;
    default: t->bad = 1;
  }
}
/* iterate fields: returns field id, sets *type; 0 on stop */
static int tr_field(TR* t, int* last, int* type) {
  if (t->p >= t->e) { t->bad = 1; return 0; }
  uint8_t h = *t->p++;
  if (h == 0) return 0;
  int d = h >> 4;
  int id = d ? *last + d : (int)tr_zz(t);
  *last = id; *type = h & 15;
  return id;
}
static int tr_list_hdr(TR* t, int* et) {
  uint8_t h = *t->p++; uint64_t n = h >> 4; *et = h & 15;
  if (n == 15) n = tr_varint(t);
  return (int)n;
}

/* ------------------------------------------------------------------------------------------ */
/* Parquet metadata model                                                                     */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int type, type_length, repetition, num_children, field_id, has_field_id;
  char name[256];
} SchemaEl;

typedef struct {
  int type, codec;
  int64_t num_values, data_page_offset, dict_page_offset, total_compressed;
  int has_dict;
} ChunkMeta;

typedef struct {
  char path[1024];     /* dotted */
  int phys, type_length, max_def, max_rep, rep_def; /* rep_def: def level at the repeated node */
  int schema_idx;
} Leaf;

typedef struct {
  const uint8_t* buf; int64_t len;
  int64_t num_rows;
  int n_schema; SchemaEl* schema;
  int n_rg; int64_t* rg_rows;
  int n_leaves; Leaf* leaves;
  ChunkMeta* chunks; /* n_rg * n_leaves */
  uint8_t* keep;     /* row groups to read (NULL: all) -- the ParquetHandler's row-group filter */
} PFile;

static void parse_schema_el(TR* t, SchemaEl* s) {
  memset(s, 0, sizeof *s); s->type = -1; s->repetition = 0;
  int last = 0, ty;
  int id;
  while ((id = tr_field(t, &last, &ty))) {
    switch (id) {
      case 1: s->type = (int)tr_zz(t); break;
      case 2: s->type_length = (int)tr_zz(t); break;
      case 3: s->repetition = (int)tr_zz(t); break;
      case 4: { uint64_t n = tr_varint(t); size_t c = n < 255 ? n : 255; memcpy(s->name, t->p, c); s->name[c] = 0; t->p += n; break; }
      case 5: s->num_children = (int)tr_zz(t); break;
      case 9: s->field_id = (int)tr_zz(t); s->has_field_id = 1; break;
      default: tr_skip(t, ty);
    }
    if (t->bad) return;
  }
}

static void parse_col_meta(TR* t, ChunkMeta* m) {
  int last = 0, ty, id;
  while ((id = tr_field(t, &last, &ty))) {
    switch (id) {
      case 1: m->type = (int)tr_zz(t); break;
      case 4: m->codec = (int)tr_zz(t); break;
      case 5: m->num_values = tr_zz(t); break;
      case 7: m->total_compressed = tr_zz(t); break;
      case 9: m->data_page_offset = tr_zz(t); break;
      case 11: m->dict_page_offset = tr_zz(t); m->has_dict = 1; break;
      default: tr_skip(t, ty);
    }
    if (t->bad) return;
  }
}

/* build leaves by DFS over the flattened schema list */
typedef struct { int idx; int def; int rep; int rep_def; char path[1024]; } Frame;
static int build_leaves(PFile* f) {
  f->leaves = calloc(f->n_schema, sizeof(Leaf));
  f->n_leaves = 0;
  /* recursive descent using explicit index */
  int pos = 1;
  /* stack of (remaining children, def, rep, rep_def, path) */
  struct { int remaining; int def, rep, rep_def; char path[1024]; } st[64];
  int sp = 0;
  st[0].remaining = f->schema[0].num_children; st[0].def = 0; st[0].rep = 0; st[0].rep_def = 0; st[0].path[0] = 0;
  while (sp >= 0) {
    if (st[sp].remaining == 0) { sp--; continue; }
    st[sp].remaining--;
    if (pos >= f->n_schema) return -1;
    SchemaEl* e = &f->schema[pos];
    int def = st[sp].def + (e->repetition != 0 ? 1 : 0);
    int rep = st[sp].rep + (e->repetition == 2 ? 1 : 0);
    int rep_def = e->repetition == 2 ? def : st[sp].rep_def;
    char path[1024];
    if (st[sp].path[0]) snprintf(path, sizeof path, "%s.%s", st[sp].path, e->name);
    else snprintf(path, sizeof path, "%s", e->name);
    if (e->num_children > 0) {
      if (sp + 1 >= 64) return -1;
      sp++;
      st[sp].remaining = e->num_children; st[sp].def = def; st[sp].rep = rep; st[sp].rep_def = rep_def;
      snprintf(st[sp].path, sizeof st[sp].path, "%s", path);
    } else {
      Leaf* l = &f->leaves[f->n_leaves++];
      snprintf(l->path, sizeof l->path, "%s", path);
      l->phys = e->type; l->type_length = e->type_length; l->max_def = def; l->max_rep = rep; l->rep_def = rep_def;
      l->schema_idx = pos;
    }
    pos++;
  }
  return 0;
}

EXPORT void dkr_close(void* h) {
  PFile* f = (PFile*)h;
  if (!f) return;
  free(f->schema); free(f->rg_rows); free(f->leaves); free(f->chunks); free(f->keep); free(f);
}

EXPORT void* dkr_open(const uint8_t* buf, int64_t len) {
  if (len < 12 || memcmp(buf, "PAR1", 4) || memcmp(buf + len - 4, "PAR1", 4)) { seterr("not a parquet file"); return NULL; }
  uint32_t flen; memcpy(&flen, buf + len - 8, 4);
  if ((int64_t)flen > len - 12) { seterr("bad footer length"); return NULL; }
  TR t = { buf + len - 8 - flen, buf + len - 8, 0 };
  PFile* f = calloc(1, sizeof(PFile));
  f->buf = buf; f->len = len;
  int last = 0, ty, id;
  /* first pass: schema + num_rows; row groups parsed after leaves are known */
  const uint8_t* rg_start = NULL; int rg_n = 0;
  while ((id = tr_field(&t, &last, &ty))) {
    if (id == 2 && ty == 9) {
      int et; int n = tr_list_hdr(&t, &et);
      f->n_schema = n; f->schema = calloc(n, sizeof(SchemaEl));
      for (int i = 0; i < n; i++) parse_schema_el(&t, &f->schema[i]);
    } else if (id == 3) {
      f->num_rows = tr_zz(&t);
    } else if (id == 4 && ty == 9) {
      rg_start = t.p;
      int et; rg_n = tr_list_hdr(&t, &et);
      for (int i = 0; i < rg_n; i++) tr_skip_struct(&t);
    } else tr_skip(&t, ty);
    if (t.bad) { seterr("corrupt footer"); dkr_close(f); return NULL; }
  }
  if (!f->schema || build_leaves(f)) { seterr("bad schema"); dkr_close(f); return NULL; }
  f->n_rg = rg_n;
  f->rg_rows = calloc(rg_n ? rg_n : 1, sizeof(int64_t));
  f->chunks = calloc((size_t)(rg_n ? rg_n : 1) * (f->n_leaves ? f->n_leaves : 1), sizeof(ChunkMeta));
  if (rg_start) {
    TR r = { rg_start, buf + len - 8, 0 };
    int et; tr_list_hdr(&r, &et);
    for (int g = 0; g < rg_n; g++) {
      int l2 = 0, t2, i2;
      while ((i2 = tr_field(&r, &l2, &t2))) {
        if (i2 == 1 && t2 == 9) {
          int et2; int nc = tr_list_hdr(&r, &et2);
          for (int c = 0; c < nc; c++) {
            ChunkMeta* m = &f->chunks[(size_t)g * f->n_leaves + c];
            int l3 = 0, t3, i3;
            while ((i3 = tr_field(&r, &l3, &t3))) {
              if (i3 == 3 && t3 == 12) parse_col_meta(&r, m);
              else tr_skip(&r, t3);
              if (r.bad) break;
            }
          }
        } else if (i2 == 3) {
          f->rg_rows[g] = tr_zz(&r);
        } else tr_skip(&r, t2);
        if (r.bad) { seterr("corrupt row group"); dkr_close(f); return NULL; }
      }
    }
  }
  return f;
}

EXPORT int64_t dkr_num_rows(void* h) { return ((PFile*)h)->num_rows; }
/* Read only the row groups with keep[g] != 0 from here on (num_rows becomes their row count). */
EXPORT void dkr_select_row_groups(void* h, const uint8_t* keep) {
  PFile* f = (PFile*)h;
  free(f->keep);
  f->keep = malloc(f->n_rg ? f->n_rg : 1);
  f->num_rows = 0;
  for (int g = 0; g < f->n_rg; g++) { f->keep[g] = keep[g] != 0; if (f->keep[g]) f->num_rows += f->rg_rows[g]; }
}
EXPORT int dkr_num_leaves(void* h) { return ((PFile*)h)->n_leaves; }
EXPORT int dkr_num_row_groups(void* h) { return ((PFile*)h)->n_rg; }
EXPORT const char* dkr_leaf_path(void* h, int i) { return ((PFile*)h)->leaves[i].path; }
EXPORT void dkr_leaf_info(void* h, int i, int* out5) {
  Leaf* l = &((PFile*)h)->leaves[i];
  out5[0] = l->phys; out5[1] = l->max_def; out5[2] = l->max_rep; out5[3] = l->rep_def; out5[4] = l->type_length;
}
EXPORT void dkr_chunk_info(void* h, int rg, int leaf, int64_t* out6) {
  PFile* f = (PFile*)h;
  ChunkMeta* m = &f->chunks[(size_t)rg * f->n_leaves + leaf];
  out6[0] = m->codec; out6[1] = m->num_values; out6[2] = m->has_dict ? m->dict_page_offset : -1;
  out6[3] = m->data_page_offset; out6[4] = m->total_compressed; out6[5] = f->rg_rows[rg];
}

/* ------------------------------------------------------------------------------------------ */
/* Snappy raw block decompression (published format: varint length, literal / copy tags)      */
/* ------------------------------------------------------------------------------------------ */
static int snappy_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  const uint8_t* p = in; const uint8_t* e = in + n;
  uint64_t ulen = 0; int s = 0;
  while (p < e) { uint8_t b = *p++; ulen |= (uint64_t)(b & 0x7f) << s; if (!(b & 0x80)) break; s += 7; }
  if ((int64_t)ulen != cap) return -1;
  int64_t o = 0;
  while (p < e) {
    uint8_t tag = *p++;
    int kind = tag & 3;
    if (kind == 0) {
      int64_t len = (tag >> 2) + 1;
      if (len > 60) {
        int nb = (int)len - 60; len = 0;
        for (int i = 0; i < nb; i++) len |= (int64_t)p[i] << (8 * i);
        len += 1; p += nb;
      }
      if (p + len > e || o + len > cap) return -1;
      memcpy(out + o, p, len); p += len; o += len;
    } else {
      int64_t len, off;
      if (kind == 1) { len = ((tag >> 2) & 7) + 4; off = ((int64_t)(tag >> 5) << 8) | *p++; }
      else if (kind == 2) { len = (tag >> 2) + 1; off = p[0] | (p[1] << 8); p += 2; }
      else { len = (tag >> 2) + 1; off = (int64_t)p[0] | ((int64_t)p[1] << 8) | ((int64_t)p[2] << 16) | ((int64_t)p[3] << 24); p += 4; }
      if (off == 0 || off > o || o + len > cap) return -1;
      for (int64_t i = 0; i < len; i++) out[o + i] = out[o - off + i];
      o += len;
    }
  }
  return o == cap ? 0 : -1;
}

/* ------------------------------------------------------------------------------------------ */
/* RLE / bit-packed hybrid                                                                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct { const uint8_t* p; const uint8_t* e; int bw; int64_t rle_left; uint32_t rle_val; int64_t bp_left; int64_t bp_bitpos; const uint8_t* bp; } Hyb;
static void hyb_init(Hyb* h, const uint8_t* p, const uint8_t* e, int bw) { memset(h, 0, sizeof *h); h->p = p; h->e = e; h->bw = bw; }
static int hyb_next(Hyb* h, uint32_t* out) {
  while (h->rle_left == 0 && h->bp_left == 0) {
    if (h->p >= h->e) return -1;
    TR t = { h->p, h->e, 0 };
    uint64_t hdr = tr_varint(&t);
    if (t.bad) return -1;
    h->p = t.p;
    if (hdr & 1) {
      int64_t groups = (int64_t)(hdr >> 1);
      h->bp_left = groups * 8; h->bp = h->p; h->bp_bitpos = 0;
      int64_t bytes = groups * h->bw;
      if (h->p + bytes > h->e) { /* truncated final run: allow, values past end read as 0 */ bytes = h->e - h->p; }
      h->p += bytes;
    } else {
      h->rle_left = (int64_t)(hdr >> 1);
      int nb = (h->bw + 7) / 8; uint32_t v = 0;
      for (int i = 0; i < nb; i++) { if (h->p >= h->e) return -1; v |= (uint32_t)(*h->p++) << (8 * i); }
      h->rle_val = v;
    }
  }
  if (h->rle_left) { h->rle_left--; *out = h->rle_val; return 0; }
  uint32_t v = 0;
  for (int i = 0; i < h->bw; i++) {
    int64_t bit = h->bp_bitpos + i;
    const uint8_t* b = h->bp + (bit >> 3);
    if (b < h->e && ((*b >> (bit & 7)) & 1)) v |= 1u << i;
  }
  h->bp_bitpos += h->bw; h->bp_left--;
  *out = v; return 0;
}
static int bitwidth(int maxv) { int w = 0; while ((1 << w) <= maxv) w++; return maxv == 0 ? 0 : w; }

/* ------------------------------------------------------------------------------------------ */
/* Column decode: level-major buffers                                                         */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint8_t* p; int64_t n, cap; } Buf;
static void buf_put(Buf* b, const void* src, int64_t n) {
  if (b->n + n > b->cap) { int64_t c = b->cap ? b->cap : 1024; while (c < b->n + n) c *= 2; b->p = realloc(b->p, c); b->cap = c; }
  if (n) memcpy(b->p + b->n, src, n);
  b->n += n;
}

typedef struct {
  Buf def, rep;        /* u8 per level */
  Buf fixed;           /* values for non-null levels, width w (bool as u8) */
  Buf offs;            /* int64 per non-null value (start offsets into chars) */
  Buf chars;
  int64_t n_levels, n_values;
} Raw;

typedef struct { int64_t n; int64_t* offs; uint8_t* chars; int64_t nchars; uint8_t* fixed; int w; } Dict;

static int phys_width(int phys, int tl) {
  switch (phys) { case 0: return 1; case 1: return 4; case 2: return 8; case 3: return 12; case 4: return 4; case 5: return 8; case 7: return tl; default: return 0; }
}

static int decode_plain(int phys, int tl, const uint8_t* p, const uint8_t* e, int64_t nv, Raw* r, int64_t* bool_bit) {
  int w = phys_width(phys, tl);
  if (phys == 0) {
    for (int64_t i = 0; i < nv; i++) {
      int64_t bit = *bool_bit + i;
      if (p + (bit >> 3) >= e) return -1;
      uint8_t v = (p[bit >> 3] >> (bit & 7)) & 1;
      buf_put(&r->fixed, &v, 1);
    }
    return 0;
  }
  if (phys == 6) {
    for (int64_t i = 0; i < nv; i++) {
      if (p + 4 > e) return -1;
      uint32_t L; memcpy(&L, p, 4); p += 4;
      if (p + L > e) return -1;
      int64_t o = r->chars.n; buf_put(&r->offs, &o, 8); buf_put(&r->chars, p, L); p += L;
    }
    return 0;
  }
  if (p + nv * w > e) return -1;
  buf_put(&r->fixed, p, nv * w);
  return 0;
}

static int decode_dict_page(int phys, int tl, const uint8_t* p, const uint8_t* e, int64_t nv, Dict* d) {
  Raw r; memset(&r, 0, sizeof r);
  int64_t bb = 0;
  if (decode_plain(phys, tl, p, e, nv, &r, &bb)) return -1;
  d->n = nv; d->w = phys_width(phys, tl);
  if (phys == 6) {
    d->offs = malloc((nv + 1) * 8);
    memcpy(d->offs, r.offs.p, nv * 8); d->offs[nv] = r.chars.n;
    d->chars = r.chars.p; d->nchars = r.chars.n; free(r.offs.p);
  } else { d->fixed = r.fixed.p; }
  return 0;
}

static int decode_delta_binary_packed(const uint8_t* p, const uint8_t* e, int64_t nv, int w, Raw* r) {
  TR t = { p, e, 0 };
  uint64_t block = tr_varint(&t), nmini = tr_varint(&t), total = tr_varint(&t);
  int64_t first = tr_zz(&t);
  if (t.bad || nmini == 0 || block % nmini || (block / nmini) % 32) return -1;
  int64_t per_mini = block / nmini;
  int64_t cur = first; int64_t got = 0;
  if ((int64_t)total < nv) return -1;
#define EMIT(v) do { if (w == 4) { int32_t x = (int32_t)(v); buf_put(&r->fixed, &x, 4); } else { int64_t x = (v); buf_put(&r->fixed, &x, 8); } got++; } while (0)
  if (nv > 0) EMIT(cur);
  while (got < nv) {
    int64_t mind = tr_zz(&t);
    if (t.bad || t.p + nmini > t.e) return -1;
    const uint8_t* bws = t.p; t.p += nmini;
    for (uint64_t m = 0; m < nmini && got < nv; m++) {
      int bw = bws[m];
      const uint8_t* mp = t.p;
      for (int64_t i = 0; i < per_mini && got < nv; i++) {
        uint64_t v = 0;
        for (int b = 0; b < bw; b++) { int64_t bit = i * bw + b; if (mp + (bit >> 3) < e && ((mp[bit >> 3] >> (bit & 7)) & 1)) v |= 1ull << b; }
        cur = (int64_t)((uint64_t)cur + (uint64_t)mind + v);
        if (w == 4) cur = (int32_t)cur;
        EMIT(cur);
      }
      t.p += per_mini * bw / 8;
    }
  }
#undef EMIT
  return 0;
}

static int decode_chunk(PFile* f, int leaf, int rg, Raw* r) {
  Leaf* L = &f->leaves[leaf];
  ChunkMeta* m = &f->chunks[(size_t)rg * f->n_leaves + leaf];
  int64_t start = m->has_dict && m->dict_page_offset > 0 && m->dict_page_offset < m->data_page_offset ? m->dict_page_offset : m->data_page_offset;
  const uint8_t* p = f->buf + start;
  const uint8_t* end = f->buf + start + m->total_compressed;
  if (end > f->buf + f->len) { seterr("chunk out of range"); return -1; }
  Dict dict; memset(&dict, 0, sizeof dict); int have_dict = 0;
  int64_t levels_seen = 0;
  int dbw = bitwidth(L->max_def), rbw = bitwidth(L->max_rep);
  int w = phys_width(L->phys, L->type_length);
  while (p < end && levels_seen < m->num_values) {
    TR t = { p, end, 0 };
    int ptype = -1, usize = 0, csize = 0, last = 0, ty, id;
    int64_t nv = 0, nrows = 0; int enc = 0, dl_enc = 3, rl_enc = 3; int dl_len = 0, rl_len = 0, is_comp = 1;
    int64_t dict_nv = 0;
    while ((id = tr_field(&t, &last, &ty))) {
      if (id == 1) ptype = (int)tr_zz(&t);
      else if (id == 2) usize = (int)tr_zz(&t);
      else if (id == 3) csize = (int)tr_zz(&t);
      else if (id == 5 && ty == 12) {
        int l2 = 0, t2, i2;
        while ((i2 = tr_field(&t, &l2, &t2))) {
          if (i2 == 1) nv = tr_zz(&t); else if (i2 == 2) enc = (int)tr_zz(&t);
          else if (i2 == 3) dl_enc = (int)tr_zz(&t); else if (i2 == 4) rl_enc = (int)tr_zz(&t);
          else tr_skip(&t, t2);
        }
      } else if (id == 7 && ty == 12) {
        int l2 = 0, t2, i2;
        while ((i2 = tr_field(&t, &l2, &t2))) { if (i2 == 1) dict_nv = tr_zz(&t); else if (i2 == 2) enc = (int)tr_zz(&t); else tr_skip(&t, t2); }
      } else if (id == 8 && ty == 12) {
        int l2 = 0, t2, i2;
        while ((i2 = tr_field(&t, &l2, &t2))) {
          if (i2 == 1) nv = tr_zz(&t); else if (i2 == 3) nrows = tr_zz(&t); else if (i2 == 4) enc = (int)tr_zz(&t);
          else if (i2 == 5) dl_len = (int)tr_zz(&t); else if (i2 == 6) rl_len = (int)tr_zz(&t);
          else if (i2 == 7) is_comp = (t2 == 1); else tr_skip(&t, t2);
        }
      } else tr_skip(&t, ty);
      if (t.bad) { seterr("corrupt page header"); return -1; }
    }
    (void)nrows;
    const uint8_t* body = t.p;
    if (body + csize > end) { seterr("page out of range"); return -1; }
    p = body + csize;
    if (ptype == 1) continue; /* index page */
    /* decompress */
    uint8_t* ubuf = NULL; const uint8_t* data; int64_t dlen;
    if (ptype == 3) {
      /* v2: levels are never compressed */
      int lv = rl_len + dl_len;
      ubuf = malloc(usize + 8);
      memcpy(ubuf, body, lv);
      if (m->codec == 0 || !is_comp) { memcpy(ubuf + lv, body + lv, csize - lv); }
      else if (m->codec == 1) { if (snappy_decompress(body + lv, csize - lv, ubuf + lv, usize - lv)) { free(ubuf); seterr("snappy error"); return -1; } }
      else { free(ubuf); seterr("unsupported codec"); return -1; }
      data = ubuf; dlen = usize;
    } else {
      if (m->codec == 0) { data = body; dlen = csize; }
      else if (m->codec == 1) {
        ubuf = malloc(usize + 8);
        if (snappy_decompress(body, csize, ubuf, usize)) { free(ubuf); seterr("snappy error"); return -1; }
        data = ubuf; dlen = usize;
      } else { seterr("unsupported codec"); return -1; }
    }
    if (ptype == 2) {
      if (decode_dict_page(L->phys, L->type_length, data, data + dlen, dict_nv, &dict)) { free(ubuf); seterr("bad dictionary page"); return -1; }
      have_dict = 1; free(ubuf); continue;
    }
    if (ptype != 0 && ptype != 3) { free(ubuf); seterr("unknown page type"); return -1; }
    const uint8_t* q = data; const uint8_t* qe = data + dlen;
    /* levels */
    uint8_t* reps = calloc(nv ? nv : 1, 1); uint8_t* defs = calloc(nv ? nv : 1, 1);
    if (ptype == 0) {
      if ((L->max_def > 0 && dl_enc != 3) || (L->max_rep > 0 && rl_enc != 3)) { seterr("unsupported level encoding"); return -1; }
      if (L->max_rep > 0) {
        uint32_t ln; memcpy(&ln, q, 4); q += 4;
        Hyb h; hyb_init(&h, q, q + ln, rbw);
        for (int64_t i = 0; i < nv; i++) { uint32_t v; if (hyb_next(&h, &v)) { seterr("bad rep levels"); return -1; } reps[i] = (uint8_t)v; }
        q += ln;
      }
      if (L->max_def > 0) {
        uint32_t ln; memcpy(&ln, q, 4); q += 4;
        Hyb h; hyb_init(&h, q, q + ln, dbw);
        for (int64_t i = 0; i < nv; i++) { uint32_t v; if (hyb_next(&h, &v)) { seterr("bad def levels"); return -1; } defs[i] = (uint8_t)v; }
        q += ln;
      }
    } else {
      if (L->max_rep > 0) { Hyb h; hyb_init(&h, q, q + rl_len, rbw); for (int64_t i = 0; i < nv; i++) { uint32_t v; if (hyb_next(&h, &v)) { seterr("bad rep levels"); return -1; } reps[i] = (uint8_t)v; } }
      q += rl_len;
      if (L->max_def > 0) { Hyb h; hyb_init(&h, q, q + dl_len, dbw); for (int64_t i = 0; i < nv; i++) { uint32_t v; if (hyb_next(&h, &v)) { seterr("bad def levels"); return -1; } defs[i] = (uint8_t)v; } }
      q += dl_len;
    }
    int64_t nn = 0;
    for (int64_t i = 0; i < nv; i++) if (defs[i] == L->max_def) nn++;
    buf_put(&r->def, defs, nv); buf_put(&r->rep, reps, nv);
    free(defs); free(reps);
    /* values */
    int rc = 0;
    if (enc == 0) {
      int64_t bb = 0; rc = decode_plain(L->phys, L->type_length, q, qe, nn, r, &bb);
    } else if (enc == 2 || enc == 8) {
      if (!have_dict) { seterr("dictionary page missing"); return -1; }
      int ibw = nn ? *q : 0; q++;
      Hyb h; hyb_init(&h, q, qe, ibw);
      for (int64_t i = 0; i < nn && !rc; i++) {
        uint32_t ix; if (hyb_next(&h, &ix) || ix >= dict.n) { rc = -1; break; }
        if (L->phys == 6) { int64_t o = r->chars.n; buf_put(&r->offs, &o, 8); buf_put(&r->chars, dict.chars + dict.offs[ix], dict.offs[ix + 1] - dict.offs[ix]); }
        else buf_put(&r->fixed, dict.fixed + (int64_t)ix * dict.w, dict.w);
      }
    } else if (enc == 5 && (L->phys == 1 || L->phys == 2)) {
      rc = decode_delta_binary_packed(q, qe, nn, w, r);
    } else if (enc == 3 && L->phys == 0) {
      uint32_t ln; memcpy(&ln, q, 4); q += 4;
      Hyb h; hyb_init(&h, q, q + ln, 1);
      for (int64_t i = 0; i < nn; i++) { uint32_t v; if (hyb_next(&h, &v)) { rc = -1; break; } uint8_t b = (uint8_t)v; buf_put(&r->fixed, &b, 1); }
    } else { seterr("unsupported encoding"); free(ubuf); return -1; }
    if (rc) { seterr("value decode error"); free(ubuf); return -1; }
    levels_seen += nv; r->n_levels += nv; r->n_values += nn;
    free(ubuf);
  }
  free(dict.offs); free(dict.chars); free(dict.fixed);
  return 0;
}

/* Assembled column (the layout the product also produces; see include/dkgpu.h dk_column).
 *   non-repeated leaf : row_def[n_rows]; fixed[n_rows*w] (0 where null) or offs[n_rows+1] + chars
 *   repeated leaf     : row_def[n_rows] (def of the row's first level), row_offs[n_rows+1] entry
 *                       offsets; entry_def[n_entries]; values entry-dense (fixed or offs+chars) */
typedef struct {
  int64_t n_rows, n_entries, n_chars;
  int32_t phys, width, max_def, max_rep, rep_def, _pad;
  uint8_t* row_def;
  int64_t* row_offs;
  uint8_t* entry_def;
  uint8_t* fixed;
  int64_t* offs;
  uint8_t* chars;
} dkr_col;

EXPORT void dkr_col_free(dkr_col* c) {
  free(c->row_def); free(c->row_offs); free(c->entry_def); free(c->fixed); free(c->offs); free(c->chars);
  memset(c, 0, sizeof *c);
}

EXPORT int dkr_read_leaf(void* h, int leaf, dkr_col* out) {
  PFile* f = (PFile*)h;
  memset(out, 0, sizeof *out);
  if (leaf < 0 || leaf >= f->n_leaves) { seterr("bad leaf"); return -1; }
  Leaf* L = &f->leaves[leaf];
  Raw r; memset(&r, 0, sizeof r);
  for (int g = 0; g < f->n_rg; g++) if ((!f->keep || f->keep[g]) && decode_chunk(f, leaf, g, &r)) return -1;
  int w = phys_width(L->phys, L->type_length);
  if (L->phys == 0) w = 1;
  out->phys = L->phys; out->width = L->phys == 6 ? 0 : w; out->max_def = L->max_def; out->max_rep = L->max_rep; out->rep_def = L->rep_def;
  int64_t nl = r.n_levels;
  const uint8_t* def = r.def.p; const uint8_t* rep = r.rep.p;
  if (L->max_rep == 0) {
    int64_t n = nl;
    out->n_rows = n; out->n_entries = n;
    out->row_def = malloc(n ? n : 1);
    if (n) memcpy(out->row_def, def, n);
    if (L->phys == 6) {
      out->offs = malloc((n + 1) * 8); out->chars = r.chars.p; out->n_chars = r.chars.n; r.chars.p = NULL;
      int64_t v = 0; const int64_t* vo = (const int64_t*)r.offs.p;
      for (int64_t i = 0; i < n; i++) {
        if (def[i] == L->max_def) { out->offs[i] = vo[v]; v++; }
        else out->offs[i] = v < r.n_values ? vo[v] : out->n_chars;
      }
      out->offs[n] = out->n_chars;
    } else {
      out->fixed = calloc(n ? n : 1, w);
      int64_t v = 0;
      for (int64_t i = 0; i < n; i++) if (def[i] == L->max_def) { memcpy(out->fixed + i * w, r.fixed.p + v * w, w); v++; }
    }
  } else {
    int64_t nrows = 0, nent = 0;
    for (int64_t i = 0; i < nl; i++) { if (rep[i] == 0) nrows++; if (def[i] >= L->rep_def) nent++; }
    out->n_rows = nrows; out->n_entries = nent;
    out->row_def = malloc(nrows ? nrows : 1);
    out->row_offs = malloc((nrows + 1) * 8);
    out->entry_def = malloc(nent ? nent : 1);
    int64_t row = -1, e = 0, v = 0;
    if (L->phys == 6) { out->offs = malloc((nent + 1) * 8); out->chars = r.chars.p; out->n_chars = r.chars.n; r.chars.p = NULL; }
    else out->fixed = calloc(nent ? nent : 1, w);
    const int64_t* vo = (const int64_t*)r.offs.p;
    for (int64_t i = 0; i < nl; i++) {
      if (rep[i] == 0) { row++; out->row_def[row] = def[i]; out->row_offs[row] = e; }
      if (def[i] >= L->rep_def) {
        out->entry_def[e] = def[i];
        if (def[i] == L->max_def) {
          if (L->phys == 6) out->offs[e] = vo[v]; else memcpy(out->fixed + e * w, r.fixed.p + v * w, w);
          v++;
        } else if (L->phys == 6) out->offs[e] = v < r.n_values ? vo[v] : out->n_chars;
        e++;
      }
    }
    out->row_offs[nrows] = e;
    if (L->phys == 6) out->offs[nent] = out->n_chars;
  }
  free(r.def.p); free(r.rep.p); free(r.fixed.p); free(r.offs.p); free(r.chars.p);
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Java UTF-8 decode with replacement (U+FFFD per maximal ill-formed subpart), re-encoded.    */
/* ------------------------------------------------------------------------------------------ */
EXPORT int64_t dkr_java_utf8(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
  int64_t o = 0, i = 0;
#define PUT(b) do { if (o >= cap) return -1; out[o++] = (uint8_t)(b); } while (0)
#define REPL() do { PUT(0xEF); PUT(0xBF); PUT(0xBD); } while (0)
  while (i < n) {
    uint8_t b = s[i];
    if (b < 0x80) { PUT(b); i++; continue; }
    int need; uint8_t lo = 0x80, hi = 0xBF;
    if (b >= 0xC2 && b <= 0xDF) need = 1;
    else if (b == 0xE0) { need = 2; lo = 0xA0; }
    else if (b >= 0xE1 && b <= 0xEC) need = 2;
    else if (b == 0xED) { need = 2; hi = 0x9F; }
    else if (b >= 0xEE && b <= 0xEF) need = 2;
    else if (b == 0xF0) { need = 3; lo = 0x90; }
    else if (b >= 0xF1 && b <= 0xF3) need = 3;
    else if (b == 0xF4) { need = 3; hi = 0x8F; }
    else { REPL(); i++; continue; }
    int64_t j = i + 1; int k;
    for (k = 0; k < need; k++, j++) {
      if (j >= n) break;
      uint8_t c = s[j];
      uint8_t l = k == 0 ? lo : 0x80, h2 = k == 0 ? hi : 0xBF;
      if (c < l || c > h2) break;
    }
    if (k == need) { for (int64_t x = i; x < j; x++) PUT(s[x]); i = j; }
    else { REPL(); i = j; }
  }
  return o;
#undef PUT
#undef REPL
}

/* ------------------------------------------------------------------------------------------ */
/* java.net.URI parse + canonical key (equal canonical keys <=> URI.equals)                   */
/* ------------------------------------------------------------------------------------------ */
/* char classes over ASCII, from RFC 2396 as used by java.net.URI */
enum { C_DIGIT = 1, C_ALPHA = 2, C_MARK = 4, C_RESERVED = 8, C_HEX = 16 };
static int cls(int c) {
  int r = 0;
  if (c >= '0' && c <= '9') r |= C_DIGIT | C_HEX;
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) r |= C_ALPHA;
  if ((c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F')) r |= C_HEX;
  if (c && strchr("-_.!~*'()", c)) r |= C_MARK;
  if (c && strchr(";/?:@&=+$,[]", c)) r |= C_RESERVED;
  return r;
}
static int is_unreserved(int c) { return (cls(c) & (C_DIGIT | C_ALPHA | C_MARK)) != 0; }
/* component classes (ASCII part) */
static int in_uric(int c) { return is_unreserved(c) || (cls(c) & C_RESERVED); }
static int in_path(int c) { return is_unreserved(c) || (c && strchr(":@&=+$,;/", c)); }
static int in_userinfo(int c) { return is_unreserved(c) || (c && strchr(";:&=+$,", c)); }
static int in_regname(int c) { return is_unreserved(c) || (c && strchr("$,;:@&=+", c)); }
static int in_server(int c) { return in_userinfo(c) || (cls(c) & (C_DIGIT | C_ALPHA)) || c == '-' || (c && strchr(".:@[]", c)); }
static int in_scheme(int c) { return (cls(c) & (C_DIGIT | C_ALPHA)) || c == '+' || c == '-' || c == '.'; }
static int in_scope(int c) { return (cls(c) & (C_DIGIT | C_ALPHA)) || c == '_' || c == '.'; }

typedef struct { const uint8_t* s; int64_t n; } US;

/* decode one UTF-8 code point at i (input already valid UTF-8) */
static uint32_t cp_at(US* u, int64_t i, int* len) {
  uint8_t b = u->s[i];
  if (b < 0x80) { *len = 1; return b; }
  if (b < 0xE0) { *len = 2; return ((b & 0x1F) << 6) | (u->s[i + 1] & 0x3F); }
  if (b < 0xF0) { *len = 3; return ((b & 0x0F) << 12) | ((u->s[i + 1] & 0x3F) << 6) | (u->s[i + 2] & 0x3F); }
  *len = 4; return ((b & 0x07) << 18) | ((u->s[i + 1] & 0x3F) << 12) | ((u->s[i + 2] & 0x3F) << 6) | (u->s[i + 3] & 0x3F);
}
static int java_space(uint32_t c) {
  return c == 0x20 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
static int java_iso_control(uint32_t c) { return c <= 0x1F || (c >= 0x7F && c <= 0x9F); }
/* a non-ASCII code point allowed where escapes are allowed ("other" chars) */
static int other_ok(uint32_t c) { return c > 128 && !java_space(c) && !java_iso_control(c); }

#define URI_ERR (-1)
/* scan [p,e) while chars are in class `ok` (+ escapes/other if esc); returns stop index or URI_ERR on bad escape */
static int64_t scan_cls(US* u, int64_t p, int64_t e, int (*ok)(int), int esc) {
  while (p < e) {
    uint8_t c = u->s[p];
    if (c < 0x80 && c && ok(c)) { p++; continue; }
    if (esc) {
      if (c == '%') {
        if (p + 3 <= e && (cls(u->s[p + 1]) & C_HEX) && (cls(u->s[p + 2]) & C_HEX)) { p += 3; continue; }
        return URI_ERR;
      }
      if (c >= 0x80) { int l; uint32_t cp = cp_at(u, p, &l); if (other_ok(cp)) { p += l; continue; } }
    }
    break;
  }
  return p;
}
static int check_cls(US* u, int64_t p, int64_t e, int (*ok)(int), int esc) { return scan_cls(u, p, e, ok, esc) == e ? 0 : URI_ERR; }
static int64_t find_stop(US* u, int64_t p, int64_t e, const char* err, const char* stop) {
  while (p < e) {
    uint8_t c = u->s[p];
    if (c < 0x80 && c && strchr(err, c)) return -1;
    if (c < 0x80 && c && strchr(stop, c)) break;
    p++;
  }
  return p;
}

typedef struct {
  int64_t sch_b, sch_e;          /* scheme, -1 if none */
  int opaque;
  int64_t ssp_b, ssp_e;
  int has_auth, server;          /* authority non-null; server-based */
  int64_t auth_b, auth_e;
  int64_t ui_b, ui_e;            /* userInfo, -1 none */
  int64_t host_b, host_e;
  int64_t port;                  /* -1 none */
  int64_t path_b, path_e;
  int64_t q_b, q_e;              /* query, -1 none */
  int64_t f_b, f_e;              /* fragment, -1 none */
} UriParts;

static int digits_only(US* u, int64_t p, int64_t e) { for (; p < e; p++) if (!(cls(u->s[p]) & C_DIGIT)) return 0; return 1; }
static int64_t parse_int_lim(US* u, int64_t p, int64_t e, int64_t lim) {
  int64_t v = 0; for (; p < e; p++) { v = v * 10 + (u->s[p] - '0'); if (v > lim) return -1; } return v;
}

/* IPv4 per JDK scanIPv4Address(strict=false) / parseIPv4Address */
static int64_t scan_byte(US* u, int64_t p, int64_t m) {
  int64_t q = p; while (q < m && (cls(u->s[q]) & C_DIGIT)) q++;
  if (q <= p) return q;
  if (q - p > 9 || parse_int_lim(u, p, q, 255) < 0) return p; /* >255 (NumberFormatException case also returns failure below) */
  return q;
}
/* returns end of IPv4 host, or -1 when not IPv4 (JDK: parse failure -> -1) */
static int64_t parse_ipv4(US* u, int64_t start, int64_t n) {
  int64_t p = start, q;
  int64_t m = p; while (m < n && ((cls(u->s[m]) & C_DIGIT) || u->s[m] == '.')) m++;
  if (m <= p) return -1;
  /* very long digit runs: JDK Integer.parseInt throws NFE -> caught -> -1 */
  for (int k = 0; k < 4; k++) {
    if ((q = scan_byte(u, p, m)) <= p) return -1;
    p = q;
    if (k < 3) { if (p < m && u->s[p] == '.') p++; else return -1; }
  }
  if (p < m) return -1;
  if (p > start && p < n && u->s[p] != ':') return -1;
  return p;
}
static int64_t parse_hostname(US* u, int64_t start, int64_t n) {
  int64_t p = start, q, l = -1;
  do {
    q = p; while (q < n && (cls(u->s[q]) & (C_DIGIT | C_ALPHA))) q++;
    if (q <= p) break;
    l = p; p = q;
    q = p; while (q < n && ((cls(u->s[q]) & (C_DIGIT | C_ALPHA)) || u->s[q] == '-')) q++;
    if (q > p) { if (u->s[q - 1] == '-') return URI_ERR; p = q; }
    if (p < n && u->s[p] == '.') p++; else break;
  } while (p < n);
  if (p < n && u->s[p] != ':') return URI_ERR;
  if (l < 0) return URI_ERR;
  if (l > start && !(cls(u->s[l]) & C_ALPHA)) return URI_ERR;
  return p;
}
/* minimal RFC 2732 IPv6 reference check (hex groups, '::' compression, optional trailing IPv4) */
static int check_ipv6(US* u, int64_t p, int64_t e) {
  int groups = 0, dbl = 0; int64_t i = p;
  if (i >= e) return URI_ERR;
  if (u->s[i] == ':') { if (i + 1 < e && u->s[i + 1] == ':') { dbl = 1; i += 2; } else return URI_ERR; }
  while (i < e) {
    int64_t j = i; while (j < e && (cls(u->s[j]) & C_HEX)) j++;
    if (j < e && u->s[j] == '.') { /* trailing IPv4 */
      int64_t k = parse_ipv4(u, i, e); if (k != e) return URI_ERR; groups += 2; i = e; break;
    }
    if (j == i || j - i > 4) return URI_ERR;
    groups++; i = j;
    if (i == e) break;
    if (u->s[i] != ':') return URI_ERR;
    i++;
    if (i < e && u->s[i] == ':') { if (dbl) return URI_ERR; dbl = 1; i++; if (i == e) break; }
    else if (i == e) return URI_ERR;
  }
  if (dbl ? groups > 7 : groups != 8) return URI_ERR;
  return 0;
}
static int parse_server(US* u, int64_t start, int64_t n, UriParts* r) {
  int64_t p = start, q;
  q = find_stop(u, p, n, "/?#", "@");
  if (q >= p && q < n && u->s[q] == '@') {
    if (check_cls(u, p, q, in_userinfo, 1)) return URI_ERR;
    r->ui_b = p; r->ui_e = q; p = q + 1;
  }
  if (p < n && u->s[p] == '[') {
    p++;
    q = find_stop(u, p, n, "/?#", "]");
    if (q > p && q < n && u->s[q] == ']') {
      int64_t rr = find_stop(u, p, q, "", "%");
      if (rr > p && rr < q) {
        if (check_ipv6(u, p, rr)) return URI_ERR;
        if (rr + 1 == q) return URI_ERR;
        if (check_cls(u, rr + 1, q, in_scope, 0)) return URI_ERR;
      } else if (check_ipv6(u, p, q)) return URI_ERR;
      r->host_b = p - 1; r->host_e = q + 1; p = q + 1;
    } else return URI_ERR;
  } else {
    q = parse_ipv4(u, p, n);
    if (q <= p) { q = parse_hostname(u, p, n); if (q == URI_ERR) return URI_ERR; }
    r->host_b = p; r->host_e = q; p = q;
  }
  if (p < n && u->s[p] == ':') {
    p++;
    q = find_stop(u, p, n, "", "/");
    if (q > p) {
      if (!digits_only(u, p, q)) return URI_ERR;
      int64_t v = parse_int_lim(u, p, q, 2147483647LL);
      if (v < 0) return URI_ERR;
      r->port = v; p = q;
    }
  }
  if (p < n) return URI_ERR;
  return 0;
}
static int parse_authority(US* u, int64_t p, int64_t n, UriParts* r) {
  int server_chars, reg_chars;
  int64_t s1;
  if (find_stop(u, p, n, "", "]") > p) {
    /* JDK quirk: taken whenever the authority does not start with ']'. L_SERVER_PERCENT matches
     * '%' as a plain char; non-ASCII "other" chars still pass through scanEscape. */
    int64_t i = p; int ok = 1;
    while (i < n) {
      uint8_t c = u->s[i];
      if (c < 0x80 && c && (in_server(c) || c == '%')) { i++; continue; }
      if (c >= 0x80) { int l; uint32_t cp = cp_at(u, i, &l); if (other_ok(cp)) { i += l; continue; } }
      ok = 0; break;
    }
    server_chars = ok;
  } else {
    s1 = scan_cls(u, p, n, in_server, 1);
    if (s1 == URI_ERR) return URI_ERR;
    server_chars = (s1 == n);
  }
  s1 = scan_cls(u, p, n, in_regname, 1);
  if (s1 == URI_ERR) return URI_ERR;
  reg_chars = (s1 == n);
  r->has_auth = 1; r->auth_b = p; r->auth_e = n;
  if (reg_chars && !server_chars) { r->server = 0; return 0; }
  int failed = 1;
  if (server_chars) {
    UriParts t = *r;
    if (parse_server(u, p, n, &t) == 0) { *r = t; r->server = 1; failed = 0; }
  }
  if (failed) {
    if (reg_chars) { r->server = 0; r->ui_b = r->host_b = -1; r->port = -1; return 0; }
    return URI_ERR;
  }
  return 0;
}
static int parse_hier(US* u, int64_t p, int64_t n, UriParts* r, int64_t* outp) {
  if (p + 1 < n && u->s[p] == '/' && u->s[p + 1] == '/') {
    p += 2;
    int64_t q = find_stop(u, p, n, "", "/?#");
    if (q > p) { if (parse_authority(u, p, q, r)) return URI_ERR; p = q; }
    else if (q < n) { /* empty authority before path/query/fragment: authority stays null */ }
    else return URI_ERR;
  }
  int64_t q = find_stop(u, p, n, "", "?#");
  if (check_cls(u, p, q, in_path, 1)) return URI_ERR;
  r->path_b = p; r->path_e = q; p = q;
  if (p < n && u->s[p] == '?') {
    p++;
    q = find_stop(u, p, n, "", "#");
    if (check_cls(u, p, q, in_uric, 1)) return URI_ERR;
    r->q_b = p; r->q_e = q; p = q;
  }
  *outp = p;
  return 0;
}
static int uri_parse(US* u, UriParts* r) {
  memset(r, 0, sizeof *r);
  r->sch_b = r->ui_b = r->host_b = r->q_b = r->f_b = -1; r->port = -1;
  int64_t n = u->n, p = find_stop(u, 0, n, "/?#", ":");
  if (p >= 0 && p < n && u->s[p] == ':') {
    if (p == 0) return URI_ERR;
    if (!(cls(u->s[0]) & C_ALPHA)) return URI_ERR;
    for (int64_t i = 1; i < p; i++) if (!(u->s[i] < 0x80 && in_scheme(u->s[i]))) return URI_ERR;
    r->sch_b = 0; r->sch_e = p;
    p++;
    if (p < n && u->s[p] == '/') {
      if (parse_hier(u, p, n, r, &p)) return URI_ERR;
    } else {
      int64_t q = find_stop(u, p, n, "", "#");
      if (q <= p) return URI_ERR;
      if (check_cls(u, p, q, in_uric, 1)) return URI_ERR;
      r->opaque = 1; r->ssp_b = p; r->ssp_e = q; p = q;
    }
  } else {
    if (parse_hier(u, 0, n, r, &p)) return URI_ERR;
  }
  if (p < n && u->s[p] == '#') {
    if (check_cls(u, p + 1, n, in_uric, 1)) return URI_ERR;
    r->f_b = p + 1; r->f_e = n; p = n;
  }
  if (p < n) return URI_ERR;
  return 0;
}

typedef struct { uint8_t* o; int64_t n, cap; int ovf; } KB;
static void kb_put(KB* k, uint8_t b) { if (k->n < k->cap) k->o[k->n] = b; else k->ovf = 1; k->n++; }
static void kb_lower(KB* k, US* u, int64_t b, int64_t e) { for (int64_t i = b; i < e; i++) { uint8_t c = u->s[i]; kb_put(k, (c >= 'A' && c <= 'Z') ? c + 32 : c); } }
/* copy with the two chars after each '%' lowered (java.net.URI.equal()) */
static void kb_pct(KB* k, US* u, int64_t b, int64_t e) {
  for (int64_t i = b; i < e; i++) {
    uint8_t c = u->s[i]; kb_put(k, c);
    if (c == '%' && i + 2 < e) {
      for (int j = 1; j <= 2; j++) { uint8_t d = u->s[i + j]; kb_put(k, (d >= 'A' && d <= 'Z') ? d + 32 : d); }
      i += 2;
    }
  }
}

/* Canonical key of the Java string (already Java-UTF-8-repaired). Component tags are control
 * bytes, which can never occur inside a parsed URI, so the encoding is injective. */
EXPORT int64_t dkr_uri_key(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
  US u = { s, n }; UriParts r;
  if (uri_parse(&u, &r)) return -1;
  KB k = { out, 0, cap, 0 };
  if (r.sch_b >= 0) { kb_put(&k, 1); kb_lower(&k, &u, r.sch_b, r.sch_e); }
  if (r.opaque) {
    kb_put(&k, 2); kb_pct(&k, &u, r.ssp_b, r.ssp_e);
  } else {
    if (r.has_auth) {
      if (r.server) {
        kb_put(&k, 3);
        if (r.ui_b >= 0) { kb_put(&k, 4); kb_pct(&k, &u, r.ui_b, r.ui_e); }
        kb_put(&k, 5); kb_lower(&k, &u, r.host_b, r.host_e);
        if (r.port >= 0) { char buf[16]; int l = snprintf(buf, sizeof buf, "%lld", (long long)r.port); kb_put(&k, 6); for (int i = 0; i < l; i++) kb_put(&k, buf[i]); }
      } else { kb_put(&k, 7); kb_pct(&k, &u, r.auth_b, r.auth_e); }
    }
    kb_put(&k, 8); kb_pct(&k, &u, r.path_b, r.path_e);
    if (r.q_b >= 0) { kb_put(&k, 9); kb_pct(&k, &u, r.q_b, r.q_e); }
  }
  if (r.f_b >= 0) { kb_put(&k, 10); kb_pct(&k, &u, r.f_b, r.f_e); }
  if (k.ovf) return -2;
  return k.n;
}

/* Full action key: canonical URI(path) + 0x00 + (DV absent ? 0x00 : 0x01 + dvUniqueId).
 * Inputs are raw UTF-8 bytes as stored; Java decoding/replacement is applied here. */
EXPORT int64_t dkr_action_key(const uint8_t* path, int64_t plen, int has_dv,
                              const uint8_t* st, int64_t stlen, const uint8_t* pid, int64_t pidlen,
                              int has_off, int32_t off, uint8_t* out, int64_t cap) {
  uint8_t* tmp = malloc(plen * 3 + 16);
  int64_t tl = dkr_java_utf8(path, plen, tmp, plen * 3 + 16);
  int64_t n = dkr_uri_key(tmp, tl, out, cap);
  free(tmp);
  if (n < 0) return n;
  if (n + 2 > cap) return -2;
  out[n++] = 0;
  if (!has_dv) { out[n++] = 0; return n; }
  out[n++] = 1;
  int64_t a = dkr_java_utf8(st, stlen, out + n, cap - n); if (a < 0) return -2; n += a;
  a = dkr_java_utf8(pid, pidlen, out + n, cap - n); if (a < 0) return -2; n += a;
  if (has_off) { char buf[40]; int l = snprintf(buf, sizeof buf, "@Optional[%d]", off); if (n + l > cap) return -2; memcpy(out + n, buf, l); n += l; }
  return n;
}

/* ------------------------------------------------------------------------------------------ */
/* Key set + checkpoint probe (ActiveAddFilesIterator.java:192-234 for isFromCheckpoint=true)  */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint64_t h; int64_t off; int32_t len; int32_t flags; } KEnt;
typedef struct { KEnt* t; int64_t cap, n; Buf keys; } KSet;
static uint64_t fnv(const uint8_t* p, int64_t n) { uint64_t h = 1469598103934665603ULL; for (int64_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ULL; } return h ? h : 1; }
EXPORT void* dkr_keyset_new(void) { KSet* k = calloc(1, sizeof(KSet)); k->cap = 1024; k->t = calloc(k->cap, sizeof(KEnt)); return k; }
EXPORT void dkr_keyset_free(void* h) { KSet* k = h; if (!k) return; free(k->t); free(k->keys.p); free(k); }
static KEnt* ks_find(KSet* k, const uint8_t* key, int64_t n, uint64_t h, int insert) {
  if (insert && (k->n + 1) * 2 > k->cap) {
    KEnt* old = k->t; int64_t oc = k->cap; k->cap *= 2; k->t = calloc(k->cap, sizeof(KEnt));
    for (int64_t i = 0; i < oc; i++) if (old[i].h) { int64_t j = old[i].h & (k->cap - 1); while (k->t[j].h) j = (j + 1) & (k->cap - 1); k->t[j] = old[i]; }
    free(old);
  }
  int64_t j = h & (k->cap - 1);
  while (k->t[j].h) {
    if (k->t[j].h == h && k->t[j].len == n && !memcmp(k->keys.p + k->t[j].off, key, n)) return &k->t[j];
    j = (j + 1) & (k->cap - 1);
  }
  if (!insert) return NULL;
  k->t[j].h = h; k->t[j].off = k->keys.n; k->t[j].len = (int32_t)n; k->t[j].flags = 0;
  buf_put(&k->keys, key, n); k->n++;
  return &k->t[j];
}
/* flags: bit0 = in addFilesFromJson, bit1 = in tombstonesFromJson */
EXPORT void dkr_keyset_or(void* h, const uint8_t* key, int64_t n, int flags) { KEnt* e = ks_find(h, key, n, fnv(key, n), 1); e->flags |= flags; }
EXPORT int dkr_keyset_get(void* h, const uint8_t* key, int64_t n) { KEnt* e = ks_find(h, key, n, fnv(key, n), 0); return e ? e->flags : 0; }

/* Probe assembled checkpoint columns. add_row_def: def of add.path (add struct non-null iff >= 1;
 * path value iff == 2). DV columns: def levels of deletionVector leaves (dv non-null iff >= 2 for
 * storageType); may be NULL when the file has no DV columns.
 * counters[0]+=addFilesSeen, [4]+=activeAddFiles, [3]+=duplicateAddFiles. Returns -1 on URI error
 * (row index in *bad_row). */
EXPORT int dkr_probe_checkpoint(void* ks, int64_t n_rows,
                                const uint8_t* path_def, const int64_t* path_offs, const uint8_t* path_chars,
                                const uint8_t* dv_st_def, const int64_t* dv_st_offs, const uint8_t* dv_st_chars,
                                const int64_t* dv_pid_offs, const uint8_t* dv_pid_chars,
                                const uint8_t* dv_off_def, const int32_t* dv_off_vals, int dv_off_maxdef,
                                uint8_t* sel, int64_t* counters, int64_t* bad_row) {
  int64_t cap = 1 << 16; uint8_t* key = malloc(cap);
  for (int64_t r = 0; r < n_rows; r++) {
    sel[r] = 0;
    if (path_def[r] < 1) continue;                 /* add struct is null */
    counters[0]++;
    int has_dv = dv_st_def && dv_st_def[r] >= 2;
    int64_t pl = path_offs[r + 1] - path_offs[r];
    int64_t need = pl * 3 + 512;
    if (need > cap) { cap = need * 2; key = realloc(key, cap); }
    int64_t kl = dkr_action_key(path_chars + path_offs[r], pl, has_dv,
                                has_dv ? dv_st_chars + dv_st_offs[r] : NULL, has_dv ? dv_st_offs[r + 1] - dv_st_offs[r] : 0,
                                has_dv ? dv_pid_chars + dv_pid_offs[r] : NULL, has_dv ? dv_pid_offs[r + 1] - dv_pid_offs[r] : 0,
                                has_dv && dv_off_def[r] == dv_off_maxdef, has_dv ? dv_off_vals[r] : 0, key, cap);
    if (kl < 0) { *bad_row = r; free(key); return -1; }
    int fl = dkr_keyset_get(ks, key, kl);
    if (fl & 1) { counters[3]++; continue; }     /* alreadyReturned -> duplicate */
    if (fl & 2) continue;                          /* alreadyDeleted */
    sel[r] = 1; counters[4]++;
  }
  free(key);
  return 0;
}
