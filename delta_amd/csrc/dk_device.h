// Device-side data model shared by the host orchestration (dk_host.cpp) and the kernels.
#pragma once
#define DK_DEVICE_TYPES 1   // dk_thrift.h's apply_page_header needs DPage / DChunk
#include <stdint.h>

namespace dk {

// One column chunk (file part x projected leaf x row group).
struct DChunk {
  const uint8_t* file;   // device copy of the file's projected chunks (padded)
  int32_t col;           // output column (DColumn index)
  int32_t phys, width, max_def, max_rep, rep_def, codec;
  int32_t dict_page;     // page index of the dictionary page, -1 if none
  int64_t dict_pos;      // string dictionaries: scratch offset (int32 per entry + 1)
  int64_t dict_hash_off; // key columns: offset of this chunk's dictionary entries in DColumn.dhash
};

enum : int32_t { PF_DICT = 1 };
enum : int32_t { PS_OK = 0, PS_BAD_HEADER = 1, PS_BAD_LEVELS = 2, PS_BAD_VALUES = 3,
                 PS_UNSUPPORTED = 4, PS_BAD_DICT = 5, PS_BAD_SNAPPY = 6 };

struct DPage {
  int64_t hdr_off;       // offset of the page header in the packed chunk image (input)
  int32_t chunk;         // DChunk index (input)
  int32_t flags;         // PF_* (input)
  // parsed header (k_page_headers)
  int32_t ptype, enc, num_values, dl_len, rl_len, csize, usize, hdr_len;
  int32_t status, is_comp;
  int64_t data_off;      // offset of the page body in the packed chunk image
  int64_t unc_off;       // offset into the decompression arena, -1 = read in place (input)
  // totals (k_tile_scan1 / k_tile_scan2: sums over the page's level tiles)
  int32_t n_rows, n_entries, n_values, pad;
  int64_t n_chars;
  // bases within the column (first tile's bases)
  int64_t row_base, entry_base, value_base, char_base;
  int64_t pos_base;      // string positions scratch offset (input, int32 per value + 1)
  // run tables of the RLE/bit-packed hybrid streams (k_page_runs), offsets into the run scratch
  // (input): rep levels, def levels, dictionary indices / RLE booleans; run_cap runs each
  // (standard writers emit >= 8 values per run; more runs -> PS_UNSUPPORTED)
  int64_t run_r, run_d, run_i;
  int32_t run_cap, nrun_r, nrun_d, nrun_i;
  int32_t idx_cover;     // values covered by the index stream's runs
  int32_t first_tile, n_tiles;   // level tiles of this page (input)
  int32_t pad2;
  int64_t vbytes;        // bytes of the value section (after the levels)
  // string positions (BYTE_ARRAY PLAIN data pages and dictionary pages): 16 KiB chunks (input)
  int32_t pchunk0, npchunk;
  int32_t pos_fail;      // speculative positions rejected -> serial walk (k_pos_fallback)
  int32_t pad3;
};

// Speculative snappy decode (k_snap_*): compressed streams are cut into DK_SNAP_SEG-byte segments,
// each walked by one lane; the walker records its first DK_SNAP_REC tag positions.
#ifndef DK_SNAP_SEG_BYTES
#define DK_SNAP_SEG_BYTES 2048
#endif
constexpr int DK_SNAP_SEG = DK_SNAP_SEG_BYTES;
constexpr int DK_SNAP_REC = 16;
struct SnapCtx {
  const DChunk* chunks;
  const DPage* pages;
  uint8_t* arena;
  const int32_t* cpage;      // compressed page -> page index
  const int32_t* sbase;      // compressed page -> first segment (n_cpages + 1)
  const int32_t* spage;      // segment -> compressed page
  int32_t nseg;
  int32_t* w_exit;           // walker: first tag start >= segment end (-1: the chain broke)
  int32_t* w_out;            // walker: output bytes of its tags
  int32_t* w_npos;           // walker: recorded positions
  int32_t* w_pos;            // [DK_SNAP_REC][nseg] tag positions
  int32_t* w_cum;            // [DK_SNAP_REC][nseg] walker output before that tag
  int32_t* relink;           // segments k_snap_link hands to the staged relink walk (or null: no budget),
  int32_t* relink_n;         // a launch's at relink[k0 ...], counted in relink_n[k0] (slices run concurrently)
  int32_t* t_entry;          // true entry (link: speculative; fix: verified)
  int32_t* t_out;            // true output bytes
  int32_t* t_exit;           // true exit (-1: malformed)
  const int32_t* fbase;      // compressed page -> first fragment (n_cpages + 1)
  int64_t* fstart;           // fragment -> compressed offset of its first tag
  int64_t* t_ob;             // segment -> output offset of its first byte within the page (k_snap_fix)
  int32_t* fseg;             // fragment -> segment holding its first output byte (k_snap_fix, bitmap mode)
  int32_t* serial;           // compressed page -> 1: decode on the serial path
  uint64_t* tbits;           // page mode: tag-start bitmap, DK_SNAP_SEG / 64 words per segment (or null)
  int32_t page_mode;         // 1: whole pages decode in order (no 64 KiB fragment starts needed)
  int32_t k0, k1;            // launch range: segments [k0, k1) (k_snap_walk / k_snap_link)
  int32_t c0;                // launch range: first compressed page (k_snap_fix)
};


// One 16 KiB chunk of a string region for the chunk-parallel position scan.
struct DPosChunk {
  int32_t page, blk0;    // (input) page, first aligned 16-byte block of the region
  int32_t cnt, base;     // candidates in the chunk, their first index
  int32_t first;         // region offset of the chunk's first candidate
  int32_t last_next;     // its last candidate's successor (offset + 4 + length)
  int32_t ok;            // every other candidate's successor is the next candidate of the chunk
  int32_t pad;
};
constexpr int DK_POS_CHUNK = 16384;
// candidate offsets k_pos_count keeps per chunk: a value takes >= 4 region bytes (an empty string is
// its length prefix alone), so a chunk holds at most DK_POS_CHUNK / 4 of them
constexpr int DK_POS_CAP = DK_POS_CHUNK / 4 + 8;
// k_expand record kinds (per-page work lists built on the device from per-group counts)
enum : int { EX_TILE = 0, EX_POSCHUNK = 1, EX_FRAG = 2, EX_SEG = 3 };

// One run of an RLE/bit-packed hybrid stream: values [start, next.start) are `val` (RLE,
// bp_idx < 0) or bit-packed from byte bp_off (relative to the page data start) on.
struct Seg {
  int32_t start;
  int32_t bp_idx;
  uint32_t val;
  uint32_t bp_off;
};

// A level tile: DK_LEVEL_TILE consecutive levels of one data page (one workgroup per tile in
// every level pass). Counts from k_tile_count / k_tile_chars, column bases from the scans.
struct DTile {
  int32_t page, lvl0;    // (input)
  int32_t n_rows, n_entries, n_values, pad;
  int64_t n_chars;
  int64_t row_base, entry_base, value_base, char_base;
};
#ifndef DK_LEVEL_TILE_LEVELS
#define DK_LEVEL_TILE_LEVELS 2048
#endif
constexpr int DK_LEVEL_TILE = DK_LEVEL_TILE_LEVELS;

struct DColumn {
  int32_t first_page, n_pages;   // data pages, contiguous in the page table, in file order
  int32_t first_tile, n_tiles;   // level tiles, contiguous, in page order
  int32_t phys, width, max_def, max_rep, rep_def, present;
  int32_t null_only;         // no value anywhere -> no value buffers are materialised
  int32_t key_hash;          // 1: this is the reconciliation key column (add.path) -> emit path hashes
  int64_t n_rows;
  uint8_t* row_def;
  int64_t* row_offs;
  uint8_t* entry_def;
  uint8_t* fixed;
  int64_t* offs;
  uint8_t* chars;
  int64_t n_entries, n_chars;    // totals (k_tile_scan1 / k_tile_scan2)
  int64_t cap_entries, cap_chars;
  // key_hash columns only: canonical-path hash (seed kDecodeSeed) per value (scratch, filled by
  // k_string_copy for PLAIN pages, 0 = not computed) and per row (forwarded by k_tile_decode;
  // 0 = null row or "compute in the probe")
  uint64_t* vhash;
  uint64_t* hash;
  uint64_t* dhash;       // key columns: path hash of every dictionary entry (k_string_copy)
};

// streaming reader: one leaf's window of batches -> validity bits + int32 offsets (dk_arrow.hip)
struct ArrowWin {
  const uint8_t* def;          // per value definition levels (row_def or entry_def), window-based
  const int64_t* offs;         // byte-array offsets (nv + 1), window-based, or null
  const int64_t* row_offs;     // repeated leaf: entry offsets per row (nr + 1), window-based, or null
  int64_t nv, nr;              // values / rows in the window
  int32_t max_def;
  uint64_t* bits;              // out: ceil(nv / 64) words
  int32_t* offs32;             // out: nv + 1
  int32_t* row_offs32;         // out: nr + 1
  int32_t* overflow;           // out: set when a rebased offset does not fit int32
};

// deletion vectors: one roaring container of one DV (dk_dv.hip)
enum : int32_t { DV_ARRAY = 0, DV_BITMAP = 1, DV_RUN = 2 };
struct DvCont {
  int64_t src;        // byte offset of the container payload in the uploaded blob
  int64_t out_word;   // first u64 word of the DV's bitmap
  int64_t word0;      // first word of the container's 64K-value range, relative to out_word
  int64_t nwords;     // words of the DV's bitmap (bound for bitmap containers)
  int32_t type, n;    // DV_*; values (array) or runs (run)
};

constexpr uint32_t kDecodeSeed = 0;   // seed of the path hashes computed during decode
constexpr int DK_COPY_TILE = 128;     // values per k_string_copy workgroup (host tile table step)

// Commit-tail actions, one per JSON line, in replay order. JA_CKADD: an add row of a JSON-format
// checkpoint part (a V2 checkpoint's JSON manifest, ActionsIterator.java:213-248): probed like a
// Parquet checkpoint row, never entered into the key table.
enum : int32_t { JA_NONE = 0, JA_ADD = 1, JA_REMOVE = 2, JA_CKADD = 3 };
struct DJsonAction {
  int32_t kind;          // JA_*
  int32_t step;          // global batch index in replay order
  int32_t row;           // row within its batch
  int32_t has_dv, has_off, dv_off;
  int64_t path_off; int32_t path_len, pad0;
  int64_t st_off; int32_t st_len, pad1;
  int64_t pid_off; int32_t pid_len, pad2;
  int64_t canon_off;     // arena offset of the canonical path stream (cap path_len + 64)
  int32_t canon_len, dv_len;   // canonical path bytes; dv stream bytes follow the path bytes
  uint64_t h;
  int32_t slot, status;
};

// Probe table slot (open addressing on the 64-bit key hash).
struct Slot {
  unsigned long long h;          // 0 = empty
  unsigned long long first_add;  // min (step<<32 | row) over JSON adds, ~0 = none
  int32_t rep;                   // representative action index
  int32_t min_rm_step;           // min step over JSON removes, INT32_MAX = none
};

enum : int32_t { E_URI = 1, E_UTF8 = 2, E_COLLISION = 4, E_PAGE = 8, E_STATS = 16, E_PART = 32 };

// Data-skipping program (a dk_program compiled by dk_skip_compile, dk_expr.cpp, laid out in one device
// buffer): the stats fields to read from each row's add.stats JSON (or add.stats_parsed columns) and
// a postfix program over them. Any number of paths, ops and literal bytes; the evaluation stack is at
// most SK_STACK deep (the compiler re-associates AND / OR chains to stay under it).
constexpr int SK_STACK = 32;        // evaluation stack (dk_expr.cpp kMaxStack)
constexpr int SK_NARROW = 8;        // programs of up to this many paths keep the values in registers
constexpr int SK_WINDOW = 32;       // paths extracted per pass over a JSON object (one mask word)
enum : int32_t { SK_LONG = 0, SK_INT = 1, SK_SHORT = 2, SK_BYTE = 3, SK_DATE = 4, SK_STRING = 5, SK_TIMESTAMP = 6, SK_DECIMAL = 7, SK_TIMESTAMP_NTZ = 8,
                 SK_FLOAT = 9, SK_DOUBLE = 10 };
enum : int32_t { OP_STAT = 0, OP_LIT = 1, OP_LT = 2, OP_LE = 3, OP_GT = 4, OP_GE = 5, OP_EQ = 6, OP_AND = 7, OP_OR = 8, OP_LIT_STR = 9, OP_TIMEADD = 10, OP_LIT_DEC = 11,
                 OP_FCMP = 12 };
enum : int32_t { FC_LT = 0, FC_LE = 1, FC_GT = 2, FC_GE = 3, FC_ALL = 4, FC_NONE = 5 };
struct DSkipProg {
  int32_t n_paths, n_ops;
  int32_t max_comps;               // most name components of a path
  const int32_t* path_type;        // [n_paths] SK_*
  const int32_t* path_comp;        // [n_paths + 1]: path p's name components are [path_comp[p], path_comp[p + 1])
  const int32_t* comp_off;         // per component: its name in names
  const int32_t* comp_len;
  const int32_t* op;               // [n_ops]
  const int32_t* arg;
  const int64_t* lit;
  const char* names;               // component names and literal bytes (UTF-8)
};

// Partition-pruning program (a dk_program compiled by dk_part_compile): the partition columns it reads
// (physical names, looked up in each row's partitionValues map when the program reads them) and a
// postfix program over their deserialized values.
constexpr int PP_STACK = 32;
enum : int32_t { PT_LONG = 0, PT_INT = 1, PT_SHORT = 2, PT_BYTE = 3, PT_STRING = 4, PT_DATE = 5, PT_DECIMAL = 6,
                 PT_BOOL = 7, PT_F32 = 8, PT_F64 = 9, PT_TIMESTAMP = 10 };
enum : int32_t { PO_FIELD = 0, PO_LIT_INT = 1, PO_LIT_STR = 2, PO_LIT_NULL = 3, PO_LT = 4, PO_LE = 5, PO_GT = 6,
                 PO_GE = 7, PO_EQ = 8, PO_NSEQ = 9, PO_ISNULL = 10, PO_ISNOTNULL = 11, PO_NOT = 12, PO_AND = 13,
                 PO_OR = 14, PO_LIT_DEC = 15, PO_FCMP = 16, PO_COALESCE = 17,
                 // string functions on the top of the stack; lit = offset | length << 32 of a pool
                 // operand, arg = 1 for a null literal (the result is null):
                 PO_STARTS_WITH = 18,    // String.startsWith(literal)
                 PO_LIKE = 19,           // LIKE pattern compiled to tokens (byte pairs: 0 b literal, 1 one
                                         // code point, 2 any run)
                 PO_SUBSTR = 20,         // SUBSTRING(s, pos[, len]): lit = (uint32)pos | len << 32, arg = has len
                 PO_LIKE_DYN = 21,       // LIKE(s, pattern) with the pattern a value (top) over s (below):
                                         // arg = the escape code point (LikeExpressionEvaluator.eval)
                 PO_TIMEADD = 22,        // TIMEADD(ts, millis): ts (below) + millis (top) * 1000, wrapping
                 PO_FCMP2 = 23 };        // two float / double / integral values compared after widening:
                                         // arg = comparison (PO_LT..PO_NSEQ) | double-wide << 8 | form of
                                         // the lower operand << 12 | of the upper << 16 (FF_*)
enum : int32_t { FF_INTEGRAL = 0, FF_FLOAT = 1, FF_DOUBLE = 2 };   // a float / double literal: its IEEE bits
struct DPartProg {
  int32_t n_fields, n_ops;
  int32_t wide;                    // the program holds PO_FCMP2: k_part_eval_wide (digit buffers in scratch)
  const int32_t* field_type;       // [n_fields] PT_*
  const int32_t* name_off;         // physical column name (map key) in pool
  const int32_t* name_len;
  const int32_t* op;               // [n_ops]
  const int32_t* arg;              // PO_FIELD: field; PO_LIT_STR / PO_LIT_DEC: length; PO_COALESCE: operands
  const int64_t* lit;              // PO_LIT_INT: value; PO_LIT_STR / PO_LIT_DEC: offset into pool
  const char* pool;                // field names and literals (UTF-8)
};

// partitionValues map rows: repeated key / value leaves (row_offs over entries), per action for the
// commit tail (act_row maps an action to its row) or per row for a checkpoint file
struct MapRows {
  int64_t n;
  const int64_t* act_row;        // null: row r is action r
  const uint8_t* row_def; int32_t rep_def; int32_t v_max_def;
  const int64_t* row_offs;
  const int64_t* k_offs; const uint8_t* k_chars;
  const uint8_t* v_def; const int64_t* v_offs; const uint8_t* v_chars;
  int64_t row_tag;
};

// Rows whose stats the skipping kernel reads: a decoded string column (row_def / offs / chars)
// or, for the commit tail, explicit (offset, length) pairs per action (length < 0 = null).
struct StatsRows {
  int64_t n;
  const uint8_t* row_def; int32_t max_def;
  int32_t marked;               // 1: only rows whose selection byte is 2 (k_stats_parsed's hand-offs)
  const int64_t* offs;          // column mode: n + 1 offsets
  const int64_t* soff;          // action mode: offset per row
  const int32_t* slen;          // action mode: length per row (< 0: null)
  const uint8_t* chars;
  int64_t row_tag;
};

// Data skipping over add.stats_parsed (typed Parquet columns of the same stats, one per program
// path): per path its definition levels and values, and how to read them.
// value kinds: TP_INT integral / date / timestamp micros (INT32 sign-extended or INT64), TP_MILLIS
// timestamp millis, TP_INT96 timestamp (nanos of day + Julian day), TP_STR UTF-8 bytes, TP_DEC
// unscaled INT32 / INT64 with a scale, TP_F32 / TP_F64 IEEE float / double
enum : int32_t { TP_INT = 0, TP_MILLIS = 1, TP_INT96 = 2, TP_STR = 3, TP_DEC = 4, TP_F32 = 5, TP_F64 = 6 };
struct TypedPath {
  const uint8_t* def;
  const uint8_t* vals;                // fixed-width values, one per row (TP_STR: null)
  const int64_t* offs;                // TP_STR: n + 1 offsets into chars
  const uint8_t* chars;
  int32_t max_def;
  int32_t width;                      // 4, 8 or 12 (INT96)
  int32_t kind;                       // TP_*
  int32_t scale;                      // TP_DEC: the decimal's scale
};
struct StatsParsedRows {
  int64_t n;
  int32_t n_paths;
  int32_t struct_def;                 // row_def >= this: add.stats_parsed is non-null
  const TypedPath* paths;             // [n_paths], device memory, in the program's path order
  // the add.stats JSON of the same rows (column mode): the reference reads only it, so a row with a
  // null add.stats keeps its selection, and a row whose typed values cannot stand for the JSON (a
  // null stats_parsed struct, a float -0.0 -- Kernel reads "-0.0" as +0.0 but "-1e-400" as -0.0 --,
  // sub-microsecond INT96 nanos) is marked (selection byte 2) for k_stats_eval over its JSON
  StatsRows js;
};

// Per-lane scratch of the wide (> SK_NARROW paths) skipping kernels: path-major arrays of `lanes`
// entries each (values, set words, typed kinds / scales / pointers); grids are sized to `lanes`.
struct SkScratch {
  long long* val;
  uint32_t* setw;
  int32_t* kind;
  int32_t* scale;
  const uint8_t** ptr;
  long long lanes;
};

// Device-side counters and error state of one replay.
struct DState {
  unsigned long long counters[5];        // commit-tail part (k_json_select)
  unsigned long long ckpt_counters[5];   // checkpoint part (k_probe_fast / k_probe_cand)
  int32_t err_flags;
  int32_t err_row_part;
  long long err_row;
};

// Column pointers the checkpoint probe reads (one checkpoint file).
struct ProbeCols {
  const uint8_t* path_def; const int64_t* path_offs; const uint8_t* path_chars;
  const uint64_t* path_hash;   // per-row path hashes from decode (seed kDecodeSeed), or null
  const uint8_t* st_def; const int64_t* st_offs; const uint8_t* st_chars;
  const int64_t* pid_offs; const uint8_t* pid_chars;
  const uint8_t* off_def; const int32_t* off_vals; int32_t off_maxdef;
  int32_t has_dv;
  int64_t n_rows;
  int64_t row_tag;   // added to the row index in error reports
};

// Owner-partitioned reconciliation (multi-GPU "owner" mode): one key record routed to the rank that
// owns its hash (h mod world), with the key's canonical bytes (canonical path stream, then the
// dvUniqueId stream) travelling in a byte buffer alongside, in the same order. Commit-tail actions
// carry their replay position (global batch step, row in batch); checkpoint candidates carry
// kind JA_CKADD. src: the sender's index of the record's action / candidate.
struct OwnerKeyRec {
  uint64_t h;
  int32_t kind, step, row;
  int32_t key_len, canon_len;       // key bytes; the first canon_len are the path stream
  int32_t src;
};
static_assert(sizeof(OwnerKeyRec) == 32, "OwnerKeyRec layout (dkgpu.h owner entry points)");

// All checkpoint files of a replay for the one-launch probe: rows numbered across the files.
struct ProbeSet {
  const ProbeCols* cols;       // per file (device memory)
  const int64_t* row0;         // n_files + 1 prefix of the files' rows
  uint8_t* const* sel;         // per file selection bytes
  int32_t n_files;
  int64_t total;
};

}  // namespace dk
