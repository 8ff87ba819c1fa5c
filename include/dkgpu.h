/*
 * libdkgpu — MI355X-native Delta Kernel snapshot state reconstruction (C ABI).
 *
 * This is the drop-in boundary a Kernel Engine binds through JNI/FFM. Every
 * entry point is plain C: pointers, sizes, status codes. Status 0 = OK; non-zero = error, with
 * the message from dk_last_error() (the Java side rethrows it as KernelEngineException, as
 * DeltaErrors.wrapEngineException would: kernel-api/.../internal/DeltaErrors.java:315-345).
 *
 * Reference interfaces replaced (paths relative to /root/reference/kernel/):
 *   dk_engine_*          Engine / DefaultEngine.create
 *                        (kernel-api/src/main/java/io/delta/kernel/engine/Engine.java:30-64,
 *                         kernel-defaults/.../defaults/engine/DefaultEngine.java:62-64)
 *   dk_parquet_*         ParquetHandler.readParquetFiles
 *                        (kernel-api/.../engine/ParquetHandler.java:64-68;
 *                         kernel-defaults/.../engine/DefaultParquetHandler.java:55-94)
 *   dk_json_tail_*       JsonHandler.readJsonFiles over the commit tail
 *                        (kernel-api/.../engine/JsonHandler.java:87-91;
 *                         kernel-defaults/.../engine/DefaultJsonHandler.java:79-157)
 *   dk_reader_*, dk_batch_*  the streaming form of ParquetHandler.readParquetFiles: a
 *                        CloseableIterator<ColumnarBatch> of <= parquet.reader.batch-size rows
 *                        (engine/ParquetHandler.java:59-68; defaults/internal/parquet/
 *                         ParquetFileReader.java:54-147, ParquetSchemaUtils.java:92-138)
 *   dk_dv_*              deletion-vector bitmaps for data reads: DeletionVectorUtils.loadNewDvAndBitmap
 *                        and SelectionColumnVector (kernel-api/.../Scan.java:176-199;
 *                         internal/deletionvectors/DeletionVectorStoredBitmap.java:50-129,
 *                         RoaringBitmapArray.java:100-229)
 *   dk_replay_*          the active-AddFile log replay behind Scan.getScanFiles
 *                        (kernel-api/.../Scan.java:101; internal/replay/LogReplay.java:194-206,
 *                         internal/replay/ActiveAddFilesIterator.java:146-275) and its
 *                         ScanMetrics counters (internal/metrics/ScanMetrics.java:28-40)
 */
#ifndef DKGPU_H
#define DKGPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dk_engine dk_engine;
typedef struct dk_parquet dk_parquet;
typedef struct dk_json_tail dk_json_tail;
typedef struct dk_replay dk_replay;
typedef struct dk_reader dk_reader;
typedef struct dk_dv_set dk_dv_set;

typedef struct dk_config {
  int32_t parquet_batch_size;  /* delta.kernel.default.parquet.reader.batch-size (default 1024) */
  int32_t json_batch_size;     /* delta.kernel.default.json.reader.batch-size (default 1024)    */
  int32_t device;              /* HIP device ordinal                                           */
  int32_t flags;               /* DK_FLAG_*                                                    */
} dk_config;

#define DK_FLAG_TIMING 1       /* record per-kernel HIP events on the engine stream */

/* Assembled column, the layout both the device decoder and the CPU oracle produce.
 *  non-repeated leaf : row_def[n_rows] (definition level per row); fixed[n_rows*width] (0 where
 *                      null) or offs[n_rows+1] + chars (zero-length where null)
 *  repeated leaf     : row_def[n_rows] (def of the row's first level: null vs empty map/list),
 *                      row_offs[n_rows+1] entry offsets; entry_def[n_entries]; values entry-dense
 *  present == 0      : the leaf is missing from the file -> every row null
 *                      (ParquetColumnReaders.NonExistentColumnReader, :119-134) */
typedef struct dk_column {
  int64_t n_rows, n_entries, n_chars;
  int32_t phys, width, max_def, max_rep, rep_def, present;
  const uint8_t* row_def;
  const int64_t* row_offs;
  const uint8_t* entry_def;
  const uint8_t* fixed;
  const int64_t* offs;
  const uint8_t* chars;
} dk_column;

const char* dk_last_error(void);
const char* dk_version(void);

int  dk_engine_create(const dk_config* cfg, dk_engine** out);
void dk_engine_destroy(dk_engine* e);

/* ---- ParquetHandler: open files (host read + footer/offset-index parse + H2D), decode on GPU --
 * leaves: dotted projected leaf paths ("add.path", "add.partitionValues.key_value.key", ...);
 * matched by exact name, then case-insensitively (ParquetSchemaUtils.java:92-119). Only the
 * projected column chunks (and their offset indexes) are read from the file and copied to HBM. */
int  dk_parquet_open(dk_engine* e, const char* const* paths, int32_t n_files,
                     const char* const* leaves, int32_t n_leaves, dk_parquet** out);
/* The same over row groups [rg_lo[i], rg_hi[i]) of file i (rg_hi < 0: to the end; NULL arrays: all
 * row groups): the file then reads as just those rows. Used to shard one checkpoint part over
 * several GPUs and for row-group pruning (ParquetFileReader.java:118-134 filters row groups). */
int  dk_parquet_open_rg(dk_engine* e, const char* const* paths, int32_t n_files,
                        const char* const* leaves, int32_t n_leaves, const int32_t* rg_lo,
                        const int32_t* rg_hi, dk_parquet** out);
/* Row counts of a file's row groups from its footer (no device work); *n = number of groups. */
int  dk_parquet_row_groups(const char* path, int64_t* rows, int32_t cap, int32_t* n);
/* keep[g] = 0 for the row groups whose footer statistics show `leaf` null in every row (used by the
 * snapshot-load P&M pass to decode only row groups that can hold a protocol / metaData row). */
int  dk_parquet_nonnull_row_groups(const char* path, const char* leaf, uint8_t* keep, int32_t cap, int32_t* n);
/* The same over an explicit ascending list of row groups per file: rg_count[i] groups taken from
 * rg_list (concatenated over the files), rg_count[i] < 0 = all groups of file i. */
int  dk_parquet_open_sel(dk_engine* e, const char* const* paths, int32_t n_files,
                         const char* const* leaves, int32_t n_leaves, const int32_t* rg_count,
                         const int32_t* rg_list, dk_parquet** out);
/* The same, asynchronous: returns once the footers, page headers and tables are read (num_rows /
 * row_offset answer at once); the chunk reads, sizing passes and value decode go on on a library
 * thread, files becoming ready slice by slice. dk_parquet_column waits for its file, every other
 * call for the whole open (its error, if any, is reported there). A replay attached meanwhile
 * attaches each file as it gets ready, and a grouped run issues each group when a wait first needs
 * it. Falls back to the synchronous open where the per-slice decode is off (DK_SLICE_DECODE=0,
 * DK_OPEN_ADAPTIVE=0, DK_SNAPPY_MODE=page, DK_ASYNC_OPEN=0). */
int  dk_parquet_open_async(dk_engine* e, const char* const* paths, int32_t n_files,
                           const char* const* leaves, int32_t n_leaves, const int32_t* rg_count,
                           const int32_t* rg_list, dk_parquet** out);

/* Row-group pruning predicate: the checkpoint predicate ActionsIterator hands the ParquetHandler for
 * checkpoint parts and sidecars (KA/internal/replay/ActionsIterator.java:336-351; the partition filter
 * rewritten onto add.partitionValues_parsed, PartitionUtils.java:275-303), in postfix over leaf
 * columns. Converted per file as ParquetFilterUtils.toParquetFilter does and evaluated per row group
 * with parquet-mr's StatisticsFilter over the footer statistics (ParquetFileReader.java:111-132). */
typedef struct dk_rg_filter {
  int32_t n_cols;                  /* leaf columns, dotted paths in pool (any number)               */
  const int32_t* col_off;          /* [n_cols]                                                      */
  const int32_t* col_len;
  int32_t n_ops;                   /* any number                                                    */
  const int32_t* op;               /* [n_ops]: 0 COL(arg) 1 LIT(arg = type: 0 long 1 integer 2 short 3 byte
                                      4 date 5 float 6 double 7 boolean 8 string 9 other; lit = value,
                                      float / double as the bits of a double, string: pool offset |
                                      length << 32) 2 NULL 3 = 4 < 5 <= 6 > 7 >= 8 AND 9 OR 10 NOT
                                      11 IS_NULL 12 IS_NOT_NULL 13 UNSUPPORTED (an unconvertible node) */
  const int32_t* arg;
  const int64_t* lit;
  const char* pool;
  int64_t pool_len;
} dk_rg_filter;
/* keep[g] = 0 for the row groups of `path` the filter proves empty (filter NULL: keep all). */
int  dk_parquet_prune_row_groups(const char* path, const dk_rg_filter* filter, uint8_t* keep, int32_t cap,
                                 int32_t* n);
int64_t dk_parquet_row_offset(dk_parquet* p, int32_t file);   /* file row of the first selected row */
int  dk_parquet_decode(dk_parquet* p);                 /* async on the engine stream */
int  dk_parquet_sync(dk_parquet* p);
int64_t dk_parquet_num_rows(dk_parquet* p, int32_t file);
/* One decoded column in library-owned pinned host memory (valid until the next decode or close).
 * The first request for a leaf queues that leaf's D2H copy for this file and every later file of
 * the set (a scan consumer reads the same leaves of every batch); each request waits for its file. */
int  dk_parquet_column(dk_parquet* p, int32_t file, int32_t leaf, dk_column* out);
/* Snapshot-load P&M pass (LogReplay.loadTableProtocolAndMetadata, internal/replay/LogReplay.java:
 * 220-314, which takes the first row whose protocol / metaData is non-null): index of the first row
 * of a decoded column with definition level >= min_def, found on the device; -1 when none. */
int  dk_parquet_first_row(dk_parquet* p, int32_t file, int32_t leaf, int32_t min_def, int64_t* row);
/* D2H copy of rows [row0, row0+n) of one decoded column; row_offs / offs rebased to the slice
 * (valid until the next call for the same column or close). */
int  dk_parquet_column_rows(dk_parquet* p, int32_t file, int32_t leaf, int64_t row0, int64_t n, dk_column* out);
/* wall ms of the open's phases: host read (+ H2D issue), page metadata, prepare passes (sizing);
 * then inside prepare: H2D completion + page headers, host page tables, device sizing passes, host
 * tile tables + output arena */
int  dk_parquet_open_ms(dk_parquet* p, double out[7]);
/* bytes read (projected column chunks) and written (decoded buffers) per decode, for roofline */
int  dk_parquet_traffic(dk_parquet* p, int64_t* bytes_read, int64_t* bytes_written);
/* algorithmic bytes one launch of a decode kernel must move ("k_string_copy", "k_tile_decode") */
int  dk_parquet_kernel_traffic(dk_parquet* p, const char* kernel, int64_t* bytes_read, int64_t* bytes_written);
void dk_parquet_close(dk_parquet* p);

/* ---- Streaming ParquetHandler.readParquetFiles (ParquetHandler.java:64-68) ----
 * The files are decoded on the GPU when the reader opens (on the reader's own HIP stream: one engine
 * may serve several threads, each reader is single-threaded like a Kernel iterator). dk_reader_next
 * then yields batches of at most dk_config.parquet_batch_size rows, file by file in input order and
 * rows in file order, never spanning two files (ParquetFileReader.java:54-147); *out = NULL once
 * exhausted. A batch stays valid until dk_batch_release, also after dk_reader_close, and closing a
 * reader before it is exhausted is safe (ScanImpl.java:376-392).
 *
 * Batch layout (pinned host memory, Arrow-like). Row-indexed arrays -- row_def, row_offs, row_index --
 * start at the batch's first row. Value-indexed arrays -- validity, entry_def, fixed, offs -- are
 * shared by the batches of one transfer window: value i of the batch is at index value_offset + i,
 * and a repeated leaf's row r holds values [row_offs[r], row_offs[r + 1]) (absolute indices, as the
 * Arrow C data interface's offset). Byte array value v = chars[offs[v], offs[v + 1]). */
#define DK_MAX_LEAF_DEPTH 8
typedef struct dk_read_options {
  /* parquet.field.id of each dotted component of each leaf (n_leaves x DK_MAX_LEAF_DEPTH, -1 = none),
   * or NULL: a component resolves by field id, then exact name, then case-insensitive name
   * (ParquetSchemaUtils.findSubFieldType, :92-119); duplicate ids in a struct group fail (:122-138) */
  const int32_t* field_ids;
  /* optional row-group predicate (best effort, as parquet-mr's StatisticsFilter, ParquetFileReader.java:
   * 111-132): row groups it proves empty are not read; NULL = read everything */
  const dk_rg_filter* predicate;
  int32_t row_index;             /* 1: batches carry the file row index of every row (the
                                    _metadata.row_index metadata column, ParquetFileReader.java:57-59,96) */
  int32_t window_rows;           /* rows per host transfer window (0: about 1M, rounded to batches) */
} dk_read_options;

typedef struct dk_batch_column {
  int32_t present;               /* 0: the file lacks the leaf -> every value null (NonExistentColumnReader) */
  int32_t phys, width, max_def, max_rep, rep_def;
  int64_t n_values;              /* values of the batch: rows, or entries of a repeated leaf */
  int64_t value_offset;          /* index of the batch's first value in the value-indexed arrays */
  const uint8_t* row_def;        /* definition level per row (null ancestors: def below their level) */
  const int32_t* row_offs;       /* repeated leaf: n_rows + 1 entry offsets (absolute value indices) */
  const uint8_t* validity;       /* bit v (LSB first) = value v is non-null (def == max_def) */
  const uint8_t* entry_def;      /* repeated leaf: definition level per entry */
  const uint8_t* fixed;          /* fixed-width values, value v at fixed + v * width (0 where null) */
  const int32_t* offs;           /* byte arrays: value offsets into chars */
  const uint8_t* chars;
} dk_batch_column;

typedef struct dk_batch {
  int32_t file;                  /* index of the input file the rows come from */
  int32_t n_cols;                /* == n_leaves, in the requested order */
  int64_t n_rows;
  const dk_batch_column* cols;
  const int64_t* row_index;      /* per row, when dk_read_options.row_index; else NULL */
} dk_batch;

int  dk_reader_open(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                    int32_t n_leaves, const dk_read_options* opt, dk_reader** out);
int  dk_reader_next(dk_reader* r, dk_batch** out);
int64_t dk_reader_num_rows(dk_reader* r, int32_t file);   /* rows the reader yields for a file */
void dk_batch_release(dk_batch* b);
void dk_reader_close(dk_reader* r);

/* ---- Deletion vectors (Scan.transformPhysicalData's DV load, Scan.java:176-199) ----
 * Each descriptor is a scan file's add.deletionVector. A DV with cardinality 0 is empty and not read;
 * "u" DVs live at <table root>/<random prefix>/deletion_vector_<uuid>.bin, "p" DVs at their absolute
 * URI. The stored bytes are checked as DeletionVectorStoredBitmap.loadFromStream does (4-byte size,
 * CRC-32) and decoded as RoaringBitmapArray.readFrom (native or portable magic, portable roaring
 * containers: org.roaringbitmap 0.9.25) into a dense deleted-row bitmap per DV on the GPU.
 * Error messages follow the reference ("DV size mismatch", "DV checksum mismatch", "Couldn't load dv:
 * ..."); an inline ("i") DV fails as it does in the reference, whose isInline() compares the storage
 * type by reference (DeletionVectorDescriptor.java:176-178, :210-215). */
typedef struct dk_dv_descriptor {
  const char* storage_type;      /* "u", "p" or "i" */
  const char* path_or_inline;
  int32_t has_offset, offset;
  int32_t size_in_bytes;
  int64_t cardinality;
} dk_dv_descriptor;
/* table_root: the scan state's table root (a Hadoop path URI such as file:/data/t) */
int  dk_dv_load(dk_engine* e, const char* table_root, const dk_dv_descriptor* dvs, int32_t n, dk_dv_set** out);
int64_t dk_dv_num_bits(dk_dv_set* s, int32_t i);     /* largest deleted row + 1 (0: empty DV) */
/* the packed bitmap (LSB first; bit r = row r deleted), ceil(num_bits / 8) bytes */
int  dk_dv_bitmap(dk_dv_set* s, int32_t i, void* dst, int64_t nbytes, int32_t dst_on_device);
/* SelectionColumnVector: sel[k] = 1 iff row_index[k] is not deleted by DV i */
int  dk_dv_selection(dk_dv_set* s, int32_t i, const int64_t* row_index, int64_t n, uint8_t* sel);
void dk_dv_free(dk_dv_set* s);

/* ---- Commit tail (host JSON parse, newest commit first, batches of json_batch_size lines) ----
 * One row per JSON line, in replay order, with the add/remove read schema. Columns are addressed
 * by the same dotted leaf names as the checkpoint (add.*, remove.path, remove.deletionVector.*). */
int  dk_json_tail_parse(dk_engine* e, const char* const* commit_paths, const int64_t* versions,
                        int32_t n_files, int32_t with_stats, dk_json_tail** out);
int64_t dk_json_tail_rows(dk_json_tail* t);
/* The same over the commit tail followed by n_checkpoint_files JSON-format checkpoint parts (a V2
 * checkpoint's JSON manifest, read by ActionsIterator.getActionsIterFromSinglePartOrV2Checkpoint
 * through JsonHandler.readJsonFiles, ActionsIterator.java:175-248): their add rows are checkpoint
 * adds (isFromCheckpoint), their removes are ignored. Rows [dk_json_tail_checkpoint_row0(t), rows)
 * are those parts' rows. */
int  dk_json_tail_parse_parts(dk_engine* e, const char* const* paths, const int64_t* versions, int32_t n_files,
                              int32_t n_checkpoint_files, int32_t with_stats, dk_json_tail** out);
int64_t dk_json_tail_checkpoint_row0(dk_json_tail* t);
/* Snapshot-load P&M scan of commit files given newest first (LogReplay.loadTableProtocolAndMetadata,
 * internal/replay/LogReplay.java:220-314): per file, the line index and byte range of the first line
 * with a non-null top-level "protocol" / "metaData" (-1: none). Files are read 16 at a time on host
 * threads; the scan stops after the block in which both were seen (*n_scanned = files scanned). */
/* One commit line's protocol (which = 0) or metaData (which = 1) action, bytes [off, off + len) of
 * `path`, decoded with DefaultJsonRow's rules for Protocol / Metadata FULL_SCHEMA and re-serialised
 * as JSON with exactly the schema's fields. Returns 2 (with *out_len set) when cap is too small. */
int  dk_json_pm_decode(const char* path, int64_t off, int64_t len, int32_t which, char* out, int64_t cap,
                       int64_t* out_len);
int  dk_log_pm_scan(const char* const* paths, int32_t n, int64_t* p_line, int64_t* p_off, int64_t* p_len,
                    int64_t* m_line, int64_t* m_off, int64_t* m_len, int32_t* n_scanned);
int  dk_json_tail_column(dk_json_tail* t, const char* leaf, dk_column* out);
void dk_json_tail_free(dk_json_tail* t);

/* ---- Predicates: ExpressionHandler.getPredicateEvaluator(inputSchema, predicate) for the two
 * predicates a scan evaluates (KA/engine/ExpressionHandler.java:58), compiled once on the host into a
 * device program (no size limits: programs live in device memory, paths / fields go through tables).
 *  dk_skip_compile: the data-skipping predicate DataSkippingUtils.constructDataSkippingFilter built
 *    (KA/internal/skipping/DataSkippingUtils.java:156-456) over the pruned stats schema, bare or wrapped
 *    as ScanImpl wraps it, =(COALESCE(skip, true), ALWAYS_TRUE) (KA/internal/ScanImpl.java:304-352).
 *    A row stays selected iff COALESCE(skip(stats), true); null / absent stats keep the row.
 *  dk_part_compile: the partition predicate rewritten over the scan-file schema
 *    (PartitionUtils.rewritePartitionPredicateOnScanFileSchema, KA/internal/util/PartitionUtils.java:
 *    324-358: element_at(add.partitionValues, '<physical name>'), inside partition_value(.., '<type>')
 *    unless the column is a string) as ScanImpl.applyPartitionPruning passes it (:245-294). A row stays
 *    selected iff the predicate is TRUE.
 * Both take JSON text (INTEGRATION.md "Predicate JSON"):
 *   {"col": ["minValues", "id"]}
 *   {"lit": <value>, "type": "<Kernel type>"}    null value = null literal; long / integer / short / byte,
 *       date (epoch days), timestamp / timestamp_ntz (micros) as JSON integers; string as a JSON string;
 *       decimal(p,s) as its BigDecimal text; float / double as "0x<IEEE bits>"; boolean as true / false;
 *       binary as hex digits
 *   {"op": "<NAME>", "args": [...]}              AND OR NOT = < <= > >= IS NOT DISTINCT FROM IS_NULL
 *       IS_NOT_NULL COALESCE ALWAYS_TRUE ALWAYS_FALSE TIMEADD ELEMENT_AT, and
 *       {"op": "PARTITION_VALUE", "type": "<Kernel type>", "args": [...]}
 * and the stats schema is Kernel StructType JSON. Status 3: the reference's evaluator throws for this
 * predicate ("Unsupported expression: ...", DefaultExpressionEvaluator.transformBinaryComparator). */
typedef struct dk_program dk_program;
#define DK_PROGRAM_SKIPPING 0
#define DK_PROGRAM_PARTITION 1
int  dk_skip_compile(const char* stats_schema_json, const char* predicate_json, dk_program** out);
int  dk_part_compile(const char* predicate_json, dk_program** out);
/* JSON description: {"kind", "stack", "paths": [{"type", "path": [...]}] | "fields": [{"type", "name"}],
 * "ops": [[op, arg, lit], ...], "pool": hex}; returns its length (writes at most cap - 1 bytes + NUL).
 * The paths are what a caller projects as the typed add.stats_parsed.<path> leaves. */
int64_t dk_program_describe(const dk_program* p, char* buf, int64_t cap);
void dk_program_free(dk_program* p);

/* ---- Engine plugin point 1 beyond the ParquetHandler: the data-skipping hooks a
 * stock ScanImpl calls through the Engine (KA/internal/ScanImpl.java:304-352):
 *   JsonHandler.parseJson(statsVector, prunedStatsSchema, selection)   (KA/engine/JsonHandler.java:68-71)
 *     -> dk_json_parse: the stats strings (n rows: offs[n + 1] into chars, isnull / selection one byte
 *        per row or NULL; host memory, or device memory when on_device -- a GPU-decoded add.stats
 *        column) parsed on the GPU with DefaultJsonRow's rules (KD/internal/data/DefaultJsonRow.java:
 *        136-357) for every leaf of the output schema (Kernel StructType JSON; any number of leaves of
 *        the stats types long, integer, short, byte, date, timestamp, timestamp_ntz, string, decimal,
 *        float, double). Unselected and null rows are all-null rows (DefaultJsonHandler.java:60-76); a
 *        row that does not decode fails the call.
 *     -> dk_parsed_column_get: one leaf as a typed column with validity (host memory, valid until
 *        dk_parsed_free), leaves in schema order (dk_parsed_leaf_path: the leaf's names as JSON).
 *   ExpressionHandler.getPredicateEvaluator(prunedStatsSchema, COALESCE(skip, true)).eval(parsed, sel)
 *                                                                       (KA/engine/ExpressionHandler.java:58)
 *     -> dk_parsed_eval: a dk_skip_compile program over the parsed rows on the GPU, ANDed into the
 *        selection in place (DefaultPredicateEvaluator.java:42-72); its stats paths must be leaves of
 *        the parsed schema. */
typedef struct dk_parsed dk_parsed;
typedef struct dk_parsed_column {
  int32_t type;            /* 0 long, 1 integer, 2 short, 3 byte, 4 date, 5 string, 6 timestamp, 7 decimal,
                              8 timestamp_ntz, 9 float, 10 double                                    */
  int64_t n;
  const uint8_t* validity; /* one byte per row: 1 = non-null                                         */
  const int64_t* values;   /* integral / date (epoch days) / timestamp(_ntz) (micros); float / double:
                              IEEE bits; decimal: the low 64 bits of the unscaled value                */
  const int64_t* values_hi;/* decimal: the high 64 bits of the (two's complement) unscaled value     */
  const int32_t* scale;    /* decimal: BigDecimal scale per row                                      */
  const uint8_t* wide;     /* decimal: 1 where the unscaled value needs more than 127 bits (use the text) */
  const int32_t* offs;     /* string (unescaped UTF-8) / decimal (the number token): n + 1 offsets     */
  const uint8_t* chars;
} dk_parsed_column;
int  dk_json_parse(dk_engine* e, const char* schema_json, int64_t n, const int64_t* offs, const uint8_t* chars,
                   const uint8_t* isnull, const uint8_t* selection, int32_t on_device, dk_parsed** out);
int32_t dk_parsed_num_leaves(const dk_parsed* ps);
int64_t dk_parsed_leaf_path(const dk_parsed* ps, int32_t leaf, char* buf, int64_t cap);
int  dk_parsed_column_get(dk_parsed* ps, int32_t leaf, dk_parsed_column* out);
int  dk_parsed_eval(dk_parsed* ps, const dk_program* prog, uint8_t* selection);
void dk_parsed_free(dk_parsed* ps);

/* ---- Replay: reconcile the tail and the checkpoint files on the GPU ----
 * ckpt may be NULL (no checkpoint). Checkpoint files are given in replay order (multi-part:
 * descending part number, LogSegment.java:171-177). */
int  dk_replay_create(dk_engine* e, dk_json_tail* tail, dk_parquet* ckpt, dk_replay** out);
/* The same in two halves: dk_replay_create(e, tail, NULL, &r) builds the commit-tail half (action
 * table, key table inputs) -- e.g. while the checkpoint files are still being opened -- and this
 * attaches the checkpoint afterwards (once per replay). */
int  dk_replay_attach_checkpoint(dk_replay* r, dk_parquet* ckpt);
/* install (prog != NULL, a dk_skip_compile program; copied) or clear the data-skipping program applied
 * after reconciliation; the tail must have been parsed with stats and the checkpoint projection must
 * include add.stats */
int  dk_replay_set_skipping(dk_replay* r, const dk_program* prog);
/* Checkpoint files whose skipping reads the typed add.stats_parsed columns instead of the add.stats
 * JSON: those where every program path is an integral / date stat whose leaf
 * add.stats_parsed.<path> was projected (INT64 for long, INT32 otherwise). The predicate is the same;
 * the columns are Spark's from_json(stats) (JsonHandler.parseJson hook), so the
 * selection equals the JSON path's. DK_NO_STATS_PARSED=1 turns it off. */
int  dk_replay_stats_parsed_files(dk_replay* r);
/* install (prog != NULL, a dk_part_compile program; copied) or clear the partition-pruning program,
 * applied before data skipping; the checkpoint projection must include add.partitionValues */
int  dk_replay_set_partition_filter(dk_replay* r, const dk_program* prog);
int  dk_replay_run(dk_replay* r);                      /* async: key build, probe, decode */
/* The same run with the checkpoint files in n_groups groups, each decoded, probed, filtered and its
 * selections copied to host memory in turn, so that ScanImpl.getScanFiles' batches can be handed
 * out while later groups still decode (CloseableIterator<FilteredColumnarBatch>.next,
 * ScanImpl.java:120-186 / ActiveAddFilesIterator.java:146-275): dk_replay_wait_file(r, -1) before
 * the commit-tail selection, dk_replay_wait_file(r, f) before file f's selection and columns
 * (dk_replay_ckpt_selection_host, dk_parquet_column), dk_replay_sync at the end for the counters. A
 * device error seen by a wait is reported after the whole run, as dk_replay_sync reports it. */
int  dk_replay_run_grouped(dk_replay* r, int32_t n_groups);
int  dk_replay_wait_file(dk_replay* r, int32_t file);
/* Grouped runs: also copy projected leaf `leaf` of each group's files to host memory as soon as the
 * group is decoded (the pinned mirror dk_parquet_column hands out), instead of at the consumer's
 * first touch -- for the columns every consumer of the scan files reads (Scan.getScanFiles' callers
 * read add.size for split planning: BenchmarkParallelCheckpointReading.java:124-135). Call after the
 * checkpoint is attached, before dk_replay_run_grouped. */
int  dk_replay_prefetch_leaf(dk_replay* r, const char* leaf);
int  dk_replay_sync(dk_replay* r);
/* counters: addFilesSeen, addFilesSeenFromDeltaFiles, activeAddFiles, duplicateAddFiles,
 * removeFilesSeenFromDeltaFiles */
int  dk_replay_counters(dk_replay* r, int64_t out[5]);
/* the same counters split into the commit-tail part and the checkpoint part (the part a shard of
 * the checkpoint contributes; ranks sum checkpoint parts and take the tail part once) */
int  dk_replay_counters_split(dk_replay* r, int64_t tail[5], int64_t ckpt[5]);
int  dk_replay_json_selection(dk_replay* r, uint8_t* out, int64_t n);
int  dk_replay_ckpt_selection(dk_replay* r, int32_t file, uint8_t* out, int64_t n);
/* zero-copy: *out = checkpoint file `file`'s selection, one byte per row, in library-owned pinned
 * memory valid until the next dk_replay_run or dk_replay_free (the first call after a sync moves
 * every file's selection to the host at once) */
int  dk_replay_ckpt_selection_host(dk_replay* r, int32_t file, const uint8_t** out);
/* the same selection packed into bits (LSB first) -- ceil(n / 8) bytes at dst, a device pointer
 * (the multi-GPU merge hands it to RCCL) when dst_on_device, else host memory */
int  dk_replay_ckpt_selection_bits(dk_replay* r, int32_t file, void* dst, int64_t n, int32_t dst_on_device);
/* every checkpoint file's packed selection at dst + offsets[file] (one synchronisation for all);
 * the multi-GPU exchange writes its collective buffer with it */
int  dk_replay_ckpt_selection_bits_all(dk_replay* r, void* dst, const int64_t* offsets, int32_t dst_on_device);
/* per-kernel average device time (us) over recorded runs (DK_FLAG_TIMING); names via index */
/* hash(path)-owner exchange (multi-GPU "alltoall" mode; the repartition of actions by path that
 * delta-spark's Snapshot.scala:478-483 performs). After dk_replay_set_exchange(r, world, rank),
 * dk_replay_run stops after the decode and routing counts; the caller then drives one exchange:
 *   dk_replay_exchange_counts   records this rank sends to each rank (int64[world])
 *   dk_replay_exchange_pack     the 8-byte records {path hash} into `send` (device, owner-major)
 *   (all-to-all of the records)
 *   dk_replay_exchange_filter   owner side: one byte per received record (1: some commit-tail key
 *                               of this rank's share has that path hash), into `flags` (device)
 *   (reverse all-to-all of the flags, in the order the records were sent)
 *   dk_replay_exchange_finish   rows answered 0 are selected; the rest take the exact key probe
 * then dk_replay_sync as usual. Every call orders itself on the replay's stream and returns with
 * the stream drained, so the caller's collectives may touch the buffers. world <= 64. */
int  dk_replay_set_exchange(dk_replay* r, int32_t world, int32_t rank);
int  dk_replay_exchange_counts(dk_replay* r, int64_t* counts);
int  dk_replay_exchange_pack(dk_replay* r, uint64_t* send);
int  dk_replay_exchange_filter(dk_replay* r, const uint64_t* recv, int64_t n, uint8_t* flags);
int  dk_replay_exchange_finish(dk_replay* r, const uint8_t* back);

/* Owner-partitioned reconciliation (multi-GPU "owner" mode): delta-spark's
 * repartition of ALL actions by path with one resolver per key (spark/src/main/scala/org/apache/
 * spark/sql/delta/Snapshot.scala:476-485) over ActiveAddFilesIterator's rules
 * (KA/internal/replay/ActiveAddFilesIterator.java:164-234). Each rank parses only its share of the
 * commit files and decodes only its share of the checkpoint; the key (URI(path), dvUniqueId) with
 * hash h is owned by rank h mod world. Key records are dk OwnerKeyRec (32 bytes: u64 h; i32 kind,
 * step, row, key_len, canon_len, src) with their canonical key bytes in a byte buffer alongside, in
 * the same order; every buffer below is device memory (the caller's RCCL all-to-alls move them).
 *   dk_json_tail_file_steps     batches per parsed commit file (the caller all-reduces them)
 *   dk_json_tail_rebase_steps   the files' first batch in the GLOBAL replay order (before replay_create)
 *   dk_replay_set_owner         owner mode for this replay (world <= 64)
 *   dk_replay_owner_begin       a new run: counters and error state cleared
 *   dk_replay_owner_tail_counts records / key bytes this rank sends to each rank (int64[world] each)
 *   dk_replay_owner_tail_pack   the records and key bytes, owner-major
 *   dk_replay_owner_tail_resolve owner: the key table of the records received (R2-R5 selection of
 *                               each, commit-tail counters), one answer byte per record (1: the add
 *                               is selected), *flags = E_COLLISION (4) on a 64-bit hash collision
 *   dk_replay_owner_reseed      after a collision on any rank: next seed, repeat from tail_counts
 *   dk_replay_owner_tail_finish origin: the answers (in send order) -> this rank's tail selection
 *   dk_replay_run               decode + key hash of every checkpoint row + routing counts
 *   dk_replay_owner_ckpt_counts / _pack   8-byte records {h} per rank, owner-major
 *   dk_replay_owner_ckpt_lookup owner: 1 = a tail key has exactly this hash, 0 = none
 *   dk_replay_owner_ckpt_apply  origin: rows answered 0 are selected, the rest are candidates
 *   dk_replay_owner_cand_counts / _pack   the candidates' key records + canonical key bytes
 *   dk_replay_owner_cand_verify owner, byte-exact: 0 = no tail key equals it (selected),
 *                               1 = a JSON add (duplicate), 2 = a tombstone only
 *   dk_replay_owner_cand_finish origin: the final selection, counters, then partition / skipping
 * then dk_replay_sync. The five counters are split: commit-tail counters of the actions this rank
 * owns, checkpoint counters of the rows this rank decoded; their sums over the ranks are the
 * reference's. */
int  dk_json_tail_file_steps(dk_json_tail* t, int32_t* steps);
int  dk_json_tail_file_row0(dk_json_tail* t, int64_t* row0);     /* first row per file + total (n_files + 1) */
int  dk_json_tail_rebase_steps(dk_json_tail* t, const int32_t* step0);
int  dk_replay_set_owner(dk_replay* r, int32_t world, int32_t rank);
int  dk_replay_owner_begin(dk_replay* r);
int  dk_replay_owner_tail_counts(dk_replay* r, int64_t* recs, int64_t* bytes);
int  dk_replay_owner_tail_pack(dk_replay* r, void* recs, void* keys);
int  dk_replay_owner_tail_resolve(dk_replay* r, const void* recs, int64_t n, const void* keys, int64_t nbytes,
                                  uint8_t* answers, int32_t* flags);
int  dk_replay_owner_reseed(dk_replay* r);
int  dk_replay_owner_tail_finish(dk_replay* r, const uint8_t* back);
int  dk_replay_owner_ckpt_counts(dk_replay* r, int64_t* counts);
int  dk_replay_owner_ckpt_pack(dk_replay* r, uint64_t* send);
int  dk_replay_owner_ckpt_lookup(dk_replay* r, const uint64_t* recv, int64_t n, uint8_t* flags);
int  dk_replay_owner_ckpt_apply(dk_replay* r, const uint8_t* back);
int  dk_replay_owner_cand_counts(dk_replay* r, int64_t* recs, int64_t* bytes);
int  dk_replay_owner_cand_pack(dk_replay* r, void* recs, void* keys);
int  dk_replay_owner_cand_verify(dk_replay* r, const void* recs, int64_t n, const void* keys, int64_t nbytes,
                                 uint8_t* answers);
int  dk_replay_owner_cand_finish(dk_replay* r, const uint8_t* back);

/* ---- Collectives of the multi-GPU owner exchange, owned by the library (delta_amd/csrc/dk_comm.cpp).
 * Kernel's Engine has no collective hook (KA/engine/Engine.java:30-64), so a JVM GpuScan cannot bring
 * one: rank 0 makes an RCCL unique id (dk_comm_unique_id), the host hands its 128 bytes to every rank by
 * any means (the JVM's own RPC, a shared file), each rank creates its communicator over xGMI
 * (dk_comm_create) and runs the whole owner protocol of a scan in ONE call, dk_replay_owner_run (the
 * repartition by path of spark/src/main/scala/org/apache/spark/sql/delta/Snapshot.scala:476-485, the
 * 14 dk_replay_owner_* steps above with their collectives: 11 per run). Every step carries a vote: a
 * rank whose local part fails returns its error, every peer returns DK_STATUS_PEER at the same step,
 * and no rank waits in a collective for a failed one. A rank that fails after the commit-tail
 * batch-count all-reduce but before its dk_replay_owner_run (e.g. its checkpoint open) calls
 * dk_comm_abort instead, which answers the run's first vote.
 * Other transports: dk_comm_create_callbacks (the caller's all-to-all / all-reduce over host memory:
 * tests over gloo, a host with its own transport) and dk_comm_create_local (`world` communicators of
 * one process, one thread per rank: one-GPU rehearsals). */
typedef struct dk_comm dk_comm;
#define DK_COMM_ID_BYTES 128
#define DK_STATUS_PEER 6            /* another rank of the collective failed at this step */
typedef struct dk_comm_callbacks {
  void* user;
  /* all-to-all of byte runs in host memory: send holds send_bytes[p] bytes for each rank p in rank
   * order; recv receives recv_bytes[p] bytes from each rank p in rank order. 0 = OK. */
  int (*alltoallv)(void* user, const void* send, const int64_t* send_bytes, void* recv, const int64_t* recv_bytes);
  /* element-wise reduction of vals[0..n) over the ranks, in place: op 0 = sum, 1 = max. 0 = OK. */
  int (*allreduce_i64)(void* user, int64_t* vals, int32_t n, int32_t op);
} dk_comm_callbacks;
int  dk_comm_unique_id(uint8_t id[DK_COMM_ID_BYTES]);
int  dk_comm_create(const uint8_t id[DK_COMM_ID_BYTES], int32_t world, int32_t rank, int32_t device, dk_comm** out);
int  dk_comm_create_callbacks(const dk_comm_callbacks* cb, int32_t world, int32_t rank, dk_comm** out);
int  dk_comm_create_local(int32_t world, int32_t on_device, dk_comm** comms /* [world] */);
int32_t dk_comm_world(const dk_comm* c);
int32_t dk_comm_rank(const dk_comm* c);
/* host values; op 0 = sum, 1 = max (the commit tail's global batch counts: dk_json_tail_file_steps) */
int  dk_comm_allreduce_i64(dk_comm* c, int64_t* vals, int32_t n, int32_t op);
int  dk_comm_alltoallv(dk_comm* c, const void* send, const int64_t* send_bytes, void* recv, const int64_t* recv_bytes,
                       int32_t on_device);
int  dk_comm_abort(dk_comm* c);
/* the last owner run (ms): [0] commit-tail exchange, [1] decode + row hashes, [2] row and candidate
 * exchanges, [3] total (wall times); [4..6] the local steps' share of [0..2]; [7] time inside
 * collectives; the payload bytes this rank sent to its peers and the number of collectives */
int  dk_comm_last_run(const dk_comm* c, double ms[8], int64_t* bytes_sent, int64_t* collectives);
/* the last owner run's local steps (ms), in dk_owner_side member order: begin, tail_counts, tail_pack,
 * tail_resolve, reseed, tail_finish, run, ckpt_counts, ckpt_pack, ckpt_lookup, ckpt_apply, cand_counts,
 * cand_pack, cand_verify, cand_finish */
int  dk_comm_last_steps(const dk_comm* c, double ms[16]);
void dk_comm_destroy(dk_comm* c);
/* dk_replay_set_owner(r, world, rank) first (world = dk_comm_world), the commit tail rebased with the
 * all-reduced batch counts; then this call; then dk_replay_sync as usual. */
int  dk_replay_owner_run(dk_replay* r, dk_comm* c);
/* The same protocol over a caller's stand-in for the device side (tests of the protocol without a GPU;
 * each member mirrors the dk_replay_owner_* call of the same name; buffers in host memory unless
 * device_buffers). */
typedef struct dk_owner_side {
  void* user;
  int32_t device_buffers;
  int (*begin)(void* user);
  int (*tail_counts)(void* user, int64_t* recs, int64_t* bytes);
  int (*tail_pack)(void* user, void* recs, void* keys);
  int (*tail_resolve)(void* user, const void* recs, int64_t n, const void* keys, int64_t nbytes, uint8_t* answers,
                      int32_t* flags);
  int (*reseed)(void* user);
  int (*tail_finish)(void* user, const uint8_t* back);
  int (*run)(void* user);
  int (*ckpt_counts)(void* user, int64_t* counts);
  int (*ckpt_pack)(void* user, uint64_t* send);
  int (*ckpt_lookup)(void* user, const uint64_t* recv, int64_t n, uint8_t* flags);
  int (*ckpt_apply)(void* user, const uint8_t* back);
  int (*cand_counts)(void* user, int64_t* recs, int64_t* bytes);
  int (*cand_pack)(void* user, void* recs, void* keys);
  int (*cand_verify)(void* user, const void* recs, int64_t n, const void* keys, int64_t nbytes, uint8_t* answers);
  int (*cand_finish)(void* user, const uint8_t* back);
} dk_owner_side;
int  dk_owner_protocol_run(const dk_owner_side* side, dk_comm* c);

/* Checkpoint Parquet writer (Table.checkpoint's ParquetHandler.writeParquetFileAtomically,
 * DefaultParquetHandler.java:110-163): CHECKPOINT_SCHEMA (SingleAction.java:30-37), encoded on the
 * device. Rows come in iterator order as row groups: action rows built by the caller as JSON lines
 * (one {"<action>": {...}} object per line, decoded with DefaultJsonRow's rules), and runs of rows
 * of the replay's checkpoint file whose surviving adds are gathered on the device from the decoded
 * columns by the replay's selection. codec: 1 SNAPPY (the reference's default), 0 UNCOMPRESSED.
 * close writes the footer and frees the writer. */
typedef struct dk_ckpt_writer dk_ckpt_writer;
int  dk_ckpt_writer_open(dk_engine* e, const char* path, int32_t codec, dk_ckpt_writer** out);
int  dk_ckpt_writer_add_json(dk_ckpt_writer* w, const char* lines, int64_t len);
int  dk_ckpt_writer_add_checkpoint_adds(dk_ckpt_writer* w, dk_replay* r, int32_t file, int64_t row0, int64_t row1,
                                        int64_t* n_rows);
int  dk_ckpt_writer_close(dk_ckpt_writer* w, int64_t* n_rows, int64_t* file_size);
int  dk_replay_kernel_stats(dk_replay* r, int32_t i, const char** name, double* avg_us, int64_t* count);
void dk_replay_free(dk_replay* r);

#ifdef __cplusplus
}
#endif
#endif
