/*
 * rfx.h — C ABI of the MI355X-native embedding-index + top-k retrieval path.
 *
 * This library replaces the arithmetic that the reference (Sapphire-Bridge/rag-foundation)
 * delegates to Gemini File Search behind its Retriever/LLM adapter:
 *   - index write  : GeminiRag.upload_file          backend/app/services/gemini_rag.py:307-352
 *                    (mock: MockGeminiRag.upload_file gemini_rag.py:614-629), called from the
 *                    ingestion worker's index step   backend/app/services/ingestion.py:45-52,225
 *   - retrieval    : GeminiRag.ask_stream / ask     gemini_rag.py:481-551 (FileSearch tool
 *                    gemini_rag.py:463-469); mock    gemini_rag.py:656-694,704-718
 *   - removal      : delete_document_from_store     gemini_rag.py:392-424 (mock 699-702)
 *                    delete_store                    gemini_rag.py:354-390 (mock 696-697)
 * The reference has no FFI of its own (it is pure Python); these entry points are what its
 * adapter would bind through ctypes (see INTEGRATION.md for the binding stub).
 *
 * Conventions
 *   - Every function returns int: RFX_OK (0) or an RFX_E* code; rfx_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - Pointers named *_d are DEVICE pointers (caller-owned, e.g. torch tensors' data_ptr()),
 *     *_h are HOST pointers.  `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - Only the index storage is owned by the library (behind an rfx_index_t handle).
 *   - Rows are identified by int64 row ids (dense, in insertion order).  Result padding for
 *     k > live rows is (score = -inf, row = -1).
 *   - Ranking rule everywhere: score descending, then row id ascending (deterministic ties).
 */
#ifndef RFX_H
#define RFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define RFX_OK 0
#define RFX_EINVAL 1   /* bad argument / shape (maps to ValueError / RuntimeError)        */
#define RFX_ENOMEM 2   /* device or host allocation failed                                  */
#define RFX_EDEVICE 3  /* HIP runtime error                                                 */
#define RFX_EIO 4      /* file read/write failed                                            */
#define RFX_EBUSY 5    /* transient: device busy / queue timeout (maps to TimeoutError,     */
                       /* i.e. RETRYABLE_EXCEPTIONS, gemini_rag.py:22-27)                   */
#define RFX_EUNSUPPORTED 6 /* configuration not supported by any kernel                     */
#define RFX_ECAPACITY 7 /* the int8 copy (rfx_index_screen) does not fit: free device memory   */
                        /* minus a reserve, or RFX_SCREEN_MAX_BYTES; the index stays exact     */

/* ---- element types of the vector store --------------------------------------------------- */
#define RFX_F32 0
#define RFX_BF16 1
#define RFX_F16 2

typedef uint64_t rfx_index_t;

/* ---- library ------------------------------------------------------------------------------ */
/* Thread-local message describing the last error on this thread ("" if none). */
const char* rfx_last_error(void);
/* ABI version (major*10000 + minor*100 + patch). */
int rfx_version(void);
/* 16-hex sha256 of the sources the library was built from (csrc/Makefile); the Python host
 * recomputes it from the tree and refuses a stale library (rfx/_lib.py). */
const char* rfx_build_id(void);
/* Number of visible HIP devices. */
int rfx_device_count(int* out_n);
/* Bind the calling thread to a device (process-level singleton per device).
 * Replaces the client construction in get_rag_client() gemini_rag.py:721-725. */
int rfx_init(int device);

/* ---- vector store (index) ----------------------------------------------------------------
 * Replaces the File Search store namespace: create_store gemini_rag.py:271-304 / mock 610-612.
 * dim must be a multiple of 64; capacity is rounded up internally and grows on demand. */
int rfx_index_create(int device, int dim, int dtype, int64_t capacity, rfx_index_t* out);
/* Drops the store (delete_store gemini_rag.py:354-390). */
int rfx_index_destroy(rfx_index_t h);
/* A question over several stores (the file-search tool's list of store names, gemini_rag.py:463-469)
 * as ONE index: a read-only view that maps the members' device memory back to back through HIP virtual
 * memory (no copy).  Member m's rows are the view's rows [out_bases[m], out_bases[m] + its rows); the rest
 * of its capacity is NaN (never returned).  The view's own device bytes are the tile records of the int8
 * copy (16 B per 32 rows, copied) and 256 B of stats, when every member holds an int8 copy.  Appends and
 * tombstones of the members show through; rfx_union_refresh copies their tile records again and sets
 * *out_stale when a member moved its memory (growth, a rebuilt or dropped copy) or was destroyed: the
 * caller then destroys the view (rfx_index_destroy) and creates a new one.  RFX_EUNSUPPORTED without
 * virtual memory (RFX_VMM=0): the caller copies instead (rfx/union.py). */
int rfx_union_create(const rfx_index_t* members, int n, void* stream, rfx_index_t* out, int64_t* out_bases);
int rfx_union_refresh(rfx_index_t view, void* stream, int* out_stale);
int rfx_index_info(rfx_index_t h, int* dim, int* dtype, int64_t* rows, int64_t* capacity,
                   int64_t* live_rows);
int rfx_index_reserve(rfx_index_t h, int64_t capacity);
/* Append n already-normalised rows of the index dtype (vector-store write of upload_file,
 * gemini_rag.py:319-327).  src_is_device selects hipMemcpy direction. */
int rfx_index_add(rfx_index_t h, const void* vecs, int64_t n, int src_is_device,
                  int64_t* out_first_row, void* stream);
/* Overwrite rows [row0, row0 + n) of the index (they must exist) with n vectors of the index dtype
 * (device or host memory): the rows are live again (a tombstone on them is lifted) and their tiles of
 * the int8 copy are re-quantised.  Used by the multi-store union view (rfx/union.py) to follow a
 * member's appends in place (the file-search tool's store list, gemini_rag.py:463-469). */
int rfx_index_write(rfx_index_t h, int64_t row0, const void* vecs, int64_t n, int src_is_device, void* stream);
/* Append n synthetic rows generated on the device from the counter-based generator
 * (splitmix64, seed, generator row id) — bench/test corpora, identical to oracle/synth.py.
 * Generator rows are gen_row0 .. gen_row0+n-1 (gen_row0 < 0: continue at the index's row
 * count); a row-sharded corpus passes its global row offset. */
int rfx_index_add_synthetic(rfx_index_t h, uint64_t seed, int64_t gen_row0, int64_t n,
                            int64_t* out_first_row, void* stream);
/* Tombstone rows (delete_document_from_store gemini_rag.py:392-424): the rows' vectors are
 * overwritten with NaN on the device so no scan can ever rank them. */
int rfx_index_tombstone(rfx_index_t h, const int64_t* rows_h, int64_t n, void* stream);
/* Copy rows [row0, row0+n) to dst (device or host). */
int rfx_index_read(rfx_index_t h, int64_t row0, int64_t n, void* dst, int dst_is_device, void* stream);
/* Device pointer to row 0 (row-major [capacity][dim] of dtype).  Valid until next add. */
int rfx_index_data(rfx_index_t h, void** out_ptr);
/* Persist / restore (ingestion deletes the source file, ingestion.py:341, so the index must
 * survive the process).  Format documented in DESIGN.md §Persistence. */
int rfx_index_save(rfx_index_t h, const char* path);
int rfx_index_load(const char* path, int device, rfx_index_t* out);
/* Append-only row file of a store (§8b's rfx_index_open): the ingestion
 * worker appends, the API processes load what was appended since their last look.  Format: a
 * 64-byte header ("RFXROWS1", u32 version 1, u32 dim, u32 dtype, zero pad) then row-major rows
 * of the dtype.  The file holds no row count: the writer publishes the committed count in the
 * store manifest (rfx/store.py) once the rows are durable, and readers never read past it, so a
 * torn tail is never read.  Tombstones travel separately (rfx/store.py tombs.bin).
 * Index row i is file row file_base + i (a row-sharded store: each shard index holds a contiguous
 * range of the file's rows; unsharded: file_base 0).
 *   rfx_rows_append: write the index's rows [row0, rows) to file rows [file_base + row0, ...) (the
 *     file is created, or cut to file_base + row0 rows first — a tail left by a crashed writer is
 *     dropped), fsync.
 *   rfx_rows_sync: append file rows [file_base + rows, file_base + upto) to the index (rows = the
 *     index's current row count); a fresh index + rfx_rows_sync(h, path, n, base) opens a store or
 *     one shard of it. */
int rfx_rows_append(rfx_index_t h, const char* path, int64_t row0, int64_t file_base);
int rfx_rows_sync(rfx_index_t h, const char* path, int64_t upto, int64_t file_base);

/* ---- search ---------------------------------------------------------------------------------
 * Retrieval slice of ask_stream (gemini_rag.py:517-551; mock 673-694): brute-force inner
 * product (cosine on normalised rows) of nq queries against all live rows, top-k per query.
 * queries_d: [nq][dim] in the index dtype.  Outputs [nq][k] (device).  ws_d/ws_bytes: caller
 * workspace of at least rfx_search_workspace_bytes(h, nq, k) bytes.  k <= 64. */
int rfx_search_workspace_bytes(rfx_index_t h, int64_t nq, int k, size_t* out_bytes);
int rfx_search(rfx_index_t h, const void* queries_d, int64_t nq, int k, float* out_scores_d,
               int64_t* out_rows_d, void* ws_d, size_t ws_bytes, void* stream);
/* The two halves of rfx_search, exposed so callers (multi-GPU merge, benchmarks) can time or
 * interleave them: the fused scan writes n_cand candidates per query (sorted partial lists,
 * cand_scores_d/cand_rows_d: [nq][n_cand], rows local int32), then the merge.  rfx_scan_topk
 * uses the front of ws_d for query staging (any ws sized by rfx_search_workspace_bytes). */
int rfx_scan_plan(rfx_index_t h, int64_t nq, int k, int* out_kernel /* 0 VALU, 1 MFMA */,
                  int64_t* out_n_cand /* candidates per query */);
int rfx_scan_topk(rfx_index_t h, const void* queries_d, int64_t nq, int k, float* cand_scores_d,
                  int32_t* cand_rows_d, void* ws_d, size_t ws_bytes, void* stream);
/* Metadata-filtered search.  Replaces the metadata_filter that ask_stream
 * accepts and forwards to Gemini (gemini_rag.py:463-469,517-551, validated at chat.py:295-335;
 * the mock ignores it, gemini_rag.py:673-694).  row_mask_d: device bitmap, bit (r & 31) of
 * word r >> 5 set = row r may be returned, at least (rows + 31) / 32 words (mask_words); one
 * mask for all nq queries.  NULL = no filter (same as rfx_search / rfx_scan_topk).  The scan
 * kernels apply it per tile in their epilogue, so the corpus is still read once. */
int rfx_search_masked(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                      int64_t mask_words, float* out_scores_d, int64_t* out_rows_d, void* ws_d,
                      size_t ws_bytes, void* stream);
int rfx_scan_topk_masked(rfx_index_t h, const void* queries_d, int64_t nq, int k,
                         const uint32_t* row_mask_d, int64_t mask_words, float* cand_scores_d,
                         int32_t* cand_rows_d, void* ws_d, size_t ws_bytes, void* stream);
/* Merge per-query candidate lists into the final top-k.  rows are int32 (rows_are_i64 = 0) or
 * int64 (1); row_offset is added to every returned row (shard base for multi-GPU). */
int rfx_topk_merge(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64,
                   int64_t nq, int64_t n_cand, int k, int64_t row_offset, float* out_scores_d,
                   int64_t* out_rows_d, void* stream);
/* Same, told that the candidates of a query are lists of list_len entries (rfx_scan_topk writes
 * sorted lists of rfx_scan_list_len entries): with list_len >= k the merge only admits scores at
 * or above the max over lists of each list's minimum among its first k entries, a lower bound of
 * the k-th best.  Exact for any list_len, sorted or not; a wrong one only costs time. */
int rfx_scan_list_len(rfx_index_t h, int64_t nq, int k, int* out_list_len);
int rfx_topk_merge_lists(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64,
                         int64_t nq, int64_t n_cand, int list_len, int k, int64_t row_offset,
                         float* out_scores_d, int64_t* out_rows_d, void* stream);
/* Multi-GPU exchange.  A rank's merged top-k as [nq][k] 16-byte records
 * {f32 score, i32 pad, i64 global row} (row_offset added) — the buffer handed to the all-gather —
 * and the merge of the gathered [world][nq][k] records into the final top-k.  Replaces nothing in
 * the reference (it has no collective); the records are rfx/dist.py pack()'s layout. */
int rfx_topk_merge_records(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64,
                           int64_t nq, int64_t n_cand, int list_len, int k, int64_t row_offset,
                           void* out_records_d, void* stream);
int rfx_merge_gathered(const void* records_d, int world, int64_t nq, int k, float* out_scores_d,
                       int64_t* out_rows_d, void* stream);
/* Merge of SORTED lists (rfx_scan_topk's output: each list of list_len entries best first, empty
 * slots (-inf, INT32_MAX) at its tail): a list is read only while its entries can still be admitted,
 * so the lists the admission bound rejects cost one load.  Writes [nq][k] scores + rows, or, when
 * out_records_d is not NULL, [nq][k] records as rfx_topk_merge_records.  Replaces the same step
 * as rfx_topk_merge_lists (the retrieval half of gemini_rag.py:517-551); unsorted input is an
 * error of the caller (use rfx_topk_merge_lists). */
int rfx_topk_merge_sorted(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64,
                          int64_t nq, int64_t n_cand, int list_len, int k, int64_t row_offset,
                          float* out_scores_d, int64_t* out_rows_d, void* out_records_d, void* stream);

/* ---- exact two-pass scan over an int8 copy of the store ------------------------
 * The int8 representation of SURVEY §8a row a3 / §8b (dtype I8), kept BESIDE the bf16/f16 rows so
 * that results stay exact: the same top-k as rfx_search on the rows alone (gemini_rag.py:517-551).
 * rfx_index_screen(h, 1) builds the copy (per 32-row tile: scale amax/127, codes rint(x/scale),
 * a live-row word; + the max row norm and max quantisation-error norm) and keeps it current
 * through add / add_synthetic / rows_sync / tombstone.  Then batched searches (64 < nq, k <= 10,
 * dim 768 or 1024, bf16/f16; the plans of kernels 6 and 8) run: an int8 MFMA screen that keeps
 * every row whose exact score can still reach the query's k-th best (a rigorous Cauchy-Schwarz
 * bound of the quantisation error), an exact re-score of those rows from the stored rows, and —
 * gated on the device, only when a query's survivors may be incomplete — the exact scan for the
 * batch.  mode 0 drops the copy; mode 2 = on, with every batch sent to the exact fallback (tests).
 * Costs dim bytes per row of extra HBM.  EUNSUPPORTED for f32 stores and other dims. */
int rfx_index_screen(rfx_index_t h, int mode, void* stream);
/* Capacity: before allocating, rfx_index_screen checks that the copy (capacity * dim + capacity / 32 * 16
 * bytes) fits in the device's free memory minus RFX_SCREEN_RESERVE_BYTES (default 4 GiB) and under
 * RFX_SCREEN_MAX_BYTES when that is set; otherwise RFX_ECAPACITY and the index stays exact (config 4
 * whole on one GPU: 204.8 GB of f16 rows + 102.4 GB of codes > 288 GB).  When an append grows the
 * index past what the copy can follow, the copy is dropped and the append succeeds (the index is
 * exact again; rfx_index_screen_state reports it): a failed copy never fails a store write
 * (ingestion.py:311-339 would mark the document ERROR while its rows are committed). */
int rfx_index_screen_state(rfx_index_t h, int* out_mode, int64_t* out_bytes, int* out_dropped);
/* Inspection (tests): tiles [tile0, tile0 + ntiles) of the copy to host buffers (any may be NULL):
 * codes [ntiles*32][dim] int8, scales [ntiles] f32, live words [ntiles], stats [3] f32 (max row norm,
 * max quantisation-error norm, max tile scale). */
int rfx_index_screen_read(rfx_index_t h, int64_t tile0, int64_t ntiles, int8_t* codes_h, float* scales_h,
                          uint32_t* live_h, float* stats_h);
/* The kernel rfx_search runs for (nq, k): 0 VALU, 1/2/3/6/8/9 exact MFMA scans, 10 the two-pass scan. */
int rfx_search_plan(rfx_index_t h, int64_t nq, int k, int* out_kernel);
/* After a two-pass search with workspace ws_d (stream-ordered; this call synchronises): per query
 * {kept screen candidates, survivors re-scored (-1 = sent to the fallback)} into diag_h [nq][2], and
 * whether the exact fallback ran for the batch (*fallback_h != 0). */
int rfx_screen_diag(rfx_index_t h, int64_t nq, int k, const void* ws_d, int32_t* diag_h, uint32_t* fallback_h);
/* The score rule every rfx_search* answer follows (one rule for every plan, round 5): a score is fl32 of
 * the f64 sum of the exact products of the stored row and query, the order (score desc, row asc).
 * rfx_rescore_topk applies it in place to a [nq][k] answer assembled from the building blocks
 * (rfx_scan_topk + rfx_topk_merge*, whose scores are the scan's own f32 sums): (scores_d, rows_d), or
 * records_d [nq][k] {f32 score, i32 pad, i64 row} when not NULL; row_offset is subtracted from every row
 * before it is read from this index (the base of a shard's records).  Rows < 0 (padding) stay last.
 * Replaces no reference entry point: the reference's scores come from Gemini (gemini_rag.py:536). */
int rfx_rescore_topk(rfx_index_t h, const void* queries_d, int64_t nq, int k, int64_t row_offset, float* scores_d,
                     int64_t* rows_d, void* records_d, void* stream);
/* rfx_search_masked writing [nq][k] merge records {f32 score, i32 pad, i64 row + row_offset} (the
 * all-gather input of the multi-GPU step) instead of scores and rows: one call per shard, whatever
 * kernel the plan picks (an empty shard writes padding records). */
int rfx_search_records(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                       int64_t mask_words, int64_t row_offset, void* out_records_d, void* ws_d, size_t ws_bytes,
                       void* stream);
/* Benchmark / profiling form of the two above: writes (out_scores_d, out_rows_d) or, when
 * out_records_d is not NULL, records; ev_scan_begin / ev_scan_end (hipEvent_t, may be NULL) are
 * recorded on the stream right before and after the scan kernel (the int8 screen of the two-pass
 * scan, the exact scan, or the one-launch VALU search as a whole). */
/* The search in two stages, for callers that overlap consecutive batches on two streams (the
 * multi-GPU step: the select / fallback / exchange of batch i run beside the screen of batch i + 1):
 * stages bit 1 = the query quantiser + the scan (kernel 10 for a two-pass plan; the whole search for any
 * other plan), bit 2 = the select + the gated exact fallback (two-pass plans; nothing otherwise).  Both
 * calls of one batch pass the same arguments; the caller orders stage 2 after stage 1 (an event).
 * scan_blocks (0 = the plan's 256): the screen's workgroups, so a batch can leave CUs free for the other
 * stream (rfx_stream_create_cu_mask); the workspace of rfx_search_workspace_bytes covers any value. */
int rfx_search_staged(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                      int64_t mask_words, int64_t row_offset, float* out_scores_d, int64_t* out_rows_d,
                      void* out_records_d, void* ws_d, size_t ws_bytes, int stages, int scan_blocks, void* stream);
/* A stream restricted to the CUs whose bits are set (hipExtStreamCreateWithCUMask; n_words 32-bit words,
 * bit i = CU i), on `device`; rfx_stream_destroy releases it. */
int rfx_stream_create_cu_mask(int device, const uint32_t* cu_mask, int n_words, void** out_stream);
int rfx_stream_destroy(void* stream);
int rfx_search_timed(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                     int64_t mask_words, int64_t row_offset, float* out_scores_d, int64_t* out_rows_d,
                     void* out_records_d, void* ws_d, size_t ws_bytes, void* stream, void* ev_scan_begin,
                     void* ev_scan_end);

/* ---- RCCL communicators (SURVEY §8b rfx_init "RCCL comm if n>1", §8e) --------------------------
 * The all-gather of per-shard records runs on RCCL over xGMI from inside the library; the host
 * language only bootstraps the communicator (passes the 128-byte id from rank 0 to the others).
 *   one process per GPU: rank 0 rfx_comm_unique_id -> every rank rfx_comm_init_rank;
 *   one process owning n GPUs (index server): rfx_comm_init_all (ncclCommInitAll).
 * rfx_allgather_records: per local device i, sends_d[i] = [nq][k] records (rfx_topk_merge_records)
 * and recvs_d[i] = [world][nq][k] records, ordered by rank, on streams[i] (arrays of n_local; a
 * rank communicator has n_local = 1).  Then rfx_merge_gathered on the same stream. */
#define RFX_COMM_ID_BYTES 128
typedef uint64_t rfx_comm_t;
int rfx_comm_unique_id(void* out_id /* RFX_COMM_ID_BYTES */);
int rfx_comm_init_rank(int world, int rank, const void* unique_id, int device, rfx_comm_t* out);
int rfx_comm_init_all(int n, const int* device_ids, rfx_comm_t* out);
int rfx_comm_info(rfx_comm_t c, int* world, int* rank, int* n_local);
int rfx_comm_destroy(rfx_comm_t c);
int rfx_allgather_records(rfx_comm_t c, const void* const* sends_d, void* const* recvs_d, int64_t nq, int k,
                          void* const* streams);
/* rfx_gather_records: the records of every rank to ONE rank (`root`), where the answer is assembled:
 * one grouped ncclSend per rank to the root and world ncclRecv on the root (one hop over xGMI's
 * point-to-point links instead of an all-gather ring's world - 1).  sends_d[i] as above;
 * recvs_d[i] = [world][nq][k] records for the local device that IS the root (rank mode: the
 * caller's device when rank == root; group mode: local device index root), NULL elsewhere. */
int rfx_gather_records(rfx_comm_t c, const void* const* sends_d, void* const* recvs_d, int root, int64_t nq,
                       int k, void* const* streams);

/* One search over a store row-sharded across the GPUs of one process (the index-server topology,
 * SURVEY §7; gemini_rag.py:721-725 get_rag_client -> one adapter over all the process's GPUs), issued from
 * C++ so the host cost of a batch does not grow with Python calls per shard: every shard's whole search
 * (rfx_search_records: kernel 10 / 11 where the shard holds its int8 copy) into [nq][k] records with
 * bases[i] added, the exchange, one rfx_merge_gathered into (out_scores_d, out_rows_d) on streams[0].
 *   handles / bases / streams / ws_d / ws_bytes / recs_d: per shard (n); queries_d on shard 0's device;
 *   qbuf_d (may be NULL): per shard a [nq][dim] buffer on its device the queries are copied into first
 *   (NULL entries, or the same pointer as queries_d: read in place — shards sharing shard 0's device);
 *   masks_d / mask_words (may be NULL): per-shard row masks; gathered_d: [n][nq][k] records on shard 0's
 *   device; comm: rfx_comm_init_all over the shards' devices in shard order (one RCCL gather to shard 0),
 *   or 0 when every shard is on one device (logical shards; recs_d[i] may then BE row i of gathered_d);
 *   src_stream: the stream that produced the queries, ordered before every shard and after the merge. */
int rfx_sharded_search(int n, const rfx_index_t* handles, const int64_t* bases, const void* queries_d,
                       void* const* qbuf_d, int64_t nq, int k, const uint32_t* const* masks_d,
                       const int64_t* mask_words, void* const* ws_d, const size_t* ws_bytes, void* const* recs_d,
                       void* gathered_d, rfx_comm_t comm, void* src_stream, void* const* streams,
                       float* out_scores_d, int64_t* out_rows_d);

/* ---- text → features (host) ---------------------------------------------------------------
 * The reference has no chunker/tokeniser of its own (chunking_config is forwarded to Gemini,
 * gemini_rag.py:324-326).  These restate the only tokeniser in the reference —
 * scripts/benchmark/metrics.py:13-19 (_normalize: lower, [^a-z0-9\s] -> ' ', split, drop
 * articles) — on UTF-8 bytes, after the caller has applied str.lower() for non-ASCII input.
 *
 * Whitespace chunking (Gemini white_space_config semantics): windows of max_tokens
 * whitespace-delimited tokens, consecutive windows overlapping by `overlap` tokens.
 * out_spans_h: [cap][2] byte offsets (start, end).  Returns the count in *out_n (if > cap
 * only the first cap are written). */
int rfx_chunk_whitespace(const char* text, int64_t len, int max_tokens, int overlap,
                         int64_t* out_spans_h, int64_t cap, int64_t* out_n);
/* Hashed bag-of-words features for n chunks (spans into text): CSR with per-chunk sorted
 * unique buckets (V a power of two) and signed counts clamped to [-256, 256]. */
int rfx_featurize(const char* text, const int64_t* spans_h, int64_t n, int V,
                  uint64_t hash_seed, int32_t* indptr_h /* n+1 */, int32_t* bucket_h,
                  int16_t* count_h, int64_t cap_nnz, int64_t* out_nnz);

/* ---- embedding (device) ---------------------------------------------------------------------
 * Chunk-embedding dense contraction on MFMA: E = F · W, F = densified CSR features [n][V]
 * (bf16), W = seeded projection [V][dim] (stored transposed, bf16), then exact L2
 * normalisation and cast to out_dtype.  Bit-identical to oracle/embed.py. */
int rfx_embed_weights(int V, int dim, uint64_t seed, void* wt_d /* [dim][V] bf16 */,
                      void* stream);
int rfx_embed_workspace_bytes(int64_t n, int V, size_t* out_bytes);
int rfx_embed(const int32_t* indptr_d, const int32_t* bucket_d, const int16_t* count_d,
              int64_t n, int V, const void* wt_d, int dim, void* out_d, int out_dtype,
              void* ws_d, size_t ws_bytes, void* stream);

/* ---- synthetic rows (tests / bench) --------------------------------------------------------- */
int rfx_synth_rows(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, void* out_d,
                   void* stream);
/* Clustered rows (IVF tests / config 5): normalise(centre(cluster(r)) + noise(r)); centres from
 * cseed (shared by corpus and queries), cluster(r) and noise from seed (oracle/ivf.py). */
int rfx_synth_clustered(uint64_t cseed, int64_t ncenters, uint64_t seed, int64_t row0, int64_t n,
                        int dim, int dtype, void* out_d, void* stream);

/* ---- IVF-Flat int8 (build plan item 8) -------------------------------------
 * No reference counterpart: the reference's only large-corpus answer is Gemini's managed index
 * (gemini_rag.py:463-469).  This extends the brute-force path for corpora where scanning every
 * row per batch is not wanted: a k-means coarse quantiser (int8 centroids, MFMA i8 scoring),
 * int8 posting lists, and a posting-list scan (v_dot4 against LDS-staged queries).  Numerics are
 * exact integer/IEEE steps restated by oracle/ivf.py (bit-exact); recall vs brute force < 1 by
 * design.  dim in {256, 512, 768, 1024}; nlist <= 16384; nprobe, k <= 64.
 * Lifecycle: create -> train (or set_centroids, e.g. broadcast from rank 0) -> add (quantise +
 * assign; posting lists rebuilt lazily) -> search. */
typedef uint64_t rfx_ivf_t;
int rfx_ivf_create(int device, int dim, int nlist, rfx_ivf_t* out);
int rfx_ivf_destroy(rfx_ivf_t h);
int rfx_ivf_info(rfx_ivf_t h, int* dim, int* nlist, int64_t* rows, int* trained);
/* k-means over n >= nlist sample rows (device, dtype f32/bf16/f16), iters Lloyd iterations */
int rfx_ivf_train(rfx_ivf_t h, const void* rows_d, int64_t n, int dtype, int iters, void* stream);
int rfx_ivf_set_centroids(rfx_ivf_t h, const int8_t* centroids_d /* [nlist][dim] */, void* stream);
int rfx_ivf_get_centroids(rfx_ivf_t h, int8_t* centroids_d, float* factors_d, void* stream);
int rfx_ivf_add(rfx_ivf_t h, const void* rows_d, int64_t n, int dtype, void* stream);
int rfx_ivf_build(rfx_ivf_t h, void* stream);
/* Persist / restore (like rfx_index_save/load): centroids, per-row codes, scales and labels. */
int rfx_ivf_save(rfx_ivf_t h, const char* path);
int rfx_ivf_load(const char* path, int device, rfx_ivf_t* out);
/* inspection (tests): per-row codes / scales / list labels in insertion order; list offsets
 * [nlist+1] and row ids in list order */
int rfx_ivf_codes(rfx_ivf_t h, int8_t* codes_d, float* inv_d, int32_t* labels_d, void* stream);
int rfx_ivf_lists(rfx_ivf_t h, int64_t* offsets_d, int32_t* ids_d, void* stream);
int rfx_ivf_search_workspace_bytes(rfx_ivf_t h, int64_t nq, int k, int nprobe, size_t* out_bytes);
/* queries_d [nq][dim] (dtype); outputs [nq][k] scores f32 / rows i64 (insertion-order row ids),
 * padded (-inf, -1) */
int rfx_ivf_search(rfx_ivf_t h, const void* queries_d, int64_t nq, int dtype, int k, int nprobe,
                   float* out_scores_d, int64_t* out_rows_d, void* ws_d, size_t ws_bytes,
                   void* stream);
/* Search + exact re-rank: the IVF keeps rerank_k (k <= rerank_k <= 64) candidates per query by
 * int8 score, each is re-scored in f32 against its original row (rows_d [rows][dim] of rows_dtype
 * in insertion order, e.g. rfx_index_data of a brute-force store holding the same rows), and the
 * top k are returned (score desc, row asc).  Lifts recall@10 above the int8 ceiling. */
int rfx_ivf_rerank_workspace_bytes(rfx_ivf_t h, int64_t nq, int k, int nprobe, int rerank_k,
                                   size_t* out_bytes);
int rfx_ivf_search_rerank(rfx_ivf_t h, const void* queries_d, int64_t nq, int dtype, int k,
                          int nprobe, int rerank_k, const void* rows_d, int rows_dtype,
                          float* out_scores_d, int64_t* out_rows_d, void* ws_d, size_t ws_bytes,
                          void* stream);
/* The re-rank step alone, for a store row-sharded over several devices (rfx/sharded.py
 * ShardedIvf; gemini_rag.py:463-469's file-search tool over an RFX_INDEX=ivf store): cand_d
 * [nq][n_cand] holds GLOBAL row ids (< 0 = padding); the candidates in [row_lo, row_lo + n_rows)
 * are re-scored in f32 against rows_d (this shard's rows: local row = global - row_lo), the others
 * come back as (-inf, -1).  out_scores_d / out_rows_d [nq][n_cand] (global rows): the merge input.
 * The same kernel and summation order as rfx_ivf_search_rerank, so a sharded store re-ranks its
 * candidates bit-identically to one device. */
int rfx_rerank_candidates(const void* queries_d, int64_t nq, int dtype, const void* rows_d,
                          int rows_dtype, int64_t row_lo, int64_t n_rows, int dim,
                          const int64_t* cand_d, int n_cand, float* out_scores_d,
                          int64_t* out_rows_d, void* stream);
/* int8 quantisation of rows (the IVF code format): codes [n][dim], inv [n] = amax / 127 */
int rfx_quantize(const void* rows_d, int64_t n, int dim, int dtype, int8_t* codes_d, float* inv_d,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RFX_H */
