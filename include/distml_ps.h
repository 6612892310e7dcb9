/*
 * distml_ps.h — C-ABI of the MI355X parameter-server push-reduce path.
 *
 * Drop-in boundary: this library replaces the body of DistML's server-side
 * plugin `abstract class DataStore` (reference: src/main/java/com/intel/distml/
 * util/DataStore.java:17-92) and its seven typed implementations under
 * util/store/. Every entry point names the reference method it replaces.
 * Plain C types only: a JNI shim, ctypes, or C++ can bind it.
 *
 * Threading: every call on one store is serialized by a mutex inside the store
 * (the reference calls a store from the PSAgent selector thread, Akka dispatcher
 * threads and the PSSync thread, PSAgent.java:278, PSActor.java:171-251,
 * PSSync.java:131). Each store owns one HIP stream on its device; every call
 * does hipSetDevice, so any host thread may call.
 *
 * Status codes map 1:1 to the exceptions the reference throws:
 *   DML_E_BAD_DESC          IllegalArgumentException  (DataStore.java:91)
 *   DML_E_KEY_OUT_OF_SHARD  ArrayIndexOutOfBoundsException (localData[indexOf(key)])
 *   DML_E_TRUNCATED         ArrayIndexOutOfBoundsException (readInt/readFloat past data.length)
 *   DML_E_NEGATIVE_COUNTER  IllegalStateException (IntMatrixStore.java:174-176, IntArrayStore.java:108-110)
 * After one of these four the store holds exactly the values the reference
 * store holds when its exception escapes handlePush (every add before the
 * failing position applied, nothing after it), and the error is recorded in
 * dml_store_error_state(). DML_E_* codes >= 16 are library/usage errors with
 * no reference counterpart.
 */
#ifndef DISTML_PS_H
#define DISTML_PS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* DataDesc constants (DataDesc.java:10-19). */
#define DML_DATA_TYPE_ARRAY   0
#define DML_DATA_TYPE_MATRIX  1
#define DML_KEY_TYPE_INT      0
#define DML_KEY_TYPE_LONG     1
#define DML_ELEMENT_TYPE_INT    0
#define DML_ELEMENT_TYPE_FLOAT  1
#define DML_ELEMENT_TYPE_LONG   2
#define DML_ELEMENT_TYPE_DOUBLE 3

/* Status codes. */
#define DML_OK                   0
#define DML_E_BAD_DESC           1
#define DML_E_KEY_OUT_OF_SHARD   2
#define DML_E_TRUNCATED          3
#define DML_E_NEGATIVE_COUNTER   4
#define DML_E_INVALID_ARG       16
#define DML_E_HIP               17
#define DML_E_NOMEM             18
#define DML_E_UNSUPPORTED       19
#define DML_E_CAPACITY          20

/* Store option flags (dml_store_create_range `flags`). */
/* FloatArrayStore reads records with VALUE_SIZE = 8 (FloatArrayStore.java:15)
 * although every writer emits key|f32 records (SparseArray.java:63-76). The
 * default follows the writer (stride keySize+4); this flag reproduces the
 * reference's stride keySize+8 read bit for bit (SURVEY.md defect 1). */
#define DML_FLAG_FLOAT_ARRAY_REF_STRIDE  0x1
/* Apply pushes asynchronously: dml_store_push returns once the bytes are
 * captured (staged); a deferred error surfaces at the next call. Default is
 * synchronous: the call returns after the apply, like the reference's ack
 * (PSAgent.java:278-281). */
#define DML_FLAG_ASYNC                   0x2
/* No identity speculation / slot reuse. By default a plain-sum
 * matrix store that receives full-range device pushes allocates a second shard
 * buffer (rows*cols values) on first use, when the device has that plus
 * max(1/8 of its memory, 4 GiB) free; this flag never allocates it. */
#define DML_FLAG_NO_SPECULATION          0x4

/* Mirrors the six big-endian int32s DataDesc puts on the wire, in wire order
 * (DataDesc.java:62-69). key/value sizes derive as in DataDesc.java:50-51. */
typedef struct dml_desc {
    int32_t data_type;
    int32_t key_type;
    int32_t value_type;
    int32_t dense_row;
    int32_t dense_column;
    int32_t ada_grad;
} dml_desc;

typedef struct dml_store dml_store; /* opaque; one per (matrix, shard) */

/* --- lifecycle --------------------------------------------------------- */

/* == DataStore.createStore(serverIndex, matrix) (DataStore.java:50-92) for a
 * KeyRange shard [first_key, last_key] (KeyRange.linearSplit, KeyRange.java:68-80),
 * followed by the store's init(keys[, cols]) (e.g. FloatMatrixStore.java:28-37):
 * the shard is zero-filled in HBM. `cols` is ignored for ARRAY stores. */
int dml_store_create_range(const dml_desc* desc, int64_t first_key, int64_t last_key,
                           int32_t cols, int32_t device, uint32_t flags, dml_store** out);
void dml_store_destroy(dml_store* s);

/* KeyRange.linearSplit(n) (KeyRange.java:68-80): shard i = [first_out[i], last_out[i]]. */
int dml_linear_split(int64_t first_key, int64_t last_key, int32_t n,
                     int64_t* first_out, int64_t* last_out);

/* --- the hot path: handlePush ------------------------------------------ */

/* == store.handlePush(format, data) (DataStore.java:30; FloatMatrixStore.java:200-238,
 * FloatArrayStore.java:110-122, IntMatrixStore.java:154-195, IntArrayStore.java:97-113,
 * FloatMatrixStoreAdaGrad.java:239-306, DoubleArrayStore.java:115-127,
 * DoubleMatrixStore.java:153-190). `data` is a host buffer BORROWED for the
 * call only (the JVM byte[]). Records use the store's own DataDesc
 * (PSAgent.java:279 passes the server-side format). */
int dml_store_push(dml_store* s, const uint8_t* data, int64_t len);

/* n sequential handlePush calls, bucket 0 first, applied as ONE ordered
 * multi-bucket reduce: each element is summed in push order, so the result is
 * bit-identical to calling handlePush n times. Host buffers, borrowed. */
int dml_store_push_batch(dml_store* s, const uint8_t* const* bufs, const int64_t* lens, int32_t n);

/* Same, for buckets already resident in device memory on the store's device
 * (the device-resident north-star path). Buffers must stay valid until the
 * next dml_store_flush (or any read call). */
int dml_store_push_batch_device(dml_store* s, const void* const* dev_bufs, const int64_t* lens, int32_t n);

/* Read barrier: every accepted push is applied; returns any deferred error. */
int dml_store_flush(dml_store* s);

/* Buffer release without a full flush (no reference counterpart: the JVM's
 * byte[] is always copied). Every push call (dml_store_push, _push_batch,
 * _push_batch_device) is numbered 1, 2, ...; dml_store_push_seq returns the
 * number of the last accepted one. dml_store_retire(s, seq) finishes every chunk
 * of the calls up to `seq` on the host (exact replays, int32 rollbacks, re-runs of
 * failed speculation: the reads of a push that may follow its device apply); when
 * it returns, those calls' device buffers are no longer read and may be reused or
 * freed. Returns the first error those chunks met (sticky, as for flush). */
int dml_store_push_seq(dml_store* s, uint64_t* seq);
int dml_store_retire(dml_store* s, uint64_t seq);

/* Pipeline counters since creation or the last reset (diagnostic): chunks
 * retired, speculative chunks and how many of them re-ran without speculation,
 * and per push how its records found their rows: identity (record r = row r,
 * verified in the reduce), reused (a kept slot-table column, verified), indexed
 * (the key index). Counted when a chunk retires: flush first. */
typedef struct dml_store_counters {
    int64_t chunks;
    int64_t spec_chunks;
    int64_t spec_reruns;
    int64_t identity_pushes;
    int64_t reused_pushes;
    int64_t indexed_pushes;
    int64_t sparse_big_chunks;  /* array chunks applied through the one-level partition (big leaves) */
    int64_t sparse_replays;     /* array chunks with leaves the exact replay applied */
    int64_t ident_launches;     /* chunks / pre-reduce pieces launched through the all-identity
                                   kernels (k_flat_ident, k_ada_ident) */
} dml_store_counters;
int dml_store_stats(dml_store* s, dml_store_counters* out, int32_t reset);

/* First error the store has seen (sticky until dml_store_clear_error):
 * status code, the key and column the reference would report, 0 if none. */
int dml_store_error_state(dml_store* s, int64_t* bad_key, int32_t* bad_col);
void dml_store_clear_error(dml_store* s);

/* --- shard access ------------------------------------------------------ */

/* KeyRange size (KeyRange.java:92-94) and rowSize() (FloatMatrixStore.java:24-26;
 * 1 for arrays). */
int dml_store_shape(dml_store* s, int64_t* rows, int32_t* cols);
/* The store's DataDesc value type (DML_ELEMENT_TYPE_*) and whether it is an AdaGrad
 * store (DataDesc.java:21-42): the element type its rows hold for dml_store_read_rows
 * (the JNI snapshot checks the Java array it fills against it). */
int dml_store_value_type(dml_store* s, int32_t* value_type, int32_t* adagrad);

/* Raw row-major shard values (rows*cols elements of the store's value type)
 * to/from host memory; test/oracle access and initial load. */
int dml_store_read_dense(dml_store* s, void* host_dst, int64_t bytes);
int dml_store_write_dense(dml_store* s, const void* host_src, int64_t bytes);
/* Device pointer of the value array (rows*cols elements) as of this call; valid
 * until the next push (a speculative full-range batch writes the store's second
 * buffer and commits it) or destroy. */
int dml_store_device_ptr(dml_store* s, void** dev_ptr);
/* AdaGrad side arrays (FloatMatrixStoreAdaGrad.java:23-24), f32 row-major. */
int dml_store_read_adagrad(dml_store* s, float* alpha_dst, float* delta_dst, int64_t elems);
/* Local rows [row0, row0 + nrows) of the shard's values (which 0, the store's value
 * type), or of AdaGrad's alpha (1) / delta (2) (f32), row-major and native-endian,
 * after every accepted push: the snapshot behind the stores' Iter, which the
 * result-collect paths read (DoubleArrayStore.java:129-157, FloatMatrixStore.java:241-269,
 * FloatArrayStore.java:124-152, FloatMatrixStoreAdaGrad.java:308-337; called from
 * LogisticRegression.scala:290-291 and Word2Vec.scala:814-817). Row ranges let a JVM
 * fill its heap arrays in bounded chunks. */
int dml_store_read_rows(dml_store* s, int32_t which, int64_t row0, int64_t nrows, void* host_dst, int64_t bytes);

/* DataStore.rand() (DataStore.java:22; PSActor OP_RAND, PSActor.java:181-201).
 * DoubleMatrixStore: exactly the reference's values — java.util.Random(1L) on every
 * shard, |nextGaussian()| per element, each row divided by its L2 norm
 * (DoubleMatrixStore.java:192-207); `seed` is not used. Float matrices, AdaGrad
 * included, draw from an unseeded java.util.Random in the reference
 * (FloatMatrixStore.java:44, FloatMatrixStoreAdaGrad.java:60), which nothing can
 * reproduce: here (a/100f - 0.5f)/rowSize with a uniform a in 0..99, in float
 * arithmetic, from a counter-based generator seeded by `seed`. Other stores: no-op. */
int dml_store_rand(dml_store* s, uint64_t seed);
/* Fill every value with v: FloatMatrixStore.setValue (FloatMatrixStore.java:61-71), what
 * set(String) does on the float matrix stores (:53-55, FloatMatrixStoreAdaGrad.java:69-71).
 * The reference's zero() is a no-op on every store (DataStore.java:24; the float stores'
 * zero(String) is an overload OP_ZERO never calls) and set() a no-op on the others: the
 * DataStore mirrors (GpuDataStore.java, distml_amd/store.py) call this only where the
 * reference's store would change. */
int dml_store_fill(dml_store* s, double v);
/* FloatMatrixStoreAdaGrad.setAlpha(initialAlpha, minAlpha, factor) (:77-82). */
int dml_store_set_alpha(dml_store* s, float initial_alpha, float min_alpha, float factor);
/* maxDelta / maxDeltaRow / maxDeltaCol printed by AdaGrad handlePush (:246, :273-277). */
int dml_store_max_delta(dml_store* s, float* max_delta, int32_t* row, int32_t* col);

/* == handleFetch(format, rows), dense-column layout (FloatMatrixStore.java:113-174,
 * IntMatrixStore.java:81-140, FloatArrayStore.java:88-108, IntArrayStore.java:78-95,
 * DoubleArrayStore.java handleFetch, FloatMatrixStoreAdaGrad.java:146-213).
 * `keys` are the intersected keys in the caller's iteration order; every key
 * must lie in the shard. Writes the reference byte layout to `out`. */
int dml_store_fetch(dml_store* s, const int64_t* keys, int64_t nkeys,
                    uint8_t* out, int64_t cap, int64_t* out_len);
/* Same for a KeyRange request: keys first..last ascending (KeyRange.intersect). */
int dml_store_fetch_range(dml_store* s, int64_t first_key, int64_t last_key,
                          uint8_t* out, int64_t cap, int64_t* out_len);

/* writeAll/readAll (FloatMatrixStore.java:74-91 etc.): big-endian row-major
 * values, the bytes DataOutputStream.writeFloat/writeInt/writeDouble emit.
 * read_all assigns the elements the stream holds before failing with
 * DML_E_TRUNCATED when it is short (readFloat's EOFException). */
int dml_store_write_all(dml_store* s, uint8_t* out_be, int64_t cap, int64_t* out_len);
int dml_store_read_all(dml_store* s, const uint8_t* in_be, int64_t len);
/* syncTo/syncFrom(stream, fromRow, toRow) (FloatMatrixStore.java:94-110,
 * IntArrayStore.java:64-75 etc.; called by PSSync.java:131,160): local rows
 * from..to inclusive, big-endian. to < from moves nothing; a negative from
 * fails before any byte; rows past the shard fail with DML_E_KEY_OUT_OF_SHARD
 * after the rows before them were moved (the reference's
 * ArrayIndexOutOfBoundsException). sync_from uses the intended row layout
 * (defect 5). */
int dml_store_sync_to(dml_store* s, int32_t from_row, int32_t to_row, uint8_t* out_be, int64_t cap,
                      int64_t* out_len);
int dml_store_sync_from(dml_store* s, int32_t from_row, int32_t to_row, const uint8_t* in_be, int64_t len);

/* Pinned host memory for callers that receive pushes or return fetches through
 * it (a JNI DirectByteBuffer over it lets NIO read a PushRequest straight into
 * DMA-able memory, PSAgent.java:27-62): pushes from it are DMA'd without
 * staging, fetch / write_all / sync_to into it skip the bounce buffers. */
int dml_host_alloc(int64_t bytes, void** host_ptr);
void dml_host_free(void* host_ptr);

/* --- stream / timing / device reduce building blocks ------------------- */

/* hipStream_t of the store, as void*. */
int dml_store_stream(dml_store* s, void** stream);
/* When enabled, the store brackets launches of its dominant reduce kernel with
 * HIP events on its stream: every launch for enable == 1, one matrix chunk in
 * `enable` for enable > 1 (events in every dispatch lengthen the boundary between
 * two reduces); dml_store_kernel_time returns the summed elapsed ms and the
 * number of timed launches since the last reset. */
int dml_store_set_timing(dml_store* s, int32_t enable);
int dml_store_kernel_time(dml_store* s, double* total_ms, int64_t* launches, int32_t reset);
/* The instantiation of that dominant kernel as last launched, in rocprof's
 * spelling without "void " and the parameter list (e.g.
 * "dml::k_reduce_rows<float, 0, 4, 4, true, true, 1, 4, 0>"); "" before any push.
 * bench.py reports a profile's counted HBM bytes only for the kernel that ran. */
int dml_store_kernel_name(dml_store* s, char* out, int32_t cap);

/* Elementwise shard += src for a dense device buffer of rows*cols values in the
 * store's layout (owner-side apply after a reduce-scatter). */
int dml_store_apply_dense_device(dml_store* s, const void* dev_src, int64_t elems);
/* Two-moment AdaGrad owner apply: dev_src holds rows x [cols Σu |
 * cols Σu²] f32 (the reduce-scattered dml_prereduce_moments_piece output of the
 * shard's rows); data += Σu, delta += Σu², alpha = initialAlpha / (factor *
 * sqrt(delta)) clamped to minAlpha where delta ends above 1, maxDelta updated
 * (FloatMatrixStoreAdaGrad.java:262-277 for the summed update; ties of maxDelta
 * go to the first element in row-major order). Within 1e-6 of the sequential
 * reference, not bit-exact: the exact path is dml_group_push_exchange. */
int dml_store_apply_adagrad_moments_device(dml_store* s, const void* dev_src, int64_t rows);

/* Ordered reduce of n device-resident full-range buckets into a dense device
 * buffer `dev_out` (rows*cols values of `value_type`, row = key - first_key):
 * out = b0 + b1 + ... in push order (rows no bucket touches are zero).
 * The multi-GPU pre-reduce before the reduce-scatter. Runs on `stream`. */
int dml_reduce_buckets_dense(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols,
                             const void* const* dev_bufs, const int64_t* lens, int32_t n,
                             void* dev_out, void* stream);

/* Piecewise pre-reduce for pipelining with the reduce-scatter: _begin enqueues
 * the key index of the n (<= 64) full-range pushes on `stream`; each _piece
 * writes the ordered sum of rows r(t) = (t / row_block) * row_stride + row_off
 * + t % row_block, t < ntask_rows, to dev_out + t*cols (rows >= `rows`, the
 * padding of linearSplit's short last shard, are zeros); _end waits for the
 * index and every piece and reports key-out-of-matrix / repeated-row errors.
 * Each piece runs on its own `stream` argument (0 = the null stream), which may
 * differ from _begin's (the first such piece waits for the index on the host),
 * so the next call's index can overlap the current call's pieces. Opaque handle. */
typedef struct dml_prereduce dml_prereduce;
int dml_prereduce_begin(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols,
                        const void* const* dev_bufs, const int64_t* lens, int32_t n, void* stream,
                        dml_prereduce** out);
int dml_prereduce_piece(dml_prereduce* p, int64_t row_block, int64_t row_stride, int64_t row_off,
                        int64_t ntask_rows, void* dev_out, void* stream);
int dml_prereduce_end(dml_prereduce* p);
/* The two-moment piece of an AdaGrad matrix's pre-reduce (begun with its desc):
 * task row t's Σu and Σu·u over the pushes, in push order, written as
 * dev_out + t*2*cols = [cols Σu | cols Σu²] (f32; rows of whole 16-B vectors
 * under 4 KiB). A call whose index found a key outside the matrix or a repeated
 * row writes zeros (_end reports the error). */
int dml_prereduce_moments_piece(dml_prereduce* p, int64_t row_block, int64_t row_stride, int64_t row_off,
                                int64_t ntask_rows, void* dev_out, void* stream);
/* Make `stream` wait (device side) for the pieces enqueued so far, e.g. the
 * communication stream that reduce-scatters the piece just written. */
int dml_prereduce_stream_wait(dml_prereduce* p, void* stream);
/* Measurement: with every > 0, the pieces of one call in `every` carry
 * start/stop events in their dispatch packets and _end adds their elapsed time
 * to a process-wide total (bench.py's roofline of the sharded path; no
 * reference counterpart). 0 turns timing off. */
int dml_prereduce_timing(int32_t every);
int dml_prereduce_kernel_time(double* ms, int64_t* launches, int32_t reset);

/* Speculative pre-reduce (the sharded path's per-call cost). A
 * context holds a ring of three workspaces for one matrix (rows*cols, the
 * whole model) on `device`. _begin_ctx is _begin within the context: full-range
 * pushes whose sampled records say "record r holds row r", or that match a
 * permutation a call three before listed (kept slot-table columns, any
 * position), skip the key index, and the pieces verify every record's key.
 * dml_prereduce_verify waits for the pieces and reads their verdict; if a
 * record was not what the sample said, it re-runs the call exactly (fresh
 * table, full key index, every piece as launched) on the context's stream and
 * sets *rerun. Consume the partial (reduce-scatter) only after verify, behind
 * dml_prereduce_stream_wait; _end then reports the call's errors as before.
 * dml_prectx_stats counts calls as dml_store_stats counts chunks. At most three
 * calls of one context may be outstanding (begun and not yet ended): a fourth
 * _begin_ctx returns DML_E_INVALID_ARG instead of reusing a busy workspace. */
typedef struct dml_prectx dml_prectx;
int dml_prectx_create(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols, int32_t device,
                      dml_prectx** out);
void dml_prectx_destroy(dml_prectx* ctx);
int dml_prectx_stats(dml_prectx* ctx, dml_store_counters* out, int32_t reset);
int dml_prereduce_begin_ctx(dml_prectx* ctx, const void* const* dev_bufs, const int64_t* lens, int32_t n,
                            void* stream, dml_prereduce** out);
int dml_prereduce_verify(dml_prereduce* p, int32_t* rerun);

/* --- per-shard split of device-resident pushes (multi-GPU exchange path) -- */

/* The client-side split of SparseMatrix.push / SparseArray.push
 * (SparseMatrix.java:46-60): the records of each of the n pushes `dev_bufs[b]`
 * (lens[b] bytes, whole records of the desc's wire layout; `cols` for matrices)
 * are partitioned by owner shard under KeyRange(0, total_rows-1).linearSplit(world)
 * (KeyRange.java:68-80), keeping each push's record order, and written to
 * `dev_out` dest-major: [dest 0: push 0's records, push 1's, ...][dest 1: ...].
 * counts[b*world + d] (host, n*world) receives the record count of push b for
 * dest d. Keys outside [0, total_rows) are dropped (the client's p.contains(k)).
 * Kernels run on `stream`; the call returns when dev_out is written.
 * DML_E_CAPACITY when out_cap is smaller than the kept bytes; world <= 64, n <= 64.
 * dev_out == NULL: counts only (nothing is copied). */
int dml_shard_split(const dml_desc* desc, int32_t cols, int64_t total_rows, int32_t world,
                    const void* const* dev_bufs, const int64_t* lens, int32_t n, void* dev_out,
                    int64_t out_cap, int64_t* counts, void* stream);

/* --- native multi-GPU shard group (RCCL) -------------------------------- *
 * One process per GPU; rank r owns shard r of KeyRange.linearSplit(world)
 * (KeyRange.java:68-80). Full-range device-resident pushes are pre-reduced in
 * push order, reduce-scattered over xGMI (ncclReduceScatter, sum) and applied
 * by the owner — the path distml_amd/group.py runs over torch.distributed, for
 * hosts without Python (the JNI deployment). The caller distributes the
 * 128-byte unique id from rank 0 (e.g. over the PS control plane). Pushes are
 * asynchronous: buffers stay valid until the next dml_group_flush, and a
 * call's key / repeated-row errors surface at the next call or the flush.
 * fp32 results differ from the sequential order only by summation order
 * (DESIGN.md §6); int32 is exact.
 * Store order: the group applies its calls to its store in call order; a push made
 * straight to the dml_group_store handle bypasses that order, and a read of that
 * handle sees only the calls applied so far — call dml_group_flush before either,
 * or push through dml_group_push_local.
 * Collective order: every rank issues the same collectives in the same order
 * whatever fails locally; a rank whose call fails (a push that is not whole
 * records, a HIP error, a failed re-run) contributes zeros to that call's
 * collective, skips its own apply and returns the error. The group is then in an
 * undefined state for that rank (the reference's PS thread ends on an exception,
 * PSAgent.java:188-191): destroy it. */
typedef struct dml_group dml_group;
int dml_group_unique_id(uint8_t* out, int32_t cap);
int dml_group_create(const uint8_t* unique_id, int32_t world, int32_t rank, int32_t device, const dml_desc* desc,
                     int64_t total_rows, int32_t cols, int32_t pieces, dml_group** out);
/* The rank's shard store (fetch / checkpoint / read), owned by the group. */
int dml_group_store(dml_group* g, dml_store** store);
/* dml_prectx_stats of the group's speculative pre-reduce (zeros before the first
 * full-range call). */
int dml_group_prereduce_stats(dml_group* g, dml_store_counters* out, int32_t reset);
int dml_group_push_full_range(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n);
/* The exact path (AdaGrad, int32-checked, arrays, key-subset pushes): each of the
 * rank's n device-resident pushes is split by owner shard (dml_shard_split), the
 * slices go to their owners in one grouped ncclSend/ncclRecv exchange, and every
 * owner applies the slices it received in rank-major push order (rank 0's n
 * pushes, then rank 1's, ...) through the store's ordered push — the reference's
 * client-split + server-apply data flow, bit-exact with errors included. Every
 * rank calls with the same n (<= 64). The owner's pushes are asynchronous: their
 * errors surface at the next exchange call or at dml_group_flush. */
int dml_group_push_exchange(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n);
/* AdaGrad's sharded path for many pushes per rank: the rank's n
 * full-range pushes pre-reduced into Σu and Σu² (dml_prereduce_moments_piece),
 * one ncclReduceScatter of both, the owner's
 * dml_store_apply_adagrad_moments_device. xGMI bytes per rank: (world-1)/world
 * x 2 x the model, whatever n is (the exchange path moves n pushes). Within
 * 1e-6, not bit-exact; errors surface at the next call or the flush. Known
 * divergences: a maxDelta tie goes to the first element in row-major order (the
 * reference's: the first in push / record order, FloatMatrixStoreAdaGrad.java:273-277),
 * and with NaN / Inf gradients alpha keeps its value. */
int dml_group_push_moments(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n);
/* Pushes the client already split to this shard (SparseMatrix.java:46-60): the
 * store's exact ordered device push (dml_store_push_batch_device), queued after
 * every earlier group call's apply; no collective. */
int dml_group_push_local(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n);
int dml_group_flush(dml_group* g);
void dml_group_destroy(dml_group* g);
/* Fault injection for tests: the nth full-range call finished from now on (1 = the
 * next) fails its verdict as a local HIP error would (0 = off). */
int dml_group_debug_fail_verify(dml_group* g, int32_t nth);

/* --- synthetic workload generators (bench/test support) ----------------- *
 * Counter-based (SplitMix64) so the CPU oracle regenerates the same bytes.
 * Spec in DESIGN.md §Synthetic data. Run on `stream` (void* hipStream_t). */
int dml_synth_dense_bucket(void* dev_out, const dml_desc* desc, int64_t first_key,
                           int64_t shard_rows, int64_t nrec, int32_t cols, uint64_t seed,
                           uint64_t perm_a, uint64_t perm_c, void* stream);
int dml_synth_sparse_bucket(void* dev_out, const dml_desc* desc, int64_t first_key,
                            int64_t key_space, int64_t nrec, uint64_t seed,
                            uint64_t perm_a, uint64_t perm_c, void* stream);
int dml_synth_fill_store(dml_store* s, uint64_t seed);

/* Diagnostic: stream `bytes` (multiple of 16, 16-B aligned) from dev_src with
 * 16-B non-temporal loads, copying them to dev_dst (copy != 0) or only reading
 * them (copy == 0; dev_dst receives at most one word); timed by HIP events on
 * `stream`, *ms = kernel time. bench.py reports the reduce's fraction of these
 * measured HBM ceilings. */
int dml_diag_stream(int32_t copy, void* dev_dst, const void* dev_src, int64_t bytes, void* stream, float* ms);
/* Random-RMW floor (diagnostic): dev_array[dev_index[i]] += dev_values[i] for i < n,
 * one plain 4-B read-modify-write per update, in the given (sorted) order, timed on
 * `stream`, *ms = kernel time. Every index must lie inside dev_array; repeated
 * indices race, so the array's values are not meaningful afterwards (scratch only).
 * bench.py's config-3 leg times the leaf apply against it: the same updates sorted
 * globally, with no partition, are the best case of the random scatter-add. */
int dml_diag_rmw_floor(float* dev_array, const uint32_t* dev_index, const float* dev_values, int64_t n, void* stream,
                       float* ms);

/* Dense stream floor (diagnostic, config 4 and its AdaGrad variant): the store's f32
 * shard (cols a multiple of 4) plus n full-range pushes whose records are rows in order
 * (lens[b] = rows x record stride; record r is taken to be row r, keys not read), each
 * element summed in push order and written once: into the speculative second buffer
 * where the store has one (as k_flat_ident writes, *out_of_place = 1; the committed
 * shard is left alone), else in place; AdaGrad stores also delta += u·u in place (alpha
 * and maxDelta untouched). The plain stream of the reduce's bytes over the same
 * allocations, timed on `stream`, *ms = kernel time: bench.py's config-4 legs report
 * their kernels against it. */
int dml_diag_dense_floor(dml_store* s, const void* const* dev_bufs, const int64_t* lens, int32_t n, void* stream,
                         float* ms, int32_t* out_of_place);

/* Row-gather floor (diagnostic, config 5): for each of the ntouched rows dev_rows[i] of
 * an int32 shard (row-major, `cols` a multiple of 4, at most 1024), read the row once,
 * add the records dev_addr[dev_ptr[i] .. dev_ptr[i+1]) (device addresses of each
 * record's first value, in push order) and write the row once: the IntMatrixStore
 * reduce's bytes with no key index, slot table or negativity check. Timed on `stream`,
 * *ms = kernel time. bench.py's config-5 leg reports the reduce against it. */
int dml_diag_gather_floor(int32_t* dev_shard, int32_t cols, const int32_t* dev_rows, const int32_t* dev_ptr,
                          const uint64_t* dev_addr, int64_t ntouched, void* stream, float* ms);

/* Ring reduce-scatter footprint (diagnostic, bench.py --emulate-rs N): the local HBM
 * traffic one rank's ring reduce-scatter of a world x chunk_bytes partial makes —
 * world - 1 steps, each reading one chunk of the partial and the chunk that arrived
 * (dev_landing, 2 x chunk_bytes) and landing their sum in a buffer (the write a peer
 * makes into this rank's), then the last sum into dev_recv — on a grid of `channels`
 * blocks (RCCL's one block per channel), enqueued on `stream`. Values are not a
 * reduce-scatter's (no peer contributes): timing only. */
int dml_diag_ring_rs(int32_t value_type, const void* dev_partial, void* dev_recv, void* dev_landing,
                     int64_t chunk_bytes, int32_t world, int32_t rank, int32_t channels, void* stream);

/* Store tuning knob (diagnostic / tests): DML_KNOB_IDENT_FULL_MIN_BYTES = the slot-table
 * size (bytes) from which an AdaGrad chunk of full-range pushes checks every record's key
 * up front (k_ident_full) instead of running the key index, so that all-identity chunks
 * run k_ada_ident (default 64 MiB: where the index's slot-table atomics leave the caches).
 * Lowering it lets tests drive that path at small sizes; results are the same either way.
 * Returns DML_E_INVALID_ARG for an unknown knob or a negative value. */
#define DML_KNOB_IDENT_FULL_MIN_BYTES 1
/* DML_KNOB_INDEX_CUS = k | pattern << 16: the store's index stream (the next chunk's key
 * index or sparse partition) on k CUs and its apply stream on the others, k = 0 (the
 * default) both on every CU; pattern 0 spreads the k CUs evenly over the CU numbering,
 * 1 takes the first k (config 3: the partition beside the leaf). */
#define DML_KNOB_INDEX_CUS 2
int dml_diag_store_knob(dml_store* s, int32_t knob, int64_t value);

/* --- misc --------------------------------------------------------------- */
const char* dml_last_error(void);   /* thread-local message for the last failure */
const char* dml_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DISTML_PS_H */
