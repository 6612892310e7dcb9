/*
 * dml_oracle.c — CPU restatement of DistML's DataStore push/fetch/checkpoint
 * loops. TEST INFRASTRUCTURE ONLY (see dml_oracle.h). PARITY UNPINNED: no
 * reference tests, fixtures or runnable reference exist for this path; pinned
 * by hand-derived JLS known-answer tests (tests/golden/kat_*.json).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math -fwrapv,
 * SSE2 scalar float/double arithmetic = IEEE binary32/binary64 as the JLS
 * requires for float/double + * / and Math.sqrt).
 *
 * Reference paths below are relative to
 * /root/reference/src/main/java/com/intel/distml/.
 */
#include "dml_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

struct orc_store {
    int32_t data_type, key_type, value_type, dense_column, ada_grad;
    int32_t key_size, value_size;      /* DataDesc.java:50-51 */
    int32_t array_value_stride;        /* FloatArrayStore VALUE_SIZE (8) or writer stride (4) */
    int64_t first, last, rows;
    int32_t cols;                      /* rowSize; 1 for arrays */
    void* data;                        /* localData, row-major */
    float* alpha;                      /* FloatMatrixStoreAdaGrad.java:23 */
    float* delta;                      /* FloatMatrixStoreAdaGrad.java:24 */
    float initial_alpha, min_alpha, factor; /* :22, :26 (factor = 1.5f) */
    float max_delta;                   /* :27-29 */
    int32_t max_delta_row, max_delta_col;
    int err;
    int64_t err_key;
    int32_t err_col;
};

/* ---- DataDesc little-endian codec (DataDesc.java:180-212) ---------------- */
static inline int32_t rd_i32(const uint8_t* p) {
    uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    return (int32_t)v;
}
static inline int64_t rd_i64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return (int64_t)v;
}
static inline float rd_f32(const uint8_t* p) { /* Float.intBitsToFloat(readInt) */
    int32_t b = rd_i32(p);
    float f;
    memcpy(&f, &b, 4);
    return f;
}
static inline double rd_f64(const uint8_t* p) { /* Double.longBitsToDouble(readLong) */
    int64_t b = rd_i64(p);
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static inline void wr_i32(uint8_t* p, int32_t v) { /* DataDesc.java:237-243 */
    uint32_t u = (uint32_t)v;
    p[0] = u & 0xff; p[1] = (u >> 8) & 0xff; p[2] = (u >> 16) & 0xff; p[3] = u >> 24;
}
static inline void wr_i64(uint8_t* p, int64_t v) { /* DataDesc.java:220-230 */
    uint64_t u = (uint64_t)v;
    for (int i = 0; i < 8; ++i) p[i] = (u >> (8 * i)) & 0xff;
}
static inline void wr_f32(uint8_t* p, float f) { int32_t b; memcpy(&b, &f, 4); wr_i32(p, b); }
static inline void wr_f64(uint8_t* p, double d) { int64_t b; memcpy(&b, &d, 8); wr_i64(p, b); }
/* DataOutputStream big-endian writers (writeAll, FloatMatrixStore.java:74-81). */
static inline void wr_be32(uint8_t* p, uint32_t u) { p[0] = u >> 24; p[1] = (u >> 16) & 0xff; p[2] = (u >> 8) & 0xff; p[3] = u & 0xff; }
static inline uint32_t rd_be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

/* readKey (DataDesc.java:131-138) -> long */
static inline int64_t rd_key(const orc_store* s, const uint8_t* p) {
    return s->key_size == 4 ? (int64_t)rd_i32(p) : rd_i64(p);
}

/* indexOf for KeyRange (FloatMatrixStore.java:176-179): (int)(key - firstKey),
 * a narrowing long->int conversion (low 32 bits, JLS 5.1.3). -1 if the array
 * access localData[index] would throw ArrayIndexOutOfBoundsException. */
static inline int64_t row_index(const orc_store* s, int64_t key) {
    int32_t idx = (int32_t)(uint32_t)((uint64_t)key - (uint64_t)s->first);
    if (idx < 0 || (int64_t)idx >= s->rows) return -1;
    return idx;
}

static int fail(orc_store* s, int code, int64_t key, int32_t col) {
    if (!s->err) { s->err = code; s->err_key = key; s->err_col = col; }
    return code;
}

/* ---- lifecycle: DataStore.createStore (DataStore.java:50-92) ------------- */
orc_store* orc_create(int32_t data_type, int32_t key_type, int32_t value_type,
                      int32_t dense_column, int32_t ada_grad,
                      int64_t first_key, int64_t last_key, int32_t cols,
                      int32_t float_array_ref_stride) {
    if (data_type != 0 && data_type != 1) return NULL;
    if (key_type != 0 && key_type != 1) return NULL;
    /* createStore has no ELEMENT_TYPE_LONG case: IllegalArgumentException (:91). */
    if (value_type != 0 && value_type != 1 && value_type != 3) return NULL;
    if (data_type == 0) cols = 1;
    if (cols <= 0 || last_key < first_key) return NULL;
    orc_store* s = (orc_store*)calloc(1, sizeof(*s));
    if (!s) return NULL;
    s->data_type = data_type; s->key_type = key_type; s->value_type = value_type;
    s->dense_column = dense_column; s->ada_grad = (data_type == 1 && value_type == 1) ? ada_grad : 0;
    s->key_size = key_type == 0 ? 4 : 8;
    s->value_size = (value_type == 0 || value_type == 1) ? 4 : 8;
    s->array_value_stride = s->value_size;
    if (data_type == 0 && value_type == 1 && float_array_ref_stride) s->array_value_stride = 8;
    s->first = first_key; s->last = last_key;
    s->rows = last_key - first_key + 1;                 /* KeyRange.size(), KeyRange.java:92-94 */
    s->cols = cols;
    s->factor = 1.5f;                                   /* FloatMatrixStoreAdaGrad.java:26 */
    size_t n = (size_t)s->rows * (size_t)cols;
    s->data = calloc(n ? n : 1, (size_t)s->value_size); /* init(): zero-filled, FloatMatrixStore.java:32-36 */
    if (!s->data) { free(s); return NULL; }
    if (s->ada_grad) {
        s->alpha = (float*)calloc(n, sizeof(float));
        s->delta = (float*)calloc(n, sizeof(float));
        if (!s->alpha || !s->delta) { orc_destroy(s); return NULL; }
    }
    return s;
}

void orc_destroy(orc_store* s) {
    if (!s) return;
    free(s->data); free(s->alpha); free(s->delta); free(s);
}
int64_t orc_elems(const orc_store* s) { return s->rows * s->cols; }
int32_t orc_value_size(const orc_store* s) { return s->value_size; }
void* orc_data(orc_store* s) { return s->data; }
float* orc_alpha(orc_store* s) { return s->alpha; }
float* orc_delta(orc_store* s) { return s->delta; }

int orc_error(const orc_store* s, int64_t* key, int32_t* col) {
    if (key) *key = s->err_key;
    if (col) *col = s->err_col;
    return s->err;
}

/* setAlpha (FloatMatrixStoreAdaGrad.java:77-82, setAlphaValue :96-106). */
void orc_set_alpha(orc_store* s, float initial_alpha, float min_alpha, float factor) {
    if (!s->ada_grad) return;
    int64_t n = s->rows * s->cols;
    for (int64_t i = 0; i < n; ++i) s->alpha[i] = initial_alpha;
    s->initial_alpha = initial_alpha; s->min_alpha = min_alpha; s->factor = factor;
}
void orc_max_delta(const orc_store* s, float* v, int32_t* row, int32_t* col) {
    *v = s->max_delta; *row = s->max_delta_row; *col = s->max_delta_col;
}

/* ---- handlePush ----------------------------------------------------------- */

/* Matrix stores, dense-column branch:
 *   FloatMatrixStore.handlePush/updateRow   FloatMatrixStore.java:200-222
 *   IntMatrixStore.handlePush/updateRow     IntMatrixStore.java:154-178
 *   DoubleMatrixStore.handlePush/updateRow  DoubleMatrixStore.java:153-175
 *   FloatMatrixStoreAdaGrad                 FloatMatrixStoreAdaGrad.java:239-284
 * and their sparse-column branches (:223-235, :180-192, :176-188, :285-303). */
static int push_matrix(orc_store* s, const uint8_t* data, int64_t len) {
    const int K = s->key_size, V = s->value_size;
    int64_t off = 0;
    while (off < len) {                                   /* while (offset < data.length) */
        if (off + K > len) return fail(s, ORC_E_TRUNCATED, 0, -1);   /* readKey past end */
        int64_t key = rd_key(s, data + off);
        off += K;
        int64_t idx = row_index(s, key);                  /* localData[indexOf(key)] */
        if (idx < 0) return fail(s, ORC_E_KEY_OUT_OF_SHARD, key, -1);
        size_t base = (size_t)idx * (size_t)s->cols;
        if (s->dense_column) {
            for (int32_t i = 0; i < s->cols; ++i) {
                if (off + V > len) return fail(s, ORC_E_TRUNCATED, key, i);
                if (s->value_type == 1) {
                    float u = rd_f32(data + off);
                    float* row = (float*)s->data + base;
                    row[i] = row[i] + u;                  /* row[i] += update; */
                    if (s->ada_grad) {
                        float* d = s->delta + base;
                        float* a = s->alpha + base;
                        float uu = u * u;                 /* float multiply (JLS 15.17.1) */
                        d[i] = d[i] + uu;                 /* deltas[i] += update * update; */
                        if ((double)d[i] > 1.0) {         /* if (deltas[i] > 1.0) */
                            a[i] = (float)((double)s->initial_alpha /
                                           ((double)s->factor * sqrt((double)d[i])));
                            if (a[i] < s->min_alpha) a[i] = s->min_alpha;
                        }
                        if (d[i] > s->max_delta) {        /* :273-277 */
                            s->max_delta = d[i];
                            s->max_delta_row = (int32_t)key;
                            s->max_delta_col = i;
                        }
                    }
                } else if (s->value_type == 0) {
                    int32_t* row = (int32_t*)s->data + base;
                    row[i] = (int32_t)((uint32_t)row[i] + (uint32_t)rd_i32(data + off)); /* wraps */
                    if (row[i] < 0) {                     /* IntMatrixStore.java:174-176 */
                        off += V;
                        return fail(s, ORC_E_NEGATIVE_COUNTER, key, i);
                    }
                } else {
                    double* row = (double*)s->data + base;
                    row[i] = row[i] + rd_f64(data + off);
                }
                off += V;
            }
        } else {
            if (off + 4 > len) return fail(s, ORC_E_TRUNCATED, key, -1);
            int32_t count = rd_i32(data + off);
            off += 4;
            for (int32_t i = 0; i < count; ++i) {
                if (off + 4 > len) return fail(s, ORC_E_TRUNCATED, key, -1);
                int32_t col = rd_i32(data + off);
                off += 4;
                if (off + V > len) return fail(s, ORC_E_TRUNCATED, key, col);
                /* AdaGrad's sparse branch indexes row[i] (defect 4, :293-299). */
                int32_t tgt = s->ada_grad ? i : col;
                if (tgt < 0 || tgt >= s->cols) return fail(s, ORC_E_KEY_OUT_OF_SHARD, key, tgt);
                if (s->value_type == 1) {
                    float u = rd_f32(data + off);
                    float* row = (float*)s->data + base;
                    row[tgt] = row[tgt] + u;
                    if (s->ada_grad) {
                        float* d = s->delta + base;
                        float* a = s->alpha + base;
                        float uu = u * u;
                        d[tgt] = d[tgt] + uu;
                        if ((double)d[tgt] > 1.0) {
                            a[tgt] = (float)((double)s->initial_alpha / sqrt((double)d[tgt]));
                            if (a[tgt] <= s->min_alpha) a[tgt] = s->min_alpha;
                        }
                    }
                } else if (s->value_type == 0) {
                    int32_t* row = (int32_t*)s->data + base;  /* no negativity check here (:183-191) */
                    row[tgt] = (int32_t)((uint32_t)row[tgt] + (uint32_t)rd_i32(data + off));
                } else {
                    double* row = (double*)s->data + base;
                    row[tgt] = row[tgt] + rd_f64(data + off);
                }
                off += V;
            }
        }
    }
    return ORC_OK;
}

/* Array stores:
 *   FloatArrayStore.handlePush   FloatArrayStore.java:110-122 (VALUE_SIZE :15)
 *   IntArrayStore.handlePush     IntArrayStore.java:97-113
 *   DoubleArrayStore.handlePush  DoubleArrayStore.java:115-127
 * Java evaluation order: key read, value read, then the array index. */
static int push_array(orc_store* s, const uint8_t* data, int64_t len) {
    const int K = s->key_size;
    const int VS = s->array_value_stride;
    int64_t off = 0;
    while (off < len) {
        if (off + K > len) return fail(s, ORC_E_TRUNCATED, 0, -1);
        int64_t key = rd_key(s, data + off);
        off += K;
        if (s->value_type == 1) {
            if (off + 4 > len) return fail(s, ORC_E_TRUNCATED, key, -1);   /* readFloat needs 4 bytes */
            float u = rd_f32(data + off);
            off += VS;
            int64_t idx = row_index(s, key);
            if (idx < 0) return fail(s, ORC_E_KEY_OUT_OF_SHARD, key, -1);
            float* a = (float*)s->data;
            a[idx] = a[idx] + u;
        } else if (s->value_type == 0) {
            if (off + 4 > len) return fail(s, ORC_E_TRUNCATED, key, -1);
            int32_t u = rd_i32(data + off);
            off += 4;
            int64_t idx = row_index(s, key);
            if (idx < 0) return fail(s, ORC_E_KEY_OUT_OF_SHARD, key, -1);
            int32_t* a = (int32_t*)s->data;
            a[idx] = (int32_t)((uint32_t)a[idx] + (uint32_t)u);
            if (a[idx] < 0) return fail(s, ORC_E_NEGATIVE_COUNTER, key, -1);
        } else {
            if (off + 8 > len) return fail(s, ORC_E_TRUNCATED, key, -1);
            double u = rd_f64(data + off);
            off += 8;
            int64_t idx = row_index(s, key);
            if (idx < 0) return fail(s, ORC_E_KEY_OUT_OF_SHARD, key, -1);
            double* a = (double*)s->data;
            a[idx] = a[idx] + u;
        }
    }
    return ORC_OK;
}

int orc_push(orc_store* s, const uint8_t* data, int64_t len) {
    if (len < 0 || (len > 0 && !data)) return ORC_E_INVALID_ARG;
    return s->data_type == 1 ? push_matrix(s, data, len) : push_array(s, data, len);
}

/* ---- CPU baseline: n pushes, optionally row-partitioned over threads ----- */
typedef struct {
    orc_store* s; const uint8_t* const* bufs; const int64_t* lens; int32_t n;
    int64_t row_lo, row_hi; int rc;
} part_arg;

/* One thread owns rows [row_lo,row_hi) and scans every record of every bucket
 * in push order, so each element still sees its adds in reference order.
 * Only used for dense-column fp32/int32/fp64 matrices without errors. */
static void* part_worker(void* p) {
    part_arg* a = (part_arg*)p;
    orc_store* s = a->s;
    const int K = s->key_size, V = s->value_size;
    const int64_t stride = K + (int64_t)V * s->cols;
    for (int32_t b = 0; b < a->n; ++b) {
        const uint8_t* d = a->bufs[b];
        int64_t nrec = a->lens[b] / stride;
        for (int64_t r = 0; r < nrec; ++r) {
            const uint8_t* rec = d + r * stride;
            int64_t idx = row_index(s, rd_key(s, rec));
            if (idx < a->row_lo || idx >= a->row_hi) continue;
            const uint8_t* v = rec + K;
            size_t base = (size_t)idx * s->cols;
            if (s->value_type == 1) {
                float* row = (float*)s->data + base;
                for (int32_t i = 0; i < s->cols; ++i) row[i] = row[i] + rd_f32(v + 4 * i);
            } else if (s->value_type == 0) {
                int32_t* row = (int32_t*)s->data + base;
                for (int32_t i = 0; i < s->cols; ++i) row[i] = (int32_t)((uint32_t)row[i] + (uint32_t)rd_i32(v + 4 * i));
            } else {
                double* row = (double*)s->data + base;
                for (int32_t i = 0; i < s->cols; ++i) row[i] = row[i] + rd_f64(v + 8 * i);
            }
        }
    }
    return NULL;
}

int orc_push_many(orc_store* s, const uint8_t* const* bufs, const int64_t* lens, int32_t n, int32_t threads) {
    if (threads <= 1 || s->data_type != 1 || !s->dense_column || s->ada_grad) {
        for (int32_t b = 0; b < n; ++b) {
            int rc = orc_push(s, bufs[b], lens[b]);
            if (rc) return rc;
        }
        return ORC_OK;
    }
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    part_arg args[256];
    int64_t per = (s->rows + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        args[t] = (part_arg){s, bufs, lens, n, t * per, (t + 1) * per < s->rows ? (t + 1) * per : s->rows, 0};
        pthread_create(&tid[t], NULL, part_worker, &args[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    return ORC_OK;
}

/* ---- handleFetch, dense-column layout ------------------------------------- *
 * Matrix: [key][cols x value] (FloatMatrixStore.java:140-153, IntMatrixStore.java:106-119,
 *          DoubleMatrixStore handleFetch); AdaGrad: [key][cols x (value, alpha)]
 *          (FloatMatrixStoreAdaGrad.java:173-190).
 * Array:   [key][value] with the store's VALUE_SIZE stride; FloatArrayStore writes
 *          4 value bytes into an 8-byte zeroed slot (FloatArrayStore.java:92-105).
 * Returns bytes written or -1 (key outside shard / capacity). */
int64_t orc_fetch(orc_store* s, const int64_t* keys, int64_t n, uint8_t* out, int64_t cap) {
    const int K = s->key_size, V = s->value_size;
    int64_t rec;
    if (s->data_type == 1) rec = K + (int64_t)s->cols * (s->ada_grad ? 8 : V);
    else rec = K + (s->value_type == 1 ? 8 : V);  /* FloatArrayStore VALUE_SIZE = 8 */
    if (n * rec > cap) return -1;
    memset(out, 0, (size_t)(n * rec));
    int64_t off = 0;
    for (int64_t j = 0; j < n; ++j) {
        int64_t idx = row_index(s, keys[j]);
        if (idx < 0) return -1;
        if (K == 4) wr_i32(out + off, (int32_t)keys[j]); else wr_i64(out + off, keys[j]);
        off += K;
        size_t base = (size_t)idx * s->cols;
        if (s->data_type == 1) {
            for (int32_t i = 0; i < s->cols; ++i) {
                if (s->value_type == 1) {
                    wr_f32(out + off, ((float*)s->data)[base + i]); off += 4;
                    if (s->ada_grad) { wr_f32(out + off, s->alpha[base + i]); off += 4; }
                } else if (s->value_type == 0) { wr_i32(out + off, ((int32_t*)s->data)[base + i]); off += 4; }
                else { wr_f64(out + off, ((double*)s->data)[base + i]); off += 8; }
            }
        } else {
            if (s->value_type == 1) { wr_f32(out + off, ((float*)s->data)[idx]); off += 8; }
            else if (s->value_type == 0) { wr_i32(out + off, ((int32_t*)s->data)[idx]); off += 4; }
            else { wr_f64(out + off, ((double*)s->data)[idx]); off += 8; }
        }
    }
    return off;
}

/* ---- writeAll / readAll: DataOutputStream big-endian (FloatMatrixStore.java:74-91) */
int64_t orc_write_all(orc_store* s, uint8_t* out, int64_t cap) {
    int64_t n = s->rows * s->cols, V = s->value_size;
    if (n * V > cap) return -1;
    for (int64_t i = 0; i < n; ++i) {
        if (V == 4) { uint32_t u; memcpy(&u, (uint8_t*)s->data + 4 * i, 4); wr_be32(out + 4 * i, u); }
        else {
            uint64_t u; memcpy(&u, (uint8_t*)s->data + 8 * i, 8);
            wr_be32(out + 8 * i, (uint32_t)(u >> 32)); wr_be32(out + 8 * i + 4, (uint32_t)u);
        }
    }
    return n * V;
}
int orc_read_all(orc_store* s, const uint8_t* in, int64_t len) {
    int64_t n = s->rows * s->cols, V = s->value_size;
    if (len < n * V) return ORC_E_TRUNCATED;   /* DataInputStream EOFException */
    for (int64_t i = 0; i < n; ++i) {
        if (V == 4) { uint32_t u = rd_be32(in + 4 * i); memcpy((uint8_t*)s->data + 4 * i, &u, 4); }
        else {
            uint64_t u = ((uint64_t)rd_be32(in + 8 * i) << 32) | rd_be32(in + 8 * i + 4);
            memcpy((uint8_t*)s->data + 8 * i, &u, 8);
        }
    }
    return ORC_OK;
}

/* ---- KeyRange.linearSplit (KeyRange.java:68-80) --------------------------- */
void orc_linear_split(int64_t first, int64_t last, int32_t n, int64_t* f, int64_t* l) {
    int64_t start = first;
    int64_t step = (last - first + n) / n;
    for (int32_t i = 0; i < n; ++i) {
        int64_t end = start + step - 1 < last ? start + step - 1 : last;  /* Math.min */
        f[i] = start; l[i] = end;
        start += step;
    }
}

/* ---- synthetic generators (spec: DESIGN.md §Synthetic data) ---------------- */
uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline int32_t synth_grad_int(uint64_t h) {   /* Irwin-Hall(4) of 16-bit uniforms, centred */
    int32_t s = (int32_t)(h & 0xFFFF) + (int32_t)((h >> 16) & 0xFFFF) +
                (int32_t)((h >> 32) & 0xFFFF) + (int32_t)((h >> 48) & 0xFFFF);
    return s - 131070;
}
static void put_value(uint8_t* p, int32_t vt, uint64_t h) {
    if (vt == 1) wr_f32(p, (float)synth_grad_int(h) * 0x1p-25f);
    else if (vt == 3) wr_f64(p, (double)synth_grad_int(h) * 0x1p-25);
    else wr_i32(p, (int32_t)(h % 5) - 2);
}
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) {
    return (uint64_t)(((unsigned __int128)a * b) % m);
}

void orc_synth_dense_bucket(uint8_t* out, int32_t key_type, int32_t value_type, int64_t first_key,
                            int64_t shard_rows, int64_t nrec, int32_t cols, uint64_t seed,
                            uint64_t perm_a, uint64_t perm_c) {
    const int K = key_type == 0 ? 4 : 8, V = value_type == 3 ? 8 : 4;
    const int64_t stride = K + (int64_t)V * cols;
    const uint64_t s0 = orc_splitmix64(seed);
    for (int64_t r = 0; r < nrec; ++r) {
        uint64_t row = (mulmod(perm_a, (uint64_t)r, (uint64_t)shard_rows) + perm_c) % (uint64_t)shard_rows;
        uint8_t* rec = out + r * stride;
        int64_t key = first_key + (int64_t)row;
        if (K == 4) wr_i32(rec, (int32_t)key); else wr_i64(rec, key);
        for (int32_t c = 0; c < cols; ++c)
            put_value(rec + K + (int64_t)V * c, value_type, orc_splitmix64(s0 + row * (uint64_t)cols + (uint64_t)c));
    }
}

void orc_synth_sparse_bucket(uint8_t* out, int32_t key_type, int32_t value_type, int32_t value_stride,
                             int64_t first_key, int64_t key_space, int64_t nrec, uint64_t seed,
                             uint64_t perm_a, uint64_t perm_c) {
    const int K = key_type == 0 ? 4 : 8;
    const int64_t stride = K + value_stride;
    const uint64_t s0 = orc_splitmix64(seed);
    for (int64_t r = 0; r < nrec; ++r) {
        uint64_t i = (mulmod(perm_a, (uint64_t)r, (uint64_t)key_space) + perm_c) % (uint64_t)key_space;
        uint8_t* rec = out + r * stride;
        int64_t key = first_key + (int64_t)i;
        if (K == 4) wr_i32(rec, (int32_t)key); else wr_i64(rec, key);
        memset(rec + K, 0, (size_t)value_stride);
        put_value(rec + K, value_type, orc_splitmix64(s0 + i));
    }
}

void orc_synth_fill(orc_store* s, uint64_t seed) {
    const uint64_t s0 = orc_splitmix64(seed);
    int64_t n = s->rows * s->cols;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t h = orc_splitmix64(s0 + (uint64_t)i);
        if (s->value_type == 1) ((float*)s->data)[i] = (float)((int32_t)(h % 100) - 50) * 0x1p-17f;
        else if (s->value_type == 3) ((double*)s->data)[i] = (double)((int32_t)(h % 100) - 50) * 0x1p-17;
        else ((int32_t*)s->data)[i] = 64 + (int32_t)(h % 51);
    }
}

/* ---- DoubleMatrixStore.rand() (DoubleMatrixStore.java:192-207) -----------
 * new Random(1L) per shard; per row: cols x Math.abs(nextGaussian()), the sum of
 * squares in double (row order, no FMA), Math.sqrt, then every element / sum.
 * java.util.Random is the 48-bit LCG of its published specification (Random's
 * class documentation: setSeed scramble, next(bits), nextDouble = 53 bits, and
 * nextGaussian = Marsaglia's polar method with StrictMath.log / StrictMath.sqrt).
 * StrictMath.log is fdlibm's __ieee754_log (e_log.c), restated below: glibc's log
 * is closer to correctly rounded and differs from it in ~7 % of arguments. */
typedef struct {
    uint64_t seed;
    int have_next;
    double next_next;
} jrandom;

static void jr_init(jrandom* r, int64_t seed) {
    r->seed = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
    r->have_next = 0;
    r->next_next = 0.0;
}
static int32_t jr_next(jrandom* r, int bits) {
    r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(uint32_t)(r->seed >> (48 - bits));
}
static double jr_next_double(jrandom* r) {
    const int64_t a = jr_next(r, 26), b = jr_next(r, 27);
    return (double)((a << 27) + b) * 0x1.0p-53;
}

static inline int32_t hi_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (int32_t)(u >> 32); }
static inline uint32_t lo_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double with_hi(double x, int32_t h) {
    uint64_t u; memcpy(&u, &x, 8);
    u = ((uint64_t)(uint32_t)h << 32) | (u & 0xffffffffULL);
    memcpy(&x, &u, 8);
    return x;
}

double orc_fdlibm_log(double x) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                        Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                        Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                        Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    volatile double zero = 0.0;
    int32_t hx = hi_word(x), k = 0, i, j;
    const uint32_t lx = lo_word(x);
    if (hx < 0x00100000) { /* x < 2^-1022 */
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / zero;
        if (hx < 0) return (x - x) / zero;
        k -= 54;
        x *= two54;
        hx = hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = with_hi(x, hx | (i ^ 0x3ff00000)); /* normalize x or x/2 */
    k += (i >> 20);
    const double f = x - 1.0;
    double dk, R;
    if ((0x000fffff & (2 + hx)) < 3) { /* |f| < 2^-20 */
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    dk = (double)k;
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

static double jr_next_gaussian(jrandom* r) {
    if (r->have_next) {
        r->have_next = 0;
        return r->next_next;
    }
    double v1, v2, s;
    do {
        v1 = 2 * jr_next_double(r) - 1;
        v2 = 2 * jr_next_double(r) - 1;
        s = v1 * v1 + v2 * v2;
    } while (s >= 1 || s == 0);
    const double multiplier = sqrt(-2 * orc_fdlibm_log(s) / s); /* StrictMath.sqrt: IEEE */
    r->next_next = v2 * multiplier;
    r->have_next = 1;
    return v1 * multiplier;
}

void orc_java_random_ints(int64_t seed, int32_t n, int32_t* out) {
    jrandom r;
    jr_init(&r, seed);
    for (int32_t i = 0; i < n; ++i) out[i] = jr_next(&r, 32);
}

void orc_java_random_gaussians(int64_t seed, int32_t n, double* out) {
    jrandom r;
    jr_init(&r, seed);
    for (int32_t i = 0; i < n; ++i) out[i] = jr_next_gaussian(&r);
}

int orc_rand(orc_store* s) {
    /* DataStore.rand() is a no-op (DataStore.java:22) except for the matrix stores;
     * the float matrices draw from an unseeded Random (FloatMatrixStore.java:44), which
     * no restatement can reproduce, so only DoubleMatrixStore is restated here. */
    if (s->data_type != 1 || s->value_type != 3) return ORC_E_INVALID_ARG;
    jrandom r;
    jr_init(&r, 1);
    double* d = (double*)s->data;
    const int32_t cols = s->cols;
    for (int64_t i = 0; i < s->rows; ++i) {
        double* row = d + i * cols;
        double sum = 0.0;
        for (int32_t j = 0; j < cols; ++j) {
            row[j] = fabs(jr_next_gaussian(&r));
            sum += row[j] * row[j];
        }
        sum = sqrt(sum);
        for (int32_t j = 0; j < cols; ++j) row[j] = row[j] / sum;
    }
    return ORC_OK;
}

/* ---- row-subset generators (full-size parity on sampled rows) --------------
 * The synthetic dense spec makes a full-range push's record for row `row` depend
 * only on (seed, row): orc_synth_dense_rows writes, for each sampled row rows[i],
 * the record orc_synth_dense_bucket would hold for it, keyed i (a compact store of
 * the sampled rows); orc_synth_fill_rows the orc_synth_fill values of those rows of
 * a `cols`-wide store. Per-element results of full-range pushes do not depend on
 * record order, so the compact store reproduces the sampled rows exactly. */
void orc_synth_dense_rows(uint8_t* out, int32_t key_type, int32_t value_type, const int64_t* rows, int64_t n,
                          int32_t cols, uint64_t seed) {
    const int K = key_type == 0 ? 4 : 8, V = value_type == 3 ? 8 : 4;
    const int64_t stride = K + (int64_t)V * cols;
    const uint64_t s0 = orc_splitmix64(seed);
    for (int64_t i = 0; i < n; ++i) {
        uint8_t* rec = out + i * stride;
        if (K == 4) wr_i32(rec, (int32_t)i); else wr_i64(rec, i);
        for (int32_t c = 0; c < cols; ++c)
            put_value(rec + K + (int64_t)V * c, value_type,
                      orc_splitmix64(s0 + (uint64_t)rows[i] * (uint64_t)cols + (uint64_t)c));
    }
}

void orc_synth_fill_rows(orc_store* s, const int64_t* rows, uint64_t seed) {
    const uint64_t s0 = orc_splitmix64(seed);
    for (int64_t i = 0; i < s->rows; ++i)
        for (int32_t c = 0; c < s->cols; ++c) {
            const int64_t at = i * s->cols + c;
            const uint64_t h = orc_splitmix64(s0 + (uint64_t)rows[i] * (uint64_t)s->cols + (uint64_t)c);
            if (s->value_type == 1) ((float*)s->data)[at] = (float)((int32_t)(h % 100) - 50) * 0x1p-17f;
            else if (s->value_type == 3) ((double*)s->data)[at] = (double)((int32_t)(h % 100) - 50) * 0x1p-17;
            else ((int32_t*)s->data)[at] = 64 + (int32_t)(h % 51);
        }
}
