/*
 * dml_oracle.h — CPU restatement of DistML's server-store push loops.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product path (distml_amd/, libdistml_ps)
 * never does.
 *
 * PARITY UNPINNED: the reference (Java 1.7 / Scala 2.10, Maven) cannot be built
 * or run here (no JDK in this image or on the GPU box) and ships no tests,
 * golden vectors or fixtures for this path. This oracle is
 * pinned instead by hand-derived known-answer tests written from the Java
 * Language Specification (tests/golden/kat_*.json, tests/test_oracle_kat.py).
 *
 * Semantics restated (each function cites the Java it follows):
 *  - little-endian record decode            DataDesc.java:180-212
 *  - KeyRange row index (int)(key-firstKey) FloatMatrixStore.java:176-186
 *  - sequential `row[i] += v` in record and push order, one IEEE rounding per
 *    add, no FMA contraction (JLS 15.18.2), int32 wrap (JLS 15.18.2)
 *  - int32 negativity check after each add   IntMatrixStore.java:174-176
 *  - AdaGrad delta/alpha update, alpha in double  FloatMatrixStoreAdaGrad.java:262-278
 *  - exceptions: the loop stops at the first failing access with every earlier
 *    add applied (Java evaluation order), reported as a status code.
 */
#ifndef DML_ORACLE_H
#define DML_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OK 0
#define ORC_E_BAD_DESC 1
#define ORC_E_KEY_OUT_OF_SHARD 2
#define ORC_E_TRUNCATED 3
#define ORC_E_NEGATIVE_COUNTER 4
#define ORC_E_INVALID_ARG 16

typedef struct orc_store orc_store;

orc_store* orc_create(int32_t data_type, int32_t key_type, int32_t value_type,
                      int32_t dense_column, int32_t ada_grad,
                      int64_t first_key, int64_t last_key, int32_t cols,
                      int32_t float_array_ref_stride);
void orc_destroy(orc_store* s);
int64_t orc_elems(const orc_store* s);
int32_t orc_value_size(const orc_store* s);
void* orc_data(orc_store* s);
float* orc_alpha(orc_store* s);
float* orc_delta(orc_store* s);

int orc_push(orc_store* s, const uint8_t* data, int64_t len);
int orc_error(const orc_store* s, int64_t* key, int32_t* col);
void orc_set_alpha(orc_store* s, float initial_alpha, float min_alpha, float factor);
void orc_max_delta(const orc_store* s, float* v, int32_t* row, int32_t* col);

int64_t orc_fetch(orc_store* s, const int64_t* keys, int64_t n, uint8_t* out, int64_t cap);
int64_t orc_write_all(orc_store* s, uint8_t* out, int64_t cap);
int orc_read_all(orc_store* s, const uint8_t* in, int64_t len);

void orc_linear_split(int64_t first, int64_t last, int32_t n, int64_t* f, int64_t* l);

/* Synthetic generators: the same byte spec as libdistml_ps's dml_synth_* (DESIGN.md). */
uint64_t orc_splitmix64(uint64_t x);
void orc_synth_dense_bucket(uint8_t* out, int32_t key_type, int32_t value_type, int64_t first_key,
                            int64_t shard_rows, int64_t nrec, int32_t cols, uint64_t seed,
                            uint64_t perm_a, uint64_t perm_c);
void orc_synth_sparse_bucket(uint8_t* out, int32_t key_type, int32_t value_type, int32_t value_stride,
                             int64_t first_key, int64_t key_space, int64_t nrec, uint64_t seed,
                             uint64_t perm_a, uint64_t perm_c);
void orc_synth_fill(orc_store* s, uint64_t seed);
/* The same generators restricted to sampled rows (record i / store row i = rows[i]). */
void orc_synth_dense_rows(uint8_t* out, int32_t key_type, int32_t value_type, const int64_t* rows, int64_t n,
                          int32_t cols, uint64_t seed);
void orc_synth_fill_rows(orc_store* s, const int64_t* rows, uint64_t seed);

/* DoubleMatrixStore.rand() (DoubleMatrixStore.java:192-207): java.util.Random(1L),
 * |nextGaussian()| rows scaled to unit norm; ORC_E_INVALID_ARG for other stores.
 * The pieces, for known-answer tests: Random(seed).nextInt() x n,
 * Random(seed).nextGaussian() x n, and fdlibm's log (StrictMath.log). */
int orc_rand(orc_store* s);
void orc_java_random_ints(int64_t seed, int32_t n, int32_t* out);
void orc_java_random_gaussians(int64_t seed, int32_t n, double* out);
double orc_fdlibm_log(double x);

/* Bench baseline: n sequential pushes, timed by the caller; optional threads>1
 * runs the dense matrix loop row-partitioned over OpenMP-free pthreads. */
int orc_push_many(orc_store* s, const uint8_t* const* bufs, const int64_t* lens, int32_t n, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif
