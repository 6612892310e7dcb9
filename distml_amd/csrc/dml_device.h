// dml_device.h — device-side helpers shared by the kernel files (dml_kernels.hip,
// dml_sparse.hip): vector load types, wire decode (DataDesc.java:131-192),
// KeyRange indexOf, IEEE element adds. Not part of the public ABI.
#pragma once
#include "dml_internal.h"

namespace dml {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(4)));  // records are 4-byte aligned only
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));
typedef uint64_t u64x8 __attribute__((ext_vector_type(8)));

// Loads through the global address space: bucket pointers come out of the
// kernarg table as generic pointers, and flat loads would force vmcnt(0)+lgkmcnt(0)
// waits (flat returns out of order).
#define DML_GLOBAL __attribute__((address_space(1)))
__device__ inline u32x4 ldg16(const uint8_t* p) { return *(const DML_GLOBAL u32x4_u*)(p); }
__device__ inline uint32_t ldg32(const uint8_t* p) { return *(const DML_GLOBAL uint32_t*)(p); }
// Streamed-once bucket bytes: non-temporal policy (no L2 retention).
__device__ inline u32x4 ldg16_nt(const uint8_t* p) {
    return __builtin_nontemporal_load((const DML_GLOBAL u32x4_u*)(p));
}
__device__ inline void stg16_nt(void* p, u32x4 v) { __builtin_nontemporal_store(v, (DML_GLOBAL u32x4_u*)(p)); }
__device__ inline void stg16(void* p, u32x4 v) { *(DML_GLOBAL u32x4_u*)(p) = v; }
// Write-through 16-B store (sc1: the line leaves the XCD's L2 at once), through a
// buffer descriptor based at a wave-uniform `base` (byte offset `off` < nbytes):
// rows a kernel writes last leave no dirty L2 lines for the kernel-end writeback
// that holds up the next dispatch on the stream (MI355X_MICROARCH.md, kernel boundary).
__device__ inline void stg16_wt(const void* base, uint32_t nbytes, uint32_t off, u32x4 v) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(nbytes);
    void* ub = (void*)(((uint64_t)hi << 32) | lo);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, (int)n, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (int)off, 0, 16);
}

// Buffer resource over [base, base + nbytes) at a wave-uniform base, and its 16-B
// non-temporal load (aux 2 = nt): 32-bit per-lane offsets instead of 64-bit
// addresses, and an offset past nbytes reads zeros (the range check), so a masked
// lane needs no select.
__device__ inline __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t nbytes) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}
__device__ inline u32x4 ldb16_nt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2);
}
// A wave-uniform 64-bit value in scalar registers (the compiler then branches on it
// with scalar branches).
__device__ inline int64_t uni64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline uint64_t uni64(uint64_t v) { return (uint64_t)uni64((int64_t)v); }
constexpr uint32_t kBufOff = 0xFFFFFFF0u;  // an offset past any range: the load reads zeros

__device__ inline uint32_t ld32(const uint8_t* p) { return ldg32(p); }
__device__ inline int64_t ld_key(const uint8_t* p, int K) {
    // DataDesc.readKey (DataDesc.java:131-138): LE int32 sign-extended, or LE int64.
    if (K == 4) return (int64_t)(int32_t)ld32(p);
    return (int64_t)((uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32));
}
// KeyRange indexOf: (int)(key - firstKey) (FloatMatrixStore.java:176-179); -1 if
// localData[index] would throw ArrayIndexOutOfBoundsException.
__device__ inline int64_t row_index(int64_t key, int64_t first, int64_t rows) {
    int32_t idx = (int32_t)(uint32_t)((uint64_t)key - (uint64_t)first);
    return (idx < 0 || (int64_t)idx >= rows) ? -1 : (int64_t)idx;
}

template <typename T> struct Elem;
template <> struct Elem<float> {
    static constexpr int VEC = 4;
    __device__ static float from_bits(uint32_t lo, uint32_t) { return __uint_as_float(lo); }
    __device__ static float load(const uint8_t* p) { return __uint_as_float(ld32(p)); }
    __device__ static float add(float a, float b) { return __fadd_rn(a, b); }
};
template <> struct Elem<int32_t> {
    static constexpr int VEC = 4;
    __device__ static int32_t from_bits(uint32_t lo, uint32_t) { return (int32_t)lo; }
    __device__ static int32_t load(const uint8_t* p) { return (int32_t)ld32(p); }
    __device__ static int32_t add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
};
template <> struct Elem<double> {
    static constexpr int VEC = 2;
    __device__ static double from_bits(uint32_t lo, uint32_t hi) {
        return __longlong_as_double((long long)((uint64_t)lo | ((uint64_t)hi << 32)));
    }
    __device__ static double load(const uint8_t* p) { return from_bits(ld32(p), ld32(p + 4)); }
    __device__ static double add(double a, double b) { return __dadd_rn(a, b); }
};

}  // namespace dml
