// dml_kernels.hip — CDNA4 (gfx950) kernels of the parameter-server push path.
//
// Compiled with -ffp-contract=off and IEEE denormals (Java forbids FMA
// contraction and flush-to-zero, JLS 15.4 / 4.2.3): every `acc + v` below is
// one IEEE binary32/binary64 rounding, exactly the reference's `row[i] += v`.
//
// Kernels
//   k_index         decode record keys -> per-row slot table (row -> record of push b)
//   k_reduce<T,M>   ordered multi-push reduce: every element of a shard row
//                   summed over the batch's pushes in push order, one RMW of
//                   the row (FloatMatrixStore.java:210-222, IntMatrixStore.java:164-178,
//                   DoubleMatrixStore.java:163-175, FloatMatrixStoreAdaGrad.java:249-284)
//   k_array_rollback int32 array stores: undo every add after the first negative
//                   counter (IntArrayStore.java:97-113); the arrays' ordered
//                   scatter-add itself is the partition + leaf path of dml_sparse.hip
//   k_fetch, k_bswap, k_fill, k_apply_dense, k_synth_*  — fetch / checkpoint /
//                   init / owner-apply / synthetic data.
#include "dml_device.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <climits>
#include <cstdlib>

namespace dml {

// Shapes measured against their alternatives (alternating builds on one box, DESIGN.md
// §4 and profiles/r05_ab_*.txt); the rejected variants (block barriers before the
// write-back, dispatch-order blocks, occupancy caps) are in the history, not here.
constexpr int kC5Wpb = 2, kC5Rpw = 4;  // k_reduce_rows DEPTH 3 (config 5): waves per block, rows per wave
constexpr int kD3Waves = 1;            // DEPTH 3: minimum waves per SIMD its registers must allow
constexpr int kAdaFlatWaves = 4;       // k_ada_flat: waves per block

__host__ __device__ inline uint64_t splitmix64_dev(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t splitmix64(uint64_t x) { return splitmix64_dev(x); }
thread_local const char* g_kernel_name = nullptr;

template <typename T>
__device__ inline void unpack(const u32x4& r, T* o) {
    if constexpr (sizeof(T) == 4) {
        o[0] = Elem<T>::from_bits(r.x, 0); o[1] = Elem<T>::from_bits(r.y, 0);
        o[2] = Elem<T>::from_bits(r.z, 0); o[3] = Elem<T>::from_bits(r.w, 0);
    } else {
        o[0] = Elem<T>::from_bits(r.x, r.y); o[1] = Elem<T>::from_bits(r.z, r.w);
    }
}
template <typename T>
__device__ inline u32x4 pack(const T* v) {
    u32x4 r;
    if constexpr (sizeof(T) == 4) {
        r.x = __builtin_bit_cast(uint32_t, v[0]); r.y = __builtin_bit_cast(uint32_t, v[1]);
        r.z = __builtin_bit_cast(uint32_t, v[2]); r.w = __builtin_bit_cast(uint32_t, v[3]);
    } else {
        uint64_t a = __builtin_bit_cast(uint64_t, v[0]), b = __builtin_bit_cast(uint64_t, v[1]);
        r.x = (uint32_t)a; r.y = (uint32_t)(a >> 32); r.z = (uint32_t)b; r.w = (uint32_t)(b >> 32);
    }
    return r;
}

// ---------------------------------------------------------------------------
// k_index: one thread per record of push b (blockIdx.y): slot[row][b] = record.
// A key outside the shard lowers ctrl->cutoff to the record's start position.
// Rows listed twice by one push are flagged (rowflag[row] = 1): atomicExch sees
// the earlier record; the reduce skips those rows and the host replays just
// them through the exact layered path.
// A bounded grid walks the (push, 256-record chunk) tasks: the launch dispatches at
// most kIndexBlocks blocks even when every push skips (identity / reused pushes of a
// speculative chunk), instead of one block per chunk of every push — 8 192 waves for
// config 2, which at the sharded path's high stream priority took dispatch slots from
// the running pre-reduce (its pieces 352-369 us against 331-347 us with the index at
// normal priority).
constexpr int kIndexBlocks = 512;
__global__ __launch_bounds__(256) void k_index(const Batch bt, int nb, int64_t nchunk, int64_t stride, int K,
                                               int64_t first, int64_t rows, int32_t* __restrict__ slot,
                                               uint32_t* __restrict__ rowflag, Ctrl* __restrict__ ctrl,
                                               uint64_t tail_cut) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && tail_cut != kNoPos)
        atomicMin(&ctrl->cutoff, (unsigned long long)tail_cut);
    const uint64_t ident = (bt.spec || bt.ident_ok) ? ctrl->ident : 0ull;
    for (int64_t t = blockIdx.x; t < (int64_t)nb * nchunk; t += gridDim.x) {
        const int b = (int)(t / nchunk);
        // identity push: the reduce verifies its keys (spec), or k_ident_full did (ident_ok)
        if ((ident >> b) & 1ull) continue;  // uniform
        const int64_t r = (t - (int64_t)b * nchunk) * 256 + threadIdx.x;
        if (r >= bt.nrec[b]) continue;
        const int64_t off = r * stride;
        const int64_t key = ld_key(bt.base[b] + off, K);
        const int64_t idx = row_index(key, first, rows);
        if (idx < 0) {
            atomicMin(&ctrl->cutoff, (unsigned long long)pos_of((uint64_t)bt.bidx[b], (uint64_t)off));
            continue;
        }
        if (bt.listed) const_cast<uint8_t*>(bt.listed)[idx] = 1u;  // every writer stores the same byte
        const int32_t old = atomicExch(&slot[idx * slot_stride(nb) + ctrl_col(ctrl, b)], (int32_t)r);
        if (old != -1 && !bt.keeps) {
            rowflag[idx] = 1u;
            ctrl->no_dup = 0u;  // benign race: every writer stores the same value
        }
    }
}

// k_ident_check: one 64-lane block per push of a speculative chunk. Push b stays
// an identity candidate if it is full-range (nrec == rows) and the records at 32
// evenly spaced positions (first and last included) plus 32 hashed ones hold row
// r at record r. Otherwise, when the workspace kept verified permutations
// (Batch::kept_cols), the push is matched by content to a kept column: the kept
// columns whose entry for the row of record 0 is 0 are the candidates (one slot-row
// load), its own position's column first, and the first candidate that maps every
// sampled record's row to that record becomes Ctrl::col[b]. Arrival order does not
// matter (PSAgent's selector applies pushes as they arrive, PSAgent.java:166-186).
// Cheap (64 key lines and a few slot lines per push); the reduce verifies every record.
__global__ __launch_bounds__(64) void k_ident_check(const Batch bt, int64_t stride, int K, int64_t first, int64_t rows,
                                                    const int32_t* __restrict__ slot, Ctrl* __restrict__ ctrl) {
    const int b = blockIdx.x, t = threadIdx.x;
    const int ss = slot_stride((int)gridDim.x);
    const bool full = bt.nrec[b] == rows && rows > 0;  // block-uniform
    int64_t r = 0, idx = -1;
    if (full) {
        r = t < 32 ? (rows > 1 ? (int64_t)t * (rows - 1) / 31 : 0)
                   : (int64_t)(splitmix64_dev(((uint64_t)b << 32) + (uint64_t)t) % (uint64_t)rows);
        idx = row_index(ld_key(bt.base[b] + r * stride, K), first, rows);
    }
    const bool ident = full && __ballot(idx != r) == 0ull;
    int col = -1;
    if (full && !ident && bt.kept_cols) {
        // sample t = 0 is record 0
        const int32_t idx0 = __shfl((int32_t)idx, 0);
        uint64_t cand = 0;
        if (idx0 >= 0) {
            const bool c = t < ss && ((bt.kept_cols >> t) & 1ull) && slot[(int64_t)idx0 * ss + t] == 0;
            cand = __ballot(c);
        }
        // the column of the same position first (a worker arriving in its usual place)
        if ((cand >> b) & 1ull) {
            if (__ballot(!(idx >= 0 && slot[idx * ss + b] == (int32_t)r)) == 0ull) col = b;
            cand &= ~(1ull << b);
        }
        while (col < 0 && cand) {
            const int c = (int)__builtin_ctzll(cand);
            cand &= cand - 1;
            if (__ballot(!(idx >= 0 && slot[idx * ss + c] == (int32_t)r)) == 0ull) col = c;
        }
    }
    if (t == 0) {
        unsigned long long clear = (ident || col >= 0) ? 0ull : (1ull << b);
        if (b == 0 && gridDim.x < 64) clear |= ~((1ull << gridDim.x) - 1ull);  // no such push
        if (clear) atomicAnd(&ctrl->ident, ~clear);
        if (col >= 0) ctrl->col[b] = (unsigned char)col;
    }
}
hipError_t launch_ident_check(const Batch& bt, int nb, int64_t stride, int K, int64_t first, int64_t rows,
                              const int32_t* slot, Ctrl* ctrl, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ident_check, dim3((unsigned)nb), dim3(64), 0, st, bt, stride, K, first, rows, slot, ctrl);
    return hipGetLastError();
}

// k_assign_cols (one wave, lane b = push b): the pushes k_ident_check neither
// verified as identity nor matched to a kept column are indexed; each keeps its own
// column when no matched push reads it, the others take the lowest free columns in
// push order. A chunk of nb pushes has slot_stride(nb) >= nb columns and at most nb
// of them are taken, so every push gets one. (One thread walking the pushes took
// 32-45 us on the next call's index chain beside a running reduce: a chain of
// dependent byte loads; here one load per lane.)
__global__ __launch_bounds__(64) void k_assign_cols(Ctrl* __restrict__ ctrl, int nb) {
    const int b = threadIdx.x;
    const unsigned long long id = ctrl->ident;
    const bool live = b < nb;
    const bool matched = live && ((id >> b) & 1ull);
    const unsigned col = live ? ctrl->col[b] : 0xFFu;
    uint64_t used = (matched && col != 0xFFu) ? 1ull << col : 0ull;  // columns matched pushes read
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) used |= (uint64_t)__shfl_xor((unsigned long long)used, m);
    const bool indexed = live && !matched;
    const bool need = indexed && ((used >> b) & 1ull);  // its own column is read by a matched push
    const uint64_t keep = __ballot(indexed && !need);   // pushes that keep their own column
    const uint64_t needs = __ballot(need);
    used |= keep;
    if (need) {
        // the k-th pushes needing a column (in push order) takes the k-th lowest free one
        int k = __popcll(needs & ((1ull << b) - 1ull));
        uint64_t freec = ~used;
        while (k-- > 0) freec &= freec - 1;
        ctrl->col[b] = (unsigned char)__builtin_ctzll(freec);
    }
}
hipError_t launch_assign_cols(Ctrl* ctrl, int nb, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_assign_cols, dim3(1), dim3(64), 0, st, ctrl, nb);
    return hipGetLastError();
}

// k_ident_full: one thread per record of a push still marked identity; any record r
// whose key is not row r clears the push's bit (the push's later blocks then stop
// at the bit).
__global__ __launch_bounds__(256) void k_ident_full(const Batch bt, int64_t stride, int K, int64_t first, int64_t rows,
                                                    Ctrl* __restrict__ ctrl) {
    const int b = blockIdx.y;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= bt.nrec[b] || !((ctrl->ident >> b) & 1ull)) return;
    if (row_index(ld_key(bt.base[b] + r * stride, K), first, rows) != r)
        atomicAnd(&ctrl->ident, ~(1ull << b));
}
hipError_t launch_ident_full(const Batch& bt, int nb, int64_t max_nrec, int64_t stride, int K, int64_t first,
                             int64_t rows, Ctrl* ctrl, hipStream_t st) {
    if (nb <= 0 || max_nrec <= 0) return hipSuccess;
    dim3 grid((unsigned)((max_nrec + 255) / 256), (unsigned)nb);
    hipLaunchKernelGGL(k_ident_full, grid, dim3(256), 0, st, bt, stride, K, first, rows, ctrl);
    return hipGetLastError();
}

hipError_t launch_index(const Batch& bt, int nb, int64_t max_nrec, int64_t stride, int K, int64_t first,
                        int64_t rows, int32_t* slot, uint32_t* rowflag, Ctrl* ctrl, uint64_t tail_cut, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    const int64_t nchunk = std::max<int64_t>(1, (max_nrec + 255) / 256);
    const unsigned grid = (unsigned)std::min<int64_t>(kIndexBlocks, nchunk * nb);
    hipLaunchKernelGGL(k_index, dim3(grid), dim3(256), 0, st, bt, nb, nchunk, stride, K, first, rows, slot, rowflag,
                       ctrl, tail_cut);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// AdaGrad maxDelta candidates: (valid, value, position), best = largest value,
// then smallest position (the first in the reference's order). Associative, so
// a block reduces them as a butterfly inside each wave, then across its waves
// through LDS; the result lands in thread 0. Every thread of the block calls it.
__device__ inline bool cand_better(bool ok, float v, uint64_t p, bool ok2, float v2, uint64_t p2) {
    return ok && (!ok2 || v > v2 || (v == v2 && p < p2));
}
template <int WPB>
__device__ inline void cand_block_best(bool& ok, float& v, uint64_t& p) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        const float ov = __shfl_xor(v, m);
        const uint32_t olo = (uint32_t)__shfl_xor((int)(uint32_t)p, m);
        const uint32_t ohi = (uint32_t)__shfl_xor((int)(uint32_t)(p >> 32), m);
        const bool ook = __shfl_xor((int)ok, m) != 0;
        const uint64_t op = (uint64_t)olo | ((uint64_t)ohi << 32);
        if (cand_better(ook, ov, op, ok, v, p)) { ok = true; v = ov; p = op; }
    }
    if constexpr (WPB > 1) {
        __shared__ float sv[WPB];
        __shared__ uint64_t sp[WPB];
        __shared__ int sok[WPB];
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { sv[w] = v; sp[w] = p; sok[w] = ok; }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 1; i < WPB; ++i)
                if (cand_better(sok[i] != 0, sv[i], sp[i], ok, v, p)) { ok = true; v = sv[i]; p = sp[i]; }
    }
}

// ---------------------------------------------------------------------------
// k_reduce: one wave per (shard row, CPW consecutive 64*VEC-column chunks); a
// block = WPB waves. The wave reads the row's slots (wave-uniform scalar loads),
// keeps its row chunks in registers, adds every push's values in push order
// (G pushes x CPW chunks of 16-B loads in flight per lane), then writes the row
// chunks once. With CPW > 1 one wave walks neighbouring 1-KiB chunks of a record
// in consecutive load instructions, so the line two chunks share is requested
// back to back (merged) instead of by two waves (fetched twice under nt loads).
// Elements at or past the batch cutoff (first key/truncation error) are not
// applied — the state the reference leaves when its exception escapes.
template <typename T, int MODE, int G, bool NT, int WPB, bool SNT, int CPW>
__global__ __launch_bounds__(64 * WPB) void k_reduce(T* __restrict__ shard, int64_t rows, int32_t cols, int32_t ngroups,
                                                const Batch bt, int nb, int64_t stride, int K,
                                                const int32_t* __restrict__ slot, const uint32_t* __restrict__ rowflag,
                                                Ctrl* __restrict__ ctrl, uint64_t tail_cut, AdaArgs ada, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    constexpr int SG = G < 8 ? 8 : G;  // slots fetched per scalar round (multiple of 8)
    static_assert(G == 2 || G == 4 || G == 8 || G == 16, "push groups of 2, 4, 8 or 16");
    static_assert(CPW == 1 || CPW == 2 || CPW == 4, "1, 2 or 4 chunks per wave");
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t task = (int64_t)blockIdx.x * WPB + wid;
    const int64_t ntask = rows * (int64_t)ngroups;

    // AdaGrad maxDelta candidate of this lane.
    float cand_v = 0.f;
    uint64_t cand_p = kNoPos;
    bool cand_ok = false;

    if (task < ntask) do {
        if (bt.prev && ctrl_abnormal(bt.prev)) break;  // predecessor needs the host first
        const int64_t trow = task / ngroups;
        const int cg = (int)(task - trow * ngroups);
        const int64_t row = rm.row(trow);
        T* const rowp = rm.out ? (T*)rm.out + trow * (int64_t)cols : shard + row * (int64_t)cols;
        if (rm.block && row >= rm.rows_total) {  // padding row of a short last shard
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const int32_t cc = ((cg * CPW + c) * 64 + lane) * VEC;
                for (int e = 0; e < VEC; ++e)
                    if (cc + e < cols) rowp[cc + e] = T(0);
            }
            break;
        }
        if (rowflag && rowflag[row]) break;  // a push repeats this row: the host replays it exactly

        int32_t c0[CPW];
        int nv[CPW], sh[CPW];
        int64_t voff[CPW], shb[CPW];
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            c0[c] = ((cg * CPW + c) * 64 + lane) * VEC;
            nv[c] = c0[c] < cols ? (cols - c0[c] < VEC ? cols - c0[c] : VEC) : 0;
            // a ragged row's last lane loads the 16 B that END at its last element
            // (in bounds: c0 >= VEC - nv) and shifts them down by sh elements
            sh[c] = nv[c] > 0 ? VEC - nv[c] : 0;
            shb[c] = (int64_t)sh[c] * (int64_t)sizeof(T);
            voff[c] = (int64_t)K + (int64_t)c0[c] * (int64_t)sizeof(T);  // value offset inside a record
        }
        if (nv[0] == 0) break;  // lanes past the row's last column idle

        uint64_t cut = ctrl->cutoff;
        if (tail_cut < cut) cut = tail_cut;
        const int cut_b = cut == kNoPos ? INT_MAX : (int)(cut >> 40);  // global push index of the cutoff
        const uint64_t cut_off = cut & kOffMask;
        uint64_t negcut = kNoPos;
        if (MODE == kRollbackI32) {
            negcut = ctrl->neg_pos;
            if (negcut == kNoPos) break;
        }
        const int32_t* srow = slot + row * slot_stride(nb);

        T acc[CPW][VEC];
        // AdaGrad: delta; the delta after the last push that left it above 1 (0 =
        // none); the last strict rise of delta (value, batch position).
        float dl[CPW][VEC], lg[CPW][VEC], rv[CPW][VEC];
        uint64_t rp[CPW][VEC];
        bool touched = false;
        bool negf = false;
        uint64_t negpos = kNoPos;

        auto load_row = [&]() {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                T* prow = rowp + c0[c];
                if (MODE == kPreReduce) {
#pragma unroll
                    for (int e = 0; e < VEC; ++e) acc[c][e] = T(0);
                } else if (nv[c] == VEC) {
                    const u32x4 t = SNT ? ldg16_nt((const uint8_t*)prow) : ldg16((const uint8_t*)prow);
                    unpack<T>(t, acc[c]);
                } else {
#pragma unroll
                    for (int e = 0; e < VEC; ++e) acc[c][e] = e < nv[c] ? prow[e] : T(0);
                }
                if constexpr (MODE == kAdaGrad) {
                    const int64_t ei = row * (int64_t)cols + c0[c];
                    if (nv[c] == VEC) {
                        const u32x4 t = SNT ? ldg16_nt((const uint8_t*)(ada.delta + ei))
                                            : ldg16((const uint8_t*)(ada.delta + ei));
                        unpack<float>(t, dl[c]);
                    }
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        if (nv[c] != VEC) dl[c][e] = e < nv[c] ? ada.delta[ei + e] : 0.f;
                        lg[c][e] = 0.f;
                        rv[c][e] = 0.f;
                        rp[c][e] = kNoPos;
                    }
                }
            }
        };

        // One contribution u to element (c, e) at batch position p.
        auto apply = [&](int c, int e, T u, uint64_t p) {
            if constexpr (MODE == kRollbackI32) {
                if (p > negcut) acc[c][e] = (T)((uint32_t)acc[c][e] - (uint32_t)u);
            } else {
                acc[c][e] = Elem<T>::add(acc[c][e], u);
                if constexpr (MODE == kAddCheckI32) {
                    if (!negf && acc[c][e] < 0) { negf = true; negpos = p; }
                }
                if constexpr (MODE == kAdaGrad) {
                    // FloatMatrixStoreAdaGrad.java:265-277. Every push whose delta ends
                    // above 1 overwrites alpha with f(delta), others leave it: the alpha
                    // the batch leaves is f(the last such delta), computed once at
                    // write-back instead of a double sqrt + divide per push. delta never
                    // falls (u*u >= 0; NaN never rises), so the last strict rise is the
                    // element's maxDelta candidate.
                    const float uu = __fmul_rn((float)u, (float)u);
                    const float nd = __fadd_rn(dl[c][e], uu);
                    if (nd > dl[c][e]) { rv[c][e] = nd; rp[c][e] = p; }
                    if (nd > 1.0f) lg[c][e] = nd;
                    dl[c][e] = nd;
                }
            }
        };

        const bool vec_ok = cols >= VEC;  // wave-uniform: vector loads for every active lane
        for (int b0 = 0; b0 < nb; b0 += SG) {
            // Wave-uniform scalar loads of 8 slots / push indices / bases at once;
            // every index < kMaxW is in bounds of the slot row and the kernarg table.
            int32_t rr[SG];
            int gbv[SG];
            const uint8_t* bp[SG];
#pragma unroll
            for (int h = 0; h < SG; h += 8) {
                const i32x8 sv = *(const i32x8*)(srow + b0 + h);
                const i32x8 gv = *(const i32x8*)(&bt.bidx[b0 + h]);
                const u64x8 pv = *(const u64x8*)(&bt.base[b0 + h]);
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const bool in = b0 + h + g < nb;
                    gbv[h + g] = in ? gv[g] : INT_MAX;
                    bp[h + g] = (const uint8_t*)pv[g];
                    rr[h + g] = (in && gbv[h + g] <= cut_b) ? sv[g] : -1;
                }
            }
            bool any = false;
#pragma unroll
            for (int g = 0; g < SG; ++g) any |= rr[g] >= 0;
            if (!any) continue;
            if (!touched) { load_row(); touched = true; }

#pragma unroll
            for (int s0 = 0; s0 < SG; s0 += G) {
                bool sub = false;
#pragma unroll
                for (int g = 0; g < G; ++g) sub |= rr[s0 + g] >= 0;
                if (!sub) continue;
                int glast = s0;  // last live push of this sub-group (absent ones carry INT_MAX)
#pragma unroll
                for (int g = 0; g < G; ++g) glast = b0 + s0 + g < nb ? s0 + g : glast;
                if (vec_ok && gbv[glast] < cut_b) {
                    // Fast path: G x CPW independent 16-B loads in flight, no branches
                    // between them; an absent slot / empty chunk re-reads the row start.
                    u32x4 raw[G][CPW];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
#pragma unroll
                        for (int c = 0; c < CPW; ++c) {
                            const bool live = rr[s0 + g] >= 0 && nv[c] > 0;
                            const uint8_t* src =
                                live ? bp[s0 + g] + (int64_t)rr[s0 + g] * stride + voff[c] - shb[c] : (const uint8_t*)rowp;
                            raw[g][c] = NT ? ldg16_nt(src) : ldg16(src);
                        }
                    }
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        if (rr[s0 + g] < 0) continue;  // wave-uniform
#pragma unroll
                        for (int c = 0; c < CPW; ++c) {
                            T t[VEC], u[VEC];
                            unpack<T>(raw[g][c], t);
#pragma unroll
                            for (int e = 0; e < VEC; ++e) {  // u[e] = t[e + sh] without runtime register indexing
                                u[e] = t[e];
#pragma unroll
                                for (int k = 1; k < VEC - e; ++k) u[e] = sh[c] == k ? t[e + k] : u[e];
                            }
                            const uint64_t pb =
                                pos_of((uint64_t)gbv[s0 + g], (uint64_t)((int64_t)rr[s0 + g] * stride + voff[c]));
#pragma unroll
                            for (int e = 0; e < VEC; ++e)
                                if (e < nv[c]) apply(c, e, u[e], pb + (uint64_t)(e * (int)sizeof(T)));
                        }
                    }
                } else {
                    // Generic path: rows narrower than one vector, or the group holding the cutoff push.
                    for (int g = 0; g < G; ++g) {
                        if (rr[s0 + g] < 0) continue;
                        const int gb = gbv[s0 + g];
#pragma unroll
                        for (int c = 0; c < CPW; ++c) {
                            const int64_t roff = (int64_t)rr[s0 + g] * stride + voff[c];
                            for (int e = 0; e < nv[c]; ++e) {
                                const uint64_t off = (uint64_t)(roff + e * (int64_t)sizeof(T));
                                if (gb == cut_b && off >= cut_off) break;
                                apply(c, e, Elem<T>::load(bp[s0 + g] + off), pos_of((uint64_t)gb, off));
                            }
                        }
                    }
                }
            }
        }

        if constexpr (MODE == kAdaGrad) {
            // Hand the slot table back clean (reduce_clears_slots): with one chunk group
            // per row this wave is the row's only reader and its slot reads are done.
            if (ngroups == 1) {
                const int nact = (cols + VEC - 1) / VEC < 64 ? (cols + VEC - 1) / VEC : 64;  // live lanes
                for (int j = lane; j < nb; j += nact) const_cast<int32_t*>(slot)[row * slot_stride(nb) + j] = -1;
            }
        }
        if (MODE == kPreReduce && !touched) {
#pragma unroll
            for (int c = 0; c < CPW; ++c)
#pragma unroll
                for (int e = 0; e < VEC; ++e) acc[c][e] = T(0);
            touched = true;
        }
        if (touched) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                T* prow = rowp + c0[c];
                if (nv[c] == VEC) {
                    if (SNT) stg16_nt(prow, pack<T>(acc[c]));
                    else stg16(prow, pack<T>(acc[c]));
                } else {
                    for (int e = 0; e < nv[c]; ++e) prow[e] = acc[c][e];
                }
                if constexpr (MODE == kAdaGrad) {
                    const int64_t ei = row * (int64_t)cols + c0[c];
                    float na[VEC];
                    bool all_a = nv[c] == VEC;
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        na[e] = 0.f;
                        if (e < nv[c] && lg[c][e] > 1.0f) {
                            na[e] = (float)((double)ada.initial_alpha / ((double)ada.factor * sqrt((double)lg[c][e])));
                            if (na[e] < ada.min_alpha) na[e] = ada.min_alpha;
                        } else {
                            all_a = false;
                        }
                    }
                    if (nv[c] == VEC) {
                        if (SNT) stg16_nt(ada.delta + ei, pack<float>(dl[c]));
                        else stg16(ada.delta + ei, pack<float>(dl[c]));
                    }
                    if (all_a) {  // every element's alpha changed: one 16-B store
                        if (SNT) stg16_nt(ada.alpha + ei, pack<float>(na));
                        else stg16(ada.alpha + ei, pack<float>(na));
                    }
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        if (e >= nv[c]) continue;
                        if (nv[c] != VEC) ada.delta[ei + e] = dl[c][e];
                        if (!all_a && lg[c][e] > 1.0f) ada.alpha[ei + e] = na[e];
                        if (rp[c][e] != kNoPos &&
                            (!cand_ok || rv[c][e] > cand_v || (rv[c][e] == cand_v && rp[c][e] < cand_p))) {
                            cand_ok = true; cand_v = rv[c][e]; cand_p = rp[c][e];
                        }
                    }
                }
            }
        }
        if (MODE == kAddCheckI32 && negf) atomicMin(&ctrl->neg_pos, (unsigned long long)negpos);
    } while (0);

    if constexpr (MODE == kAdaGrad) {
        cand_block_best<WPB>(cand_ok, cand_v, cand_p);
        if (threadIdx.x == 0) {
            DeltaCand c;
            c.value = cand_v; c.valid = cand_ok; c.pos = cand_p;
            ada.cand[blockIdx.x] = c;
        }
    }
}

// ---------------------------------------------------------------------------
// Blocks are dealt to the 8 XCDs round robin (block b on XCD b % 8), each XCD with
// its own L2. xcd_block() renumbers them so that XCD x runs the x-th contiguous run
// of block indices, in dispatch order: neighbouring blocks' data meets in one L2.
// A bijection on [0, gridDim.x) for any grid size.
__device__ inline int64_t xcd_block() {
    const int64_t nbk = gridDim.x, b = blockIdx.x, per = (nbk + 7) / 8, x = b % 8, i = b / 8;
    const int64_t full = nbk - (per - 1) * 8;  // XCDs 0..full-1 hold `per` blocks, the others per - 1
    return x < full ? x * per + i : full * per + (x - full) * (per - 1) + i;
}

// k_reduce_rows: the plain-sum shapes (kAdd, kAddCheckI32, kPreReduce) with
// RPW neighbouring rows per wave. One push at a time: the wave scalar-loads the
// push's base / index and its RPW slots, issues RPW x CPW 16-B nt loads (16 for
// config 2: four whole records), then adds them in push order. Fewer, longer
// waves whose shard reads and write-backs come in RPW x larger bursts: measured
// +8..20 % over one row per wave on config 2 (scripts/ubench_reduce.hip).
// A batch with a cutoff (key / truncation error) takes a register-light
// element-wise path instead (in-place RMW of the wave's own rows, same order),
// so the hot loop carries no cutoff logic. Same results as k_reduce bit for bit
// (same per-element add order, cutoff and negativity rules); rows narrower than
// one vector use k_reduce.
template <typename T, int MODE, int CPW, int RPW, bool NT, bool FULL, int DEPTH, int WPB = 4, int SNT = 0>
__global__ __launch_bounds__(64 * WPB, DEPTH == 3 ? kD3Waves : 1) void k_reduce_rows(T* __restrict__ shard, int64_t rows, int32_t cols,
                                                     int32_t ngroups, const Batch bt, int nb, int64_t stride, int K,
                                                     int32_t* __restrict__ slot,
                                                     const uint32_t* __restrict__ rowflag, Ctrl* __restrict__ ctrl,
                                                     uint64_t tail_cut, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    static_assert(MODE == kAdd || MODE == kAddCheckI32 || MODE == kPreReduce, "plain-sum modes only");
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // DEPTH 3 (rows that are not whole lines, e.g. config 5's 4000-B rows): XCD-
    // contiguous blocks, so the line two neighbouring rows share is written from one
    // L2 (config 5 0.635 -> 0.653 of 8 TB/s, 3 rounds on one box)
    const int64_t blk = DEPTH == 3 ? xcd_block() : (int64_t)blockIdx.x;
    const int64_t task = blk * WPB + wid;
    const int64_t ntask = (rows + RPW - 1) / RPW * (int64_t)ngroups;
    if (task >= ntask) return;
    if (bt.prev && ctrl_abnormal(bt.prev)) return;  // predecessor needs the host first
    const int64_t tb = task / ngroups;
    const int cg = (int)(task - tb * ngroups);

    int32_t c0[CPW];
    int nv[CPW], sh[CPW];
    int64_t voff[CPW], shb[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        c0[c] = ((cg * CPW + c) * 64 + lane) * VEC;
        // FULL: cols is a multiple of 64*VEC*CPW (every lane owns whole vectors; the
        // chunk offsets fold into the loads' immediate offsets)
        nv[c] = FULL ? VEC : c0[c] < cols ? (cols - c0[c] < VEC ? cols - c0[c] : VEC) : 0;
        sh[c] = nv[c] > 0 ? VEC - nv[c] : 0;  // ragged last lane: load the 16 B ending at its last element
        shb[c] = (int64_t)sh[c] * (int64_t)sizeof(T);
        voff[c] = (int64_t)K + (int64_t)c0[c] * (int64_t)sizeof(T);
    }
    // Lanes past the row's last column (nv == 0) stay in the wave: every access
    // below is guarded by nv, and the batch table below is read from all 64 lanes.

    int64_t row[RPW];
    T* rowp[RPW];
    unsigned live = 0;
    const uint8_t* fb = nullptr;  // a readable address inside a live row (target of absent loads)
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int64_t trow = tb * RPW + r;
        const int64_t tr = trow < rows ? trow : tb * RPW;
        row[r] = rm.row(tr);
        rowp[r] = rm.out ? (T*)rm.out + tr * (int64_t)cols : shard + row[r] * (int64_t)cols;
        if (trow >= rows) continue;
        if (rm.block && row[r] >= rm.rows_total) {  // padding row of a short last shard: zeros
#pragma unroll
            for (int c = 0; c < CPW; ++c)
#pragma unroll
                for (int e = 0; e < VEC; ++e)
                    if (e < nv[c]) rowp[r][c0[c] + e] = T(0);
            continue;
        }
        // a push repeats this row: the host replays it exactly (a keeping chunk's index
        // flags nothing: no dependent flag load ahead of the row loads)
        if (rowflag && !bt.keeps && rowflag[row[r]]) continue;
        // a row no push of the chunk lists: its shard row is neither read nor written
        // (the index marked the listed ones; the load runs beside the flag load above)
        if (MODE != kPreReduce && bt.listed && !bt.listed[row[r]]) continue;
        live |= 1u << r;
        if (!fb) fb = (const uint8_t*)rowp[r];
    }
    if (!live) return;

    uint64_t cut = ctrl->cutoff;
    if (tail_cut < cut) cut = tail_cut;
    uint64_t negpos = kNoPos;  // kAddCheckI32: earliest add that left a counter negative
    // Identity speculation (Batch::spec): pushes in ctrl->ident take slot = row and
    // every such record's key is verified below; a chunk that met a cutoff or a
    // repeated row turns into a no-op the host re-runs without speculation.
    uint64_t ident = 0;
    bool bad = false;
    // (the sharded pre-reduce speculates the same way: a failed verification re-runs
    // the call's pieces before its partial is reduce-scattered, dml_prereduce_verify)
    constexpr bool kSpecMode = MODE == kAdd || MODE == kPreReduce;
    if constexpr (kSpecMode) {
        if (bt.spec) {
            if (cut != kNoPos || ctrl->no_dup == 0u) {
                if (lane == 0) ctrl->spec_ok = 0u;
                return;
            }
            ident = ctrl->ident;
        }
    }
    if constexpr (MODE == kPreReduce)
        if (bt.ident_ok) ident = ctrl->ident;  // verified before the launch: slot = row, no key checks

    if (cut != kNoPos) {
        // Error batch: element-wise RMW of the wave's rows in place, pushes in order,
        // stopping at the cutoff byte (the state the reference leaves when it throws).
        const int cut_b = (int)(cut >> 40);
        const uint64_t cut_off = cut & kOffMask;
        for (int r = 0; r < RPW; ++r) {
            if (!(live >> r & 1u)) continue;
            T* const rp = rowp[r];
            if (MODE == kPreReduce)
                for (int c = 0; c < CPW; ++c)
                    for (int e = 0; e < nv[c]; ++e) rp[c0[c] + e] = T(0);
            const int32_t* srow = slot + row[r] * slot_stride(nb);
            for (int b = 0; b < nb; ++b) {
                const int gb = bt.bidx[b];
                if (gb > cut_b) break;
                const int32_t rr = srow[b];
                if (rr < 0) continue;
                for (int c = 0; c < CPW; ++c)
                    for (int e = 0; e < nv[c]; ++e) {
                        const uint64_t off = (uint64_t)((int64_t)rr * stride + voff[c] + e * (int64_t)sizeof(T));
                        if (gb == cut_b && off >= cut_off) break;
                        const T v = Elem<T>::add(rp[c0[c] + e], Elem<T>::load(bt.base[b] + off));
                        rp[c0[c] + e] = v;
                        if (MODE == kAddCheckI32 && v < 0) {
                            const uint64_t p = pos_of((uint64_t)gb, off);
                            if (p < negpos) negpos = p;
                        }
                    }
            }
        }
        if (MODE == kAddCheckI32 && negpos != kNoPos) atomicMin(&ctrl->neg_pos, (unsigned long long)negpos);
        return;
    }

    // The wave's shard rows, loaded up front (a row no push lists is read but not written).
    T acc[RPW][CPW][VEC];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const bool ld = MODE != kPreReduce && (live >> r & 1u);
            // the input row: in place, or the speculative chunk's input buffer
            const T* const lrow = (MODE == kAdd && bt.src) ? (const T*)bt.src + row[r] * (int64_t)cols : rowp[r];
            if (ld && nv[c] == VEC) {
                unpack<T>(ldg16((const uint8_t*)(lrow + c0[c])), acc[r][c]);
            } else {
#pragma unroll
                for (int e = 0; e < VEC; ++e) acc[r][c][e] = ld && e < nv[c] ? lrow[c0[c] + e] : T(0);
            }
        }
    unsigned touched = 0;
    const uint8_t* const fbv = fb + (int64_t)c0[0] * (int64_t)sizeof(T);  // FULL: absent rows re-read a live row
    // The batch table in registers, lane j = push j (kMaxW == 64 == wave size): the
    // rows' slots and the push bases, read per push with v_readlane (no scalar-memory
    // round trip between two pushes' loads). All 64 lanes are active here (no lane
    // has returned), so every lane v_readlane reads holds its value.
    static_assert(kMaxW == 64, "one push per lane");
    int32_t vslot[RPW];
    // lanes >= nb read past the row's entries (another row's): masked to -1;
    // an identity push (speculation) holds row r at record r when r < nrec;
    // every other push reads its column (Ctrl::col: its own, or the kept column a
    // slot-reuse push was matched to, verified like an identity push)
    const bool lane_ident = lane < nb && ctrl_identity(ctrl, ident, lane);
    const int lcol = lane < nb ? ctrl_col(ctrl, lane) : lane;
#pragma unroll
    for (int r = 0; r < RPW; ++r)
        vslot[r] = ((live >> r & 1u) && lane < nb)
                       ? (lane_ident ? (row[r] < bt.nrec[lane] ? (int32_t)row[r] : -1) : slot[row[r] * slot_stride(nb) + lcol])
                       : -1;
    if (!bt.spec && ngroups == 1) {
        // Hand the slot rows back as the next batch's index expects them (-1 = no
        // record), so the host skips the slot-table memset (reduce_clears_slots); the
        // int32 rollback (rare) rebuilds the table with a second index. Only when this
        // wave is its rows' one reader (rows wider than CPW chunks have several). A
        // speculative chunk keeps its table: its full-range columns are permutations
        // the next chunk in this workspace may reuse (Batch::kept_cols). Entries read
        // as -1 are left alone: a row no push lists costs no write (config 5: 11 % of
        // the shard's rows, one 128-B slot line each).
#pragma unroll
        for (int r = 0; r < RPW; ++r)
            if ((live >> r & 1u) && lane < nb && (lane_ident || vslot[r] >= 0))
                slot[row[r] * slot_stride(nb) + lcol] = -1;
    }
    const uint64_t vbase = lane < nb ? (uint64_t)bt.base[lane] : 0ull;
    // Speculative chunks verify identity records through lane 63 of the wave's last
    // chunk when that lane owns no column (spec_idle, wave-uniform): its load of the
    // record start carries the key at no extra instruction; otherwise one key load.
    const bool spec_idle = !FULL && ident != 0ull && ((cg * CPW + CPW - 1) * 64 + 63) * VEC >= cols;
    const bool spec_lane = spec_idle && lane == 63;
    // One record vector into a row chunk, as the reference adds it (one add per element).
    // Whole-vector rows (cols % VEC == 0, wave-uniform): no lane is ragged, so no shift
    // select; a lane past the row's last column adds what it loaded and never stores it.
    // kAddCheckI32: the counters after every add are OR-ed into negbits (one instruction
    // per element); the first negative's position is found after the loop, only when
    // some lane saw one (rare), by replaying the wave's adds from the shard (neg_first).
    const bool aligned = FULL || cols % VEC == 0;
    uint32_t negbits = 0;
    auto add_vec = [&](T (&a)[VEC], const u32x4& rw, int c) {
        T t[VEC];
        unpack<T>(rw, t);
        if (aligned) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) a[e] = Elem<T>::add(a[e], t[e]);
            if constexpr (MODE == kAddCheckI32)
                negbits |= nv[c] > 0 ? ((uint32_t)a[0] | (uint32_t)a[1] | (uint32_t)a[2] | (uint32_t)a[3]) : 0u;
        } else {
            T u[VEC];
#pragma unroll
            for (int e = 0; e < VEC; ++e) {  // u[e] = t[e + sh] without runtime register indexing
                u[e] = t[e];
#pragma unroll
                for (int k = 1; k < VEC - e; ++k) u[e] = sh[c] == k ? t[e + k] : u[e];
            }
#pragma unroll
            for (int e = 0; e < VEC; ++e)
                if (e < nv[c]) {
                    a[e] = Elem<T>::add(a[e], u[e]);
                    if constexpr (MODE == kAddCheckI32) negbits |= (uint32_t)a[e];
                }
        }
    };
    if constexpr (DEPTH == 3) {
        // Pair-packed: the wave's (push, row) records in push order, RPW of them per
        // load group whatever push they come from. A batch whose pushes list few of
        // these rows (LDA's and Word2Vec's touched-row pushes) keeps RPW x CPW loads in
        // flight instead of one push's mostly absent rows; full pushes give exactly
        // the push-major groups. Per row the adds stay in push order.
        uint64_t pm[RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) pm[r] = __ballot(lane < nb && vslot[r] >= 0);  // wave-uniform
        for (;;) {
            int pb[RPW], pr[RPW];
            int np = 0;
#pragma unroll
            for (int g = 0; g < RPW; ++g) {
                int bmin = 64, rsel = 0;  // the lowest push any row still holds, its first row
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    const int tz = pm[r] ? (int)__builtin_ctzll(pm[r]) : 64;
                    if (tz < bmin) { bmin = tz; rsel = r; }
                }
                pb[g] = bmin;
                pr[g] = rsel;
                if (bmin < 64) {
#pragma unroll
                    for (int r = 0; r < RPW; ++r)
                        if (r == rsel) pm[r] &= pm[r] - 1;  // bmin is its lowest set bit
                    ++np;
                }
            }
            if (np == 0) break;
            u32x4 raw[RPW][CPW];
            int32_t prr[RPW];
            int64_t kv[RPW];  // identity verification: the key each group element read
#pragma unroll
            for (int g = 0; g < RPW; ++g) {
                const int b = pb[g] < 64 ? pb[g] : 0;
                int32_t vs = vslot[0];
#pragma unroll
                for (int r = 1; r < RPW; ++r) vs = pr[g] == r ? vslot[r] : vs;
                const int32_t rr = pb[g] < 64 ? __builtin_amdgcn_readlane(vs, b) : -1;
                prr[g] = rr;
                const uint8_t* bp =
                    (const uint8_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vbase, b)) |
                                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vbase >> 32), b) << 32));
                if constexpr (FULL) {
                    const uint8_t* rb = rr >= 0 ? bp + (int64_t)rr * stride + voff[0] : fbv;
#pragma unroll
                    for (int c = 0; c < CPW; ++c) {
                        const uint8_t* src = rb + c * 64 * VEC * (int)sizeof(T);
                        raw[g][c] = NT ? ldg16_nt(src) : ldg16(src);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < CPW; ++c) {
                        // an idle lane of the last chunk (spec_lane) loads the record's key
                        // for the identity verification instead of a dummy address
                        const uint8_t* src = (rr >= 0 && nv[c] > 0) ? bp + (int64_t)rr * stride + voff[c] - shb[c]
                                             : (c == CPW - 1 && spec_lane && rr >= 0) ? bp + (int64_t)rr * stride
                                                                                     : fb;
                        raw[g][c] = NT ? ldg16_nt(src) : ldg16(src);
                    }
                }
                if constexpr (MODE == kAdd) {
                    // wave-uniform: the identity record's key, compared after the adds (an
                    // early compare would wait for this group's loads before the next is issued)
                    kv[g] = bt.first;
                    if (rr >= 0 && ((ident >> b) & 1ull) && !spec_idle) kv[g] = ld_key(bp + (int64_t)rr * stride, K);
                }
            }
#pragma unroll
            for (int g = 0; g < RPW; ++g) {
                if (pb[g] >= 64) continue;  // wave-uniform
                touched |= 1u << pr[g];
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    if (r != pr[g]) continue;  // wave-uniform: static register indices below
#pragma unroll
                    for (int c = 0; c < CPW; ++c) add_vec(acc[r][c], raw[g][c], c);
                }
            }
            if constexpr (MODE == kAdd) {
                if (ident) {
#pragma unroll
                    for (int g = 0; g < RPW; ++g) {
                        if (pb[g] >= 64 || prr[g] < 0 || !((ident >> pb[g]) & 1ull)) continue;  // wave-uniform
                        int64_t rw = row[0];
#pragma unroll
                        for (int r = 1; r < RPW; ++r) rw = pr[g] == r ? row[r] : rw;
                        int64_t k = kv[g];
                        if (spec_idle) {
                            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)raw[g][CPW - 1].x, 63);
                            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)raw[g][CPW - 1].y, 63);
                            k = K == 4 ? (int64_t)(int32_t)lo : (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
                        }
                        bad |= row_index(k, bt.first, rows) != rw;
                    }
                }
            }
        }
    } else
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        int32_t rr[RPW];
        unsigned has = 0;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            rr[r] = __builtin_amdgcn_readlane(vslot[r], b);
            has |= (rr[r] >= 0 ? 1u : 0u) << r;
        }
        // a slot-keeping chunk: every live row of every (full-range) push has a record
        if (kSpecMode && bt.keeps && (has & live) != live) bad = true;
        if (!has) continue;
        touched |= has;
        const uint8_t* bp = (const uint8_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vbase, b)) |
                                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vbase >> 32), b) << 32));
        u32x4 raw[RPW][CPW];
        int64_t kv[RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if constexpr (kSpecMode) {
                // identity / reused push (every push of a keeping chunk): verify the key
                // of every record taken as row r
                kv[r] = bt.spec && (bt.keeps || ((ident >> b) & 1ull)) && rr[r] >= 0
                            ? ld_key(bp + (int64_t)rr[r] * stride, K)
                            : bt.first + row[r];
            }
            if constexpr (FULL) {
                // one address per row; the chunks are immediate offsets of the loads
                const uint8_t* rb = rr[r] >= 0 ? bp + (int64_t)rr[r] * stride + voff[0] : fbv;
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    const uint8_t* src = rb + c * 64 * VEC * (int)sizeof(T);
                    raw[r][c] = NT ? ldg16_nt(src) : ldg16(src);
                }
            } else {
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    const uint8_t* src =
                        (rr[r] >= 0 && nv[c] > 0) ? bp + (int64_t)rr[r] * stride + voff[c] - shb[c] : fb;
                    raw[r][c] = NT ? ldg16_nt(src) : ldg16(src);
                }
            }
        }
        if constexpr (kSpecMode) {
#pragma unroll
            for (int r = 0; r < RPW; ++r) bad |= row_index(kv[r], bt.first, rm.block ? rm.rows_total : rows) != row[r];
        }
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if (rr[r] < 0) continue;  // wave-uniform
#pragma unroll
            for (int c = 0; c < CPW; ++c) add_vec(acc[r][c], raw[r][c], c);
        }
    }

    if constexpr (MODE == kAddCheckI32) {
        // neg_first: some add left a counter negative. Replay this wave's adds element by
        // element from the shard rows (still unwritten: this wave stores them below), in
        // push order, and take the earliest position that left a counter negative (min
        // over positions = first in the reference's order, IntMatrixStore.java:172-176).
        // The push loop is outermost and wave-uniform, so each push's slot of row r is read
        // once, with every lane active; a lane's elements keep their running
        // sums in registers, so the adds per element stay in push order.
        if (__ballot((int32_t)negbits < 0)) {
            for (int r = 0; r < RPW; ++r) {
                if (!(touched >> r & 1u)) continue;
                T a[CPW][VEC];
#pragma unroll
                for (int c = 0; c < CPW; ++c)
#pragma unroll
                    for (int e = 0; e < VEC; ++e) a[c][e] = e < nv[c] ? rowp[r][c0[c] + e] : T(0);
                for (int b = 0; b < nb; ++b) {
                    const int32_t rrb = __builtin_amdgcn_readlane(vslot[r], b);
                    if (rrb < 0) continue;  // wave-uniform
#pragma unroll
                    for (int c = 0; c < CPW; ++c)
#pragma unroll
                        for (int e = 0; e < VEC; ++e) {
                            if (e >= nv[c]) continue;
                            const uint64_t off = (uint64_t)((int64_t)rrb * stride + voff[c] + e * (int64_t)sizeof(T));
                            a[c][e] = Elem<T>::add(a[c][e], Elem<T>::load(bt.base[b] + off));
                            if (a[c][e] < 0) {
                                const uint64_t p = pos_of((uint64_t)bt.bidx[b], off);
                                if (p < negpos) negpos = p;
                            }
                        }
                }
            }
        }
    }
    if (MODE == kPreReduce) touched = live;  // every pre-reduce row is written (zeros if no push has it)
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        if (!(touched >> r & 1u)) continue;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            T* prow = rowp[r] + c0[c];
            if (nv[c] == VEC) {
                if constexpr (SNT == 1) {
                    stg16_nt(prow, pack<T>(acc[r][c]));
                } else if constexpr (SNT == 2) {
                    stg16_wt(rowp[r], (uint32_t)(cols * (int)sizeof(T)), (uint32_t)(c0[c] * (int)sizeof(T)),
                             pack<T>(acc[r][c]));
                } else {
                    stg16(prow, pack<T>(acc[r][c]));
                }
            } else {
#pragma unroll
                for (int e = 0; e < VEC; ++e)
                    if (e < nv[c]) prow[e] = acc[r][c][e];
            }
        }
    }
    if (MODE == kAddCheckI32 && negpos != kNoPos) atomicMin(&ctrl->neg_pos, (unsigned long long)negpos);
    if (kSpecMode && bad) ctrl->spec_ok = 0u;  // an identity push is not: the host re-runs the chunk
}

// ---------------------------------------------------------------------------
// k_reduce_flat: plain sums (kAdd / kPreReduce) of rows narrower than 4 KiB
// whose pushes list most rows (config 4's 800-B Word2Vec rows). A wave owns R
// neighbouring rows, R = min(16, 512 / (cols / VEC)), and maps their R x cols
// elements onto its 64 lanes as one flat run of 16-B vectors: lane l, step j
// owns vector j*64 + l, so every lane works (k_reduce_rows leaves 14 of 64 lanes
// idle at 200 columns) and the shard block is read and written as one
// contiguous span. The wave's slot rows sit in LDS; per push a lane reads its
// vector's record from there and issues up to JMAX 16-B loads, then adds them in
// push order (one IEEE rounding per add, the reference's order per element).
// Same results as k_reduce_rows bit for bit: same cutoff, repeated-row,
// pre-reduce row-map and identity-speculation rules (an identity push's record r
// is row r; lanes 0..R-1 load the R records' keys beside the round's vector loads
// of the same lines and verify them after the adds).
template <typename T, int MODE, int JMAX, int PB>
__global__ __launch_bounds__(256) void k_reduce_flat(T* __restrict__ shard, int64_t rows, int32_t cols, int32_t R,
                                                     const Batch bt, int nb, int64_t stride, int K,
                                                     int32_t* __restrict__ slot, const uint32_t* __restrict__ rowflag,
                                                     Ctrl* __restrict__ ctrl, uint64_t tail_cut, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    constexpr int RMAX = 16;
    static_assert(MODE == kAdd || MODE == kPreReduce, "plain sums only");
    __shared__ int32_t s_slot[4][RMAX * kMaxW];  // per wave: [row][push], -1 = no record / skipped row
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-contiguous blocks (xcd_block): the line two neighbouring waves' rows share is
    // written from one L2 (config-4 leg 0.692 -> 0.704 of 8 TB/s, 2 rounds)
    const int64_t t0 = (xcd_block() * 4 + wid) * R;  // first task row of the wave
    if (t0 >= rows) return;
    if (bt.prev && ctrl_abnormal(bt.prev)) return;  // predecessor needs the host first
    uint64_t cut = ctrl->cutoff;
    if (tail_cut < cut) cut = tail_cut;
    uint64_t ident = 0;  // identity speculation (Batch::spec), see k_reduce_rows
    {
        if (bt.spec) {
            if (cut != kNoPos || ctrl->no_dup == 0u) {
                if (lane == 0) ctrl->spec_ok = 0u;
                return;
            }
            ident = ctrl->ident;
        }
    }
    if constexpr (MODE == kPreReduce)
        if (bt.ident_ok) ident = ctrl->ident;  // verified before the launch (k_ident_full)
    const int NV = cols / VEC;
    const int nrow = (int)(rows - t0 < (int64_t)R ? rows - t0 : (int64_t)R);
    const int ss = slot_stride(nb);
    int32_t* const ls = s_slot[wid];
    auto model_row = [&](int64_t t) { return rm.row(t); };
    auto out_ptr = [&](int rlj, int cvj) {
        const int64_t t = t0 + rlj;
        return (rm.out ? (T*)rm.out + t * (int64_t)cols : shard + model_row(t) * (int64_t)cols) + cvj * VEC;
    };
    // speculative verification: lane l < nrow checks the record of task row t0 + l,
    // model row lrow (its row map evaluated once, not per push round)
    const int64_t lrow = model_row(t0 + lane);
    const bool lchk = lane < nrow && !(rm.block && lrow >= rm.rows_total);  // padding rows have no record
    const int64_t vrows = rm.block ? rm.rows_total : rows;
    // bit rl of padm / flg: task row t0 + rl is padding of a short last shard / a row a
    // push repeats (one flag load per row; a keeping chunk's index flags nothing)
    const uint32_t padm = (uint32_t)__ballot(lane < nrow && rm.block && lrow >= rm.rows_total);
    const uint32_t flg =
        (rowflag && !bt.keeps) ? (uint32_t)__ballot(lane < nrow && !((padm >> lane) & 1u) && rowflag[lrow] != 0u) : 0u;
    // the wave's slot rows into LDS (rows a push repeats, and padding rows, stay -1;
    // the table is handed back clean for the next batch's index)
    for (int e = lane; e < nrow * nb; e += 64) {
        const int rl = e / nb, b = e - rl * nb;
        const int64_t mr = model_row(t0 + rl);
        int32_t v = -1;
        if (!(((padm | flg) >> rl) & 1u)) {
            if (ctrl_identity(ctrl, ident, b)) {  // identity push: record = row
                v = mr < bt.nrec[b] ? (int32_t)mr : -1;
            } else {
                const int cb = ctrl_col(ctrl, b);
                v = slot[mr * ss + cb];
                // a speculative chunk keeps its table (Batch::kept_cols, see k_reduce_rows)
                if (!bt.spec && v >= 0) slot[mr * ss + cb] = -1;
            }
        }
        ls[rl * kMaxW + b] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // this lane's vectors: (row << 16 | vector within the row); bit j of `on` / `wr`:
    // the vector belongs to a row this batch updates / is written back
    int rc[JMAX];
    uint32_t on = 0, wr = 0;
    T acc[JMAX][VEC];
    const int nvec = nrow * NV;
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
        const int v = j * 64 + lane;
        const int rlj = v < nvec ? v / NV : 0;
        const int cvj = v < nvec ? v - rlj * NV : 0;
        rc[j] = (rlj << 16) | cvj;
        const int64_t mr = model_row(t0 + rlj);
        const bool pad = (padm >> rlj) & 1u;
        const bool flagged = (flg >> rlj) & 1u;
        const bool o = v < nvec && !pad && !flagged;
        on |= (o ? 1u : 0u) << j;
        wr |= ((v < nvec && (MODE == kPreReduce ? !flagged : o)) ? 1u : 0u) << j;
        if (MODE != kPreReduce && o) {
            // the input row: in place, or the speculative chunk's input buffer
            const T* const ip = (MODE == kAdd && bt.src) ? (const T*)bt.src + mr * (int64_t)cols + cvj * VEC
                                                         : out_ptr(rlj, cvj);
            unpack<T>(ldg16((const uint8_t*)ip), acc[j]);
        } else {
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[j][e] = T(0);
        }
    }
    bool bad = false;
    if (cut != kNoPos) {
        // error batch: element by element, pushes in order, up to the cutoff byte
        const int cut_b = (int)(cut >> 40);
        const uint64_t cut_off = cut & kOffMask;
        for (int j = 0; j < JMAX; ++j) {
            if (!(on >> j & 1u)) continue;
            for (int b = 0; b < nb; ++b) {
                const int gb = bt.bidx[b];
                if (gb > cut_b) break;
                const int32_t rr = ls[(rc[j] >> 16) * kMaxW + b];
                if (rr < 0) continue;
                for (int e = 0; e < VEC; ++e) {
                    const uint64_t off = (uint64_t)((int64_t)rr * stride + K +
                                                    (int64_t)((rc[j] & 0xFFFF) * VEC + e) * (int64_t)sizeof(T));
                    if (gb == cut_b && off >= cut_off) break;
                    acc[j][e] = Elem<T>::add(acc[j][e], Elem<T>::load(bt.base[b] + off));
                }
            }
        }
    } else {
        // PB pushes per round: all their loads in flight, then added push by push
#pragma unroll 1
        for (int b0 = 0; b0 < nb; b0 += PB) {
            int32_t rr[PB][JMAX];
            u32x4 raw[PB][JMAX];
            int64_t kv[PB];  // identity pushes: lane l < nrow holds record t0+l's key
#pragma unroll
            for (int p = 0; p < PB; ++p) {
                const int b = b0 + p < nb ? b0 + p : nb - 1;
                const uint8_t* const bp = bt.base[b];
                {
                    // verified pushes (identity, reused, or every push of a slot-keeping
                    // chunk): lane l < nrow loads the key of row t0+l's record
                    const bool kl = bt.spec && b0 + p < nb && (bt.keeps || ((ident >> b) & 1ull)) && lane < nrow;
                    const int32_t kr = kl ? ls[lane * kMaxW + b] : 0;
                    kv[p] = !kl ? bt.first + lrow
                                : kr >= 0 ? ld_key(bp + (int64_t)kr * stride, K) : bt.first - 1;  // no record: fails
                }
#pragma unroll
                for (int j = 0; j < JMAX; ++j) {
                    rr[p][j] = (b0 + p < nb && (on >> j & 1u)) ? ls[(rc[j] >> 16) * kMaxW + b] : -1;
                    const uint8_t* src = bp + (int64_t)(rr[p][j] >= 0 ? rr[p][j] : 0) * stride + K +
                                         (int64_t)(rc[j] & 0xFFFF) * 16;
                    raw[p][j] = rr[p][j] >= 0 ? ldg16_nt(src) : u32x4{0u, 0u, 0u, 0u};
                }
            }
#pragma unroll
            for (int p = 0; p < PB; ++p)
#pragma unroll
                for (int j = 0; j < JMAX; ++j) {
                    if (rr[p][j] < 0) continue;
                    T u[VEC];
                    unpack<T>(raw[p][j], u);
#pragma unroll
                    for (int e = 0; e < VEC; ++e) acc[j][e] = Elem<T>::add(acc[j][e], u[e]);
                }
            if (bt.spec && (ident || bt.keeps)) {
#pragma unroll
                for (int p = 0; p < PB; ++p) bad |= lchk && row_index(kv[p], bt.first, vrows) != lrow;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < JMAX; ++j)
        if (wr >> j & 1u) {
            // non-temporal for the pre-reduce partial too: world-1 config-4 call
            // 28.61-28.66 -> 28.03-28.27 ms against cached stores (same box, 2 rounds)
            stg16_nt(out_ptr(rc[j] >> 16, rc[j] & 0xFFFF), pack<T>(acc[j]));
        }
    if (bad) ctrl->spec_ok = 0u;  // an identity push is not: the host re-runs the chunk
}

// k_flat_ident: k_reduce_flat for the chunks the host has seen to be all identity
// after the index (every push full-range, verified record r = row r, no cutoff, no
// repeated row: config 4's steady state), with nothing else in it. Same row / vector
// ownership and the same adds in push order (bit-identical to k_reduce_flat), but
//  - record offsets from the wave's first model row are 32-bit per-lane constants
//    every push shares (buffer loads at a wave-uniform base; a lane without a vector
//    reads zeros from the range check), no slot table, no LDS;
//  - a ring of D pushes in flight: push b+D-1's loads are issued before push b's
//    adds, so a wave never drains to zero between pushes;
//  - the block's waves write their rows after a block barrier: the shard's writes
//    leave a CU in one burst instead of trickling between the pushes' reads. Writes
//    interleaved with this read stream cost ~2.4 TB/s marginal against ~6.8 for reads
//    (scripts/ubench_flat.hip): the burst is what this kernel gains most from.
// Keys of every record are still verified (speculative chunks): a mismatch clears
// ctrl->spec_ok and the host re-runs the chunk exactly, as for k_reduce_flat.
template <typename T, int MODE, int J, int D, int NW>
__global__ __launch_bounds__(NW * 64) void k_flat_ident(T* __restrict__ shard, int64_t rows, int32_t cols, int32_t R,
                                                        const Batch bt, int nb, int64_t stride, int K,
                                                        Ctrl* __restrict__ ctrl, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    static_assert(MODE == kAdd || MODE == kPreReduce, "plain sums only");
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t t0 = (xcd_block() * NW + wid) * R;
    // every wave reaches the block barrier below: a wave past the last row does no
    // work; one behind a predecessor that needs the host first reads its rows (the
    // check does not hold up the loads) and writes nothing
    const bool inr = t0 < rows;
    const int nrow = !inr ? 0 : (int)(rows - t0 < (int64_t)R ? rows - t0 : (int64_t)R);
    const int NV = cols / VEC, nvec = nrow * NV;
    const int64_t mr0 = inr ? uni64(rm.row(t0)) : 0;
    const int64_t mrl = inr ? uni64(rm.row(t0 + nrow - 1)) : 0;
    // per lane j: record offset from record mr0 (push buffers), element offset from
    // row mr0 (input shard) and from the output base; kBufOff = no vector here
    uint32_t loff[J], soff[J], ooff[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int v = j * 64 + lane;
        const int rl = v / NV, cv = v - rl * NV;
        const bool on = v < nvec;
        const int64_t mr = on ? rm.row(t0 + rl) : mr0;
        const bool pad = rm.block && mr >= rm.rows_total;  // padding row of a short last shard
        loff[j] = on && !pad ? (uint32_t)((mr - mr0) * stride + K + cv * 16) : kBufOff;
        soff[j] = on && !pad ? (uint32_t)(((mr - mr0) * cols + cv * VEC) * (int64_t)sizeof(T)) : kBufOff;
        const int64_t orow = rm.out ? (int64_t)rl : mr - mr0;
        ooff[j] = on ? (uint32_t)((orow * cols + cv * VEC) * (int64_t)sizeof(T)) : kBufOff;
    }
    const uint32_t span = (uint32_t)((mrl - mr0 + 1) * stride);  // records mr0 .. mrl
    const uint32_t sspan = (uint32_t)((mrl - mr0 + 1) * cols * (int64_t)sizeof(T));
    T acc[J][VEC];
    bool bad = false;
    if (inr) {
        if constexpr (MODE == kAdd) {
            // the input rows: in place, or the speculative chunk's input buffer
            const T* const ib = (bt.src ? (const T*)bt.src : shard) + mr0 * cols;
            const __amdgpu_buffer_rsrc_t is = buf_rsrc(ib, sspan);
#pragma unroll
            for (int j = 0; j < J; ++j) unpack<T>(ldb16_nt(is, soff[j]), acc[j]);
        } else {
#pragma unroll
            for (int j = 0; j < J; ++j)
#pragma unroll
                for (int e = 0; e < VEC; ++e) acc[j][e] = T(0);
        }
        // key verification: lane l < nrow checks the record of task row t0 + l
        const int64_t lrow = rm.row(t0 + lane);
        const bool lchk = bt.spec && lane < nrow && !(rm.block && lrow >= rm.rows_total);
        const int64_t vrows = rm.block ? rm.rows_total : rows;
        const uint32_t koff = lchk ? (uint32_t)((lrow - mr0) * stride) : kBufOff;
        u32x4 ring[D][J];
        uint32_t key[D];
        auto issue = [&](int b, u32x4 (&raw)[J], uint32_t& k) {
            const __amdgpu_buffer_rsrc_t rs = buf_rsrc(bt.base[b] + mr0 * stride, span);
            k = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)koff, 0, 2);  // the key's low word
#pragma unroll
            for (int j = 0; j < J; ++j) raw[j] = ldb16_nt(rs, loff[j]);
        };
        auto add = [&](const u32x4 (&raw)[J], uint32_t k, int b) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                T u[VEC];
                unpack<T>(raw[j], u);
#pragma unroll
                for (int e = 0; e < VEC; ++e) acc[j][e] = Elem<T>::add(acc[j][e], u[e]);
            }
            if (lchk) {
                // 8-byte keys: the high word beside the low one (one more load, rare shape)
                const int64_t kv =
                    K == 4 ? (int64_t)(int32_t)k
                           : (int64_t)((uint64_t)k | ((uint64_t)ld32(bt.base[b] + lrow * stride + 4) << 32));
                bad |= row_index(kv, bt.first, vrows) != lrow;
            }
        };
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if (d < nb) issue(d, ring[d], key[d]);
#pragma unroll 1
        for (int b0 = 0; b0 < nb; b0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int b = b0 + d, bn = b + D - 1;  // bn's loads go to slot (d + D - 1) % D
                if (bn < nb) issue(bn, ring[(d + D - 1) % D], key[(d + D - 1) % D]);
                if (b < nb) add(ring[d], key[d], b);
            }
        }
    }
    // every wave of the block has read its rows: the block's writes leave together
    __syncthreads();
    if (!inr || (bt.prev && ctrl_abnormal(bt.prev))) return;
    T* const ob = rm.out ? (T*)rm.out + t0 * (int64_t)cols : shard + mr0 * cols;
    const __amdgpu_buffer_rsrc_t os = buf_rsrc(ob, rm.out ? (uint32_t)(nrow * cols * (int64_t)sizeof(T)) : sspan);
#pragma unroll
    for (int j = 0; j < J; ++j) __builtin_amdgcn_raw_buffer_store_b128(pack<T>(acc[j]), os, (int)ooff[j], 0, 2);
    if (bad) ctrl->spec_ok = 0u;  // an identity push is not: the host re-runs the chunk
}

// k_ada_flat: FloatMatrixStoreAdaGrad's push (FloatMatrixStoreAdaGrad.java:262-277)
// in k_reduce_flat's layout, for rows narrower than 4 KiB whose pushes list most
// rows (config 4's AdaGrad variant: 800-B rows). k_reduce gives such a row one
// wave with 50 of 64 lanes busy and a few KiB of traffic — 10 M short waves per
// batch; here a wave owns R neighbouring rows as one flat run of 16-B vectors
// (JMAX per lane) and keeps, per element, data, delta, the last delta above 1
// (alpha at write-back) and the last strict rise of delta (its maxDelta
// candidate, with the push that made it; the position is rebuilt from the slot
// rows in LDS at the end). Same per-element arithmetic and order as k_reduce, so
// the results (data, alpha, delta, maxDelta/row/col) are the same bit for bit.
template <int JMAX, int PB, int NW>
__global__ __launch_bounds__(NW * 64) void k_ada_flat(float* __restrict__ shard, int64_t rows, int32_t cols, int32_t R,
                                                  const Batch bt, int nb, int64_t stride, int K,
                                                  int32_t* __restrict__ slot, const uint32_t* __restrict__ rowflag,
                                                  Ctrl* __restrict__ ctrl, uint64_t tail_cut, AdaArgs ada) {
    constexpr int VEC = 4;
    constexpr int RMAX = 16;
    __shared__ int32_t s_slot[NW][RMAX * kMaxW];  // per wave: [row][push], -1 = no record / skipped row
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-contiguous blocks (xcd_block): config-4 AdaGrad leg 0.590 -> 0.643 of 8 TB/s
    // (2 rounds, same box): the data / delta lines two waves share meet in one L2
    const int64_t t0 = (xcd_block() * NW + wid) * R;  // first row of the wave
    float cand_v = 0.f;
    uint64_t cand_p = kNoPos;
    bool cand_ok = false;
    // every wave reaches the block barrier before the write-back (a wave past the last
    // row, or behind a predecessor that needs the host first, does no work)
    const bool live = t0 < rows && !(bt.prev && ctrl_abnormal(bt.prev));
    int32_t* const ls = s_slot[wid];
    bool all_id = false;
    // record of push b for the row of this lane's vector j
    auto rec_of = [&](int rl, int b) -> int32_t { return all_id ? (int32_t)(t0 + rl) : ls[rl * kMaxW + b]; };
    int rc[JMAX];  // (row << 16 | vector within the row)
    uint32_t on = 0, tch = 0;
    float acc[JMAX][VEC], dl[JMAX][VEC], lg[JMAX][VEC], rv[JMAX][VEC];
    int rb[JMAX][VEC];  // chunk push index of the element's last strict rise (-1: none)
    if (live) do {
        const int NV = cols / VEC;
        const int nrow = (int)(rows - t0 < (int64_t)R ? rows - t0 : (int64_t)R);
        const int ss = slot_stride(nb);
        // identity pushes checked record by record before the launch (Batch::ident_ok)
        const uint64_t ident = bt.ident_ok ? ctrl->ident : 0ull;
        const uint64_t nbm = nb >= 64 ? ~0ull : (1ull << nb) - 1ull;
        // Every push identity (the 4a leg's ascending full-range pushes): the key index
        // ran for none of them, so no row is flagged and record r holds row r. No slot
        // rows, no flag reads: the data, delta and record loads issue at once instead
        // of behind two dependent DRAM round trips.
        all_id = (ident & nbm) == nbm;  // wave-uniform
        uint32_t flg = 0;                          // bit rl: row t0 + rl is flagged (the host replays it)
        if (!all_id) {
            // the rows' flags, one load per row, and the wave's slot rows into LDS,
            // handed back clean (-1) for the next batch; flagged rows stay -1 there
            if (rowflag) flg = (uint32_t)__ballot(lane < nrow && rowflag[t0 + lane] != 0u);
            for (int e = lane; e < nrow * nb; e += 64) {
                const int rl = e / nb, b = e - rl * nb;
                const int64_t r = t0 + rl;
                int32_t v = -1;
                if (!((flg >> rl) & 1u)) {
                    if ((ident >> b) & 1ull) {
                        v = r < bt.nrec[b] ? (int32_t)r : -1;  // record = row; the index skipped it
                    } else {
                        v = slot[r * ss + b];
                        if (v >= 0) slot[r * ss + b] = -1;
                    }
                }
                ls[rl * kMaxW + b] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const int nvec = nrow * NV;
#pragma unroll
        for (int j = 0; j < JMAX; ++j) {
            const int v = j * 64 + lane;
            const int rlj = v < nvec ? v / NV : 0;
            const int cvj = v < nvec ? v - rlj * NV : 0;
            rc[j] = (rlj << 16) | cvj;
            const int64_t ei = (t0 + rlj) * (int64_t)cols + cvj * VEC;
            const bool o = v < nvec && !((flg >> rlj) & 1u);
            on |= (o ? 1u : 0u) << j;
            if (o) {
                unpack<float>(ldg16_nt((const uint8_t*)(shard + ei)), acc[j]);
                unpack<float>(ldg16_nt((const uint8_t*)(ada.delta + ei)), dl[j]);
            } else {
#pragma unroll
                for (int e = 0; e < VEC; ++e) acc[j][e] = dl[j][e] = 0.f;
            }
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                lg[j][e] = 0.f;
                rv[j][e] = 0.f;
                rb[j][e] = -1;
            }
        }
        // one contribution u of push b to element (j, e): k_reduce's apply()
        auto upd = [&](int j, int e, float u, int b) {
            acc[j][e] = __fadd_rn(acc[j][e], u);
            const float nd = __fadd_rn(dl[j][e], __fmul_rn(u, u));
            if (nd > dl[j][e]) { rv[j][e] = nd; rb[j][e] = b; }
            if (nd > 1.0f) lg[j][e] = nd;
            dl[j][e] = nd;
        };
        uint64_t cut = ctrl->cutoff;
        if (tail_cut < cut) cut = tail_cut;
        if (cut != kNoPos) {
            // error batch: element by element, pushes in order, up to the cutoff byte
            const int cut_b = (int)(cut >> 40);
            const uint64_t cut_off = cut & kOffMask;
            // j and e unrolled: the per-element state stays in registers (a runtime
            // index would move the arrays to scratch for the whole kernel)
#pragma unroll
            for (int j = 0; j < JMAX; ++j) {
                if (!(on >> j & 1u)) continue;
                for (int b = 0; b < nb; ++b) {
                    const int gb = bt.bidx[b];
                    if (gb > cut_b) break;
                    const int32_t rr = rec_of(rc[j] >> 16, b);
                    if (rr < 0) continue;
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        const uint64_t off = (uint64_t)((int64_t)rr * stride + K +
                                                        (int64_t)((rc[j] & 0xFFFF) * VEC + e) * 4);
                        if (!(gb == cut_b && off >= cut_off)) {
                            tch |= 1u << j;
                            upd(j, e, Elem<float>::load(bt.base[b] + off), b);
                        }
                    }
                }
            }
        } else {
            // PB pushes per round: all their loads in flight, then applied push by push
#pragma unroll 1
            for (int b0 = 0; b0 < nb; b0 += PB) {
                int32_t rr[PB][JMAX];
                u32x4 raw[PB][JMAX];
#pragma unroll
                for (int q = 0; q < PB; ++q) {
                    const int b = b0 + q < nb ? b0 + q : nb - 1;
                    const uint8_t* const bp = bt.base[b];
#pragma unroll
                    for (int j = 0; j < JMAX; ++j) {
                        rr[q][j] = (b0 + q < nb && (on >> j & 1u)) ? rec_of(rc[j] >> 16, b) : -1;
                        const uint8_t* src =
                            bp + (int64_t)(rr[q][j] >= 0 ? rr[q][j] : 0) * stride + K + (int64_t)(rc[j] & 0xFFFF) * 16;
                        raw[q][j] = rr[q][j] >= 0 ? ldg16_nt(src) : u32x4{0u, 0u, 0u, 0u};
                    }
                }
#pragma unroll
                for (int q = 0; q < PB; ++q)
#pragma unroll
                    for (int j = 0; j < JMAX; ++j) {
                        if (rr[q][j] < 0) continue;
                        tch |= 1u << j;
                        float u[VEC];
                        unpack<float>(raw[q][j], u);
#pragma unroll
                        for (int e = 0; e < VEC; ++e) upd(j, e, u[e], b0 + q);
                    }
            }
        }
    } while (0);
    if (live) {
        // write-back of the touched vectors: data, delta, alpha where the last delta
        // a push left above 1 sets it (FloatMatrixStoreAdaGrad.java:268-272), and
        // this lane's maxDelta candidate
#pragma unroll
        for (int j = 0; j < JMAX; ++j) {
            if (!(tch >> j & 1u)) continue;
            const int rl = rc[j] >> 16, cv = rc[j] & 0xFFFF;
            const int64_t ei = (t0 + rl) * (int64_t)cols + cv * VEC;
            stg16_nt(shard + ei, pack<float>(acc[j]));
            stg16_nt(ada.delta + ei, pack<float>(dl[j]));
            float na[VEC];
            bool all_a = true;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                na[e] = 0.f;
                if (lg[j][e] > 1.0f) {
                    na[e] = (float)((double)ada.initial_alpha / ((double)ada.factor * sqrt((double)lg[j][e])));
                    if (na[e] < ada.min_alpha) na[e] = ada.min_alpha;
                } else {
                    all_a = false;
                }
            }
            if (all_a) stg16_nt(ada.alpha + ei, pack<float>(na));
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                if (!all_a && lg[j][e] > 1.0f) ada.alpha[ei + e] = na[e];
                if (rb[j][e] >= 0) {
                    const int b = rb[j][e];
                    const int32_t rr = rec_of(rl, b);
                    const uint64_t p = pos_of((uint64_t)bt.bidx[b],
                                              (uint64_t)((int64_t)rr * stride + K + (int64_t)(cv * VEC + e) * 4));
                    if (!cand_ok || rv[j][e] > cand_v || (rv[j][e] == cand_v && p < cand_p)) {
                        cand_ok = true;
                        cand_v = rv[j][e];
                        cand_p = p;
                    }
                }
            }
        }
    }
    cand_block_best<NW>(cand_ok, cand_v, cand_p);
    if (threadIdx.x == 0) {
        DeltaCand c;
        c.value = cand_v;
        c.valid = cand_ok;
        c.pos = cand_p;
        ada.cand[blockIdx.x] = c;
    }
}


// Occupancy cap: dynamic LDS (unused by the kernels) so that at most `bpc`
// 256-thread blocks fit on a CU (160 KiB of LDS per CU). 0 = no cap.
constexpr unsigned kLdsPerCU = 160 * 1024;
inline unsigned lds_for_blocks_per_cu(int bpc) { return bpc > 0 ? kLdsPerCU / (unsigned)(bpc + 1) + 256u : 0u; }

template <typename T, int MODE, int G = 8, bool NT = false, int WPB = 4, int SNT = 0, int CPW = 1, int RPW = 1,
          bool FULL = false>
static hipError_t launch_reduce_t(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                                  int64_t stride, int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                                  uint64_t tail_cut,
                                  const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out, LaunchEv ev = {},
                                  RowMap rm = {}, int bpc = 0) {
    constexpr int VEC = Elem<T>::VEC;
    const int32_t nchunks = (cols + 64 * VEC - 1) / (64 * VEC);
    const int32_t ngroups = (nchunks + CPW - 1) / CPW;
    const int64_t ntask = (rows + RPW - 1) / RPW * ngroups;
    const int64_t nblocks = (ntask + WPB - 1) / WPB;
    if (nblocks_out) *nblocks_out = nblocks;
    if (nblocks <= 0) return hipSuccess;
    // blocks per CU: the shape's cap (unused dynamic LDS), 0 = none
    const unsigned occ_lds = lds_for_blocks_per_cu(bpc);
    if constexpr (RPW > 1) {
        static_assert(MODE != kAdaGrad && MODE != kRollbackI32, "k_reduce_rows shapes");
        static const std::string kn =
            kname("k_reduce_rows", type_name<T>(), MODE, CPW, RPW, NT, FULL, G == 3 ? 3 : 1, WPB, SNT);
        g_kernel_name = kn.c_str();
        if (ev.start || ev.stop)
            hipExtLaunchKernelGGL((k_reduce_rows<T, MODE, CPW, RPW, NT, FULL, G == 3 ? 3 : 1, WPB, SNT>), dim3((unsigned)nblocks),
                                  dim3(64 * WPB), occ_lds, st, ev.start, ev.stop, 0, (T*)shard, rows, cols, ngroups, bt, nb, stride,
                                  K, const_cast<int32_t*>(slot), rowflag, ctrl, tail_cut, rm);
        else
            hipLaunchKernelGGL((k_reduce_rows<T, MODE, CPW, RPW, NT, FULL, G == 3 ? 3 : 1, WPB, SNT>), dim3((unsigned)nblocks),
                               dim3(64 * WPB), occ_lds, st, (T*)shard, rows, cols, ngroups, bt, nb, stride, K, const_cast<int32_t*>(slot), rowflag,
                               ctrl, tail_cut, rm);
    } else {
        static const std::string kn = kname("k_reduce", type_name<T>(), MODE, G, NT, WPB, SNT != 0, CPW);
        g_kernel_name = kn.c_str();
        if (ev.start || ev.stop)
            hipExtLaunchKernelGGL((k_reduce<T, MODE, G, NT, WPB, SNT, CPW>), dim3((unsigned)nblocks), dim3(64 * WPB),
                                  occ_lds, st, ev.start, ev.stop, 0, (T*)shard, rows, cols, ngroups, bt, nb, stride,
                                  K, slot, rowflag, ctrl, tail_cut, ada, rm);
        else
            hipLaunchKernelGGL((k_reduce<T, MODE, G, NT, WPB, SNT, CPW>), dim3((unsigned)nblocks), dim3(64 * WPB),
                               occ_lds, st, (T*)shard, rows, cols, ngroups, bt, nb, stride, K, slot, rowflag, ctrl,
                               tail_cut, ada, rm);
    }
    return hipGetLastError();
}

// Shape rule (measured, scripts/ubench_reduce.hip, scripts/exp_variants.py): a
// wave owns RPW neighbouring rows and walks up to CPW = 4 neighbouring 1-KiB
// chunks of each, RPW x CPW 16-B nt loads of one push in flight. Whole 4-KiB
// rows: RPW = 2 with the CU capped at 2 blocks (8 waves, 64 KiB of loads in
// flight); other widths RPW = 4 at their register-limited occupancy. AdaGrad and
// the int32 rollback keep one row and one chunk per wave (k_reduce: their
// per-element state triples the registers).
template <typename T, int MODE>
static hipError_t launch_auto(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride, int K,
                              const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl, uint64_t tail_cut,
                              const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out, LaunchEv ev, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    const int32_t nchunks = (cols + 64 * VEC - 1) / (64 * VEC);
#define DML_L(G, CPW, RPW) launch_reduce_t<T, MODE, G, true, 4, false, CPW, RPW>(shard, rows, cols, bt, nb, stride, K, \
                                                     slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev, rm)
// whole-chunk rows store write-through (SNT 2, stg16_wt): no dirty L2 lines for the
// kernel-end writeback, so the next reduce on the stream starts sooner (config 2:
// 0.3455 -> 0.3365 ms/step with sampled timing, same box)
#define DML_LF(G, CPW, RPW, BPC) launch_reduce_t<T, MODE, G, true, 4, 2, CPW, RPW, true>(shard, rows, cols, bt, nb, \
                                                     stride, K, slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev, rm, BPC)
    if constexpr (MODE == kAdaGrad) {
        // G8 with nt shard / delta / alpha traffic (measured best: G4 +10 %, G16 +35 %,
        // 8-wave blocks +15 %, cached stores slower). The candidate buffer
        // holds one entry per 4-wave block.
        return launch_reduce_t<T, MODE, 8, true, 4, true, 1, 1>(shard, rows, cols, bt, nb, stride, K, slot, rowflag,
                                                                ctrl, tail_cut, ada, st, nblocks_out, ev, rm);
    } else if constexpr (MODE == kRollbackI32) {
        return DML_L(8, 1, 1);
    } else {
        if (cols < VEC) return DML_L(16, 1, 1);  // narrower than one vector: k_reduce's generic path
        // whole 4-KiB rows: four rows per wave and at most 8 waves per CU (128 KiB of
        // loads in flight per CU): config 2 355.7-358.3 us against 362.6-367.7 us for
        // two rows at 8 waves, 381 us for four rows uncapped or at 12 waves, 367 us at
        // 6 waves; 1-wave blocks at 8 per CU equal
        if (cols % (64 * VEC * 4) == 0) return DML_LF(1, 4, 4, 2);
        // Other widths: pair-packed load groups (DEPTH 3) over 4 rows per wave.
        // Non-temporal shard stores (the rows are written once per batch): config 5
        // 460 -> 433 us; config 2's FULL shape measured no gain from them (it stores
        // write-through, DML_LF above).
#define DML_LN(G, CPW, RPW) launch_reduce_t<T, MODE, G, true, 4, 1, CPW, RPW>(shard, rows, cols, bt, nb, stride, K, \
                                                     slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev, rm)
#define DML_LFN(G, CPW, RPW) launch_reduce_t<T, MODE, G, true, 4, 1, CPW, RPW, true>(shard, rows, cols, bt, nb, \
                                                     stride, K, slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev, rm, 0)
        if (MODE != kPreReduce) {
            // Rows of >= 4 chunks that do not fill them (config 5's 4000-B int32 rows in
            // 4004-B records): cached record loads (the line two neighbouring records
            // share is fetched once) and 2-wave blocks (a finished block frees its slot
            // sooner): config 5 428 -> 400 us, 0.565 -> 0.604 of peak, measured against
            // nt loads, 1/4/8-wave blocks, CPW 1/2, RPW 2, cached stores.
            if (nchunks >= 4)
                return launch_reduce_t<T, MODE, 3, false, kC5Wpb, 1, 4, kC5Rpw>(shard, rows, cols, bt, nb, stride, K,
                                                                               slot, rowflag, ctrl, tail_cut, ada, st,
                                                                               nblocks_out, ev, rm);
            if (cols % (64 * VEC * 2) == 0) return DML_LFN(1, 2, 4);
            if (nchunks >= 2) return DML_LN(3, 2, 4);
            if (cols % (64 * VEC) == 0) return DML_LFN(1, 1, 4);
            return DML_LN(3, 1, 4);
        }
#undef DML_LN
#undef DML_LFN
        if (nchunks >= 4) return DML_L(3, 4, 4);
        if (cols % (64 * VEC * 2) == 0) return DML_LF(1, 2, 4, 0);
        if (nchunks >= 2) return DML_L(3, 2, 4);
        if (cols % (64 * VEC) == 0) return DML_LF(1, 1, 4, 0);
        return DML_L(3, 1, 4);
    }
#undef DML_L
#undef DML_LF
}

// k_reduce_flat launch (narrow dense rows, see the kernel): R rows per wave.
template <typename T, int MODE, int JMAX, int PB>
static hipError_t launch_flat_t(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride,
                                int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl, uint64_t tail_cut,
                                hipStream_t st, int64_t* nblocks_out, LaunchEv ev, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC;
    const int NV = cols / VEC;
    const int R = std::max(1, std::min(16, JMAX * 64 / NV));
    const int64_t nblocks = ((rows + R - 1) / R + 3) / 4;
    if (nblocks_out) *nblocks_out = nblocks;
    if (nblocks <= 0) return hipSuccess;
    static const std::string kn = kname("k_reduce_flat", type_name<T>(), MODE, JMAX, PB);
    g_kernel_name = kn.c_str();
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL((k_reduce_flat<T, MODE, JMAX, PB>), dim3((unsigned)nblocks), dim3(256), 0, st, ev.start,
                              ev.stop, 0, (T*)shard, rows, cols, R, bt, nb, stride, K, const_cast<int32_t*>(slot),
                              rowflag, ctrl, tail_cut, rm);
    else
        hipLaunchKernelGGL((k_reduce_flat<T, MODE, JMAX, PB>), dim3((unsigned)nblocks), dim3(256), 0, st, (T*)shard,
                           rows, cols, R, bt, nb, stride, K, const_cast<int32_t*>(slot), rowflag, ctrl, tail_cut, rm);
    return hipGetLastError();
}

// One push per round: JMAX 8 (R = 10 rows at 200 columns) measured within 2 % of
// 4 x 1, 4 x 2, 8 x 2 and 4 x 4 (config 4, ascending and permuted), and of
// occupancy caps at 1-3 blocks per CU (all slower); nt record loads 2-3 % faster
// than cached ones; JMAX 12 (below) beat 8 on permuted pushes.
template <typename T, int MODE>
static hipError_t launch_flat(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride, int K,
                              const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl, uint64_t tail_cut,
                              hipStream_t st, int64_t* nblocks_out, LaunchEv ev, RowMap rm) {
    // JMAX 12: config 4's 800-B rows as 15 rows per wave (750 of 768 vector slots);
    // permuted pushes 4 775-4 801 -> 4 905-4 925 GiB/s against JMAX 8 (10 rows),
    // ascending equal, JMAX 16 in between (same box, 2 rounds)
    return launch_flat_t<T, MODE, 12, 1>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut, st,
                                         nblocks_out, ev, rm);
}

// k_flat_ident launch: the all-identity chunks of the flat shape (the host checked
// the index's Ctrl). J = 8 vectors per lane (10 rows of 200 fp32 per wave), three
// pushes in flight, 8-wave blocks (one per CU at 2 waves per SIMD): the best of the
// shapes scripts/ubench_flat.hip measured (config 4: 0.768 of 8 TB/s against 0.727
// for k_reduce_flat's loop on one box).
constexpr int kFlatIdentJ = 8;  // 16-B vectors per lane

int flat_ident_rows_per_wave(int vtype, int32_t cols) {
    const int NV = cols / (vtype == kF64 ? 2 : 4);
    return std::max(1, std::min(16, kFlatIdentJ * 64 / std::max(NV, 1)));
}

template <typename T, int MODE>
static hipError_t launch_flat_ident_t(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                                      int64_t stride, int K, Ctrl* ctrl, hipStream_t st, int64_t* nblocks_out,
                                      LaunchEv ev, RowMap rm) {
    constexpr int VEC = Elem<T>::VEC, J = kFlatIdentJ, D = 3, NW = kFlatIdentWaves;  // D: pushes in flight
    const int NV = cols / VEC;
    const int R = std::max(1, std::min(16, J * 64 / NV));
    const int64_t nblocks = ((rows + R - 1) / R + NW - 1) / NW;
    if (nblocks_out) *nblocks_out = nblocks;
    if (nblocks <= 0) return hipSuccess;
    static const std::string kn = kname("k_flat_ident", type_name<T>(), MODE, J, D, NW);
    g_kernel_name = kn.c_str();
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL((k_flat_ident<T, MODE, J, D, NW>), dim3((unsigned)nblocks), dim3(NW * 64), 0, st,
                              ev.start, ev.stop, 0, (T*)shard, rows, cols, R, bt, nb, stride, K, ctrl, rm);
    else
        hipLaunchKernelGGL((k_flat_ident<T, MODE, J, D, NW>), dim3((unsigned)nblocks), dim3(NW * 64), 0, st,
                           (T*)shard, rows, cols, R, bt, nb, stride, K, ctrl, rm);
    return hipGetLastError();
}

hipError_t launch_flat_ident(int vtype, int mode, void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                             int64_t stride, int K, Ctrl* ctrl, hipStream_t st, int64_t* nblocks_out, LaunchEv ev,
                             RowMap rm) {
#define DML_FI(T, M) launch_flat_ident_t<T, M>(shard, rows, cols, bt, nb, stride, K, ctrl, st, nblocks_out, ev, rm)
    if (vtype == kF32) return mode == kAdd ? DML_FI(float, kAdd) : DML_FI(float, kPreReduce);
    if (vtype == kI32) return mode == kAdd ? DML_FI(int32_t, kAdd) : DML_FI(int32_t, kPreReduce);
    if (vtype == kF64) return mode == kAdd ? DML_FI(double, kAdd) : DML_FI(double, kPreReduce);
#undef DML_FI
    return hipErrorInvalidValue;
}

// The flat narrow-row kernels apply to plain sums (and AdaGrad chunks of at most 4
// pushes) of rows narrower than 4 KiB (whole vectors) when every push of the chunk
// lists at least half the rows (dense pushes; sparse ones keep the pair-packed
// k_reduce_rows / k_reduce).
bool use_flat(int vtype, int mode, int32_t cols, const Batch& bt, int nb, int64_t rows) {
    if (mode != kAdd && mode != kPreReduce && !(mode == kAdaGrad && vtype == kF32 && nb <= 4)) return false;
    const int VEC = vtype == kF64 ? 2 : 4;
    const int elem = vtype == kF64 ? 8 : 4;
    if (cols % VEC || (int64_t)cols * elem >= 4096 || nb <= 0) return false;
    for (int b = 0; b < nb; ++b)
        if (2 * bt.nrec[b] < rows) return false;
    return true;
}

bool flat_ident_ok(const Ctrl& h, const Batch& bt, int nb, int64_t need, uint64_t tail_cut) {
    if (nb <= 0 || tail_cut != kNoPos || h.cutoff != kNoPos || h.no_dup == 0u) return false;
    for (int b = 0; b < nb; ++b)
        if (!ctrl_identity(&h, h.ident, b) || bt.nrec[b] < need) return false;
    return true;
}

// Identity speculation pays where the double-buffered reduce streams as fast as
// the in-place one (measured), and is only offered to the kernels
// whose loops verify a slot-keeping chunk completely (every live row of every
// push has a record, every record's key is checked): whole 4-KiB rows
// (k_reduce_rows FULL, the DEPTH-1 loop) and the flat kernel's rows under 4 KiB.
// Rows of >= 4 KiB that are not whole 4-KiB multiples run the pair-packed DEPTH-3
// loop, which checks identity records only: no speculation there.
bool spec_shape(int vtype, int32_t cols) {
    const int VEC = vtype == kF64 ? 2 : 4;
    const int64_t bytes = (int64_t)cols * (vtype == kF64 ? 8 : 4);
    return bytes % 4096 == 0 || (cols % VEC == 0 && bytes < 4096);
}

// k_ada_flat launch: R rows per wave (R = 5 at 200 columns), NW waves per block.
template <int JMAX, int PB, int NW>
static hipError_t launch_ada_flat_t(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride,
                                    int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                                    uint64_t tail_cut, const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out,
                                    LaunchEv ev) {
    const int NV = cols / 4;
    const int R = std::max(1, std::min(16, JMAX * 64 / NV));
    const int64_t nblocks = ((rows + R - 1) / R + NW - 1) / NW;
    if (nblocks_out) *nblocks_out = nblocks;
    if (nblocks <= 0) return hipSuccess;
    static const std::string kn = kname("k_ada_flat", JMAX, PB, NW);
    g_kernel_name = kn.c_str();
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL((k_ada_flat<JMAX, PB, NW>), dim3((unsigned)nblocks), dim3(NW * 64), 0, st, ev.start,
                              ev.stop, 0, (float*)shard, rows, cols, R, bt, nb, stride, K, const_cast<int32_t*>(slot),
                              rowflag, ctrl, tail_cut, ada);
    else
        hipLaunchKernelGGL((k_ada_flat<JMAX, PB, NW>), dim3((unsigned)nblocks), dim3(NW * 64), 0, st, (float*)shard,
                           rows, cols, R, bt, nb, stride, K, const_cast<int32_t*>(slot), rowflag, ctrl, tail_cut, ada);
    return hipGetLastError();
}

// k_ada_ident: k_ada_flat for the AdaGrad chunks the host has seen to be all identity
// after the index (every push full-range with record r = row r, checked record by
// record before the launch; no cutoff, no repeated row: config 4's AdaGrad steady
// state), at most 4 pushes, laid out as the plain data / delta stream: a thread owns U
// 16-B vectors of the shard, 256 apart inside its block's 256·U-vector tile (each
// wave's stores are whole 1 KiB runs), wherever rows begin; a vector's record offset
// (row = e / cols) is computed per vector. Every load (data, delta, NB pushes) is in
// flight before the first add. The same per-element arithmetic, order, alpha and
// maxDelta candidates as k_ada_flat (bit for bit; the candidate is reduced per block,
// max value then lowest position). One vector per thread (U = 1, 54-60 VGPRs, full
// occupancy) ran 8.58-8.61 ms on the config-4 AdaGrad leg against 9.30-9.33 ms for the
// previous row-per-wave shape (8 vectors per lane, 10 rows per wave, 2-wave blocks, 170
// VGPRs) and 8.41-8.95 ms for 2 or 4 vectors, alternating builds on one box
// (profiles/r06_ab_ada_vec.txt): 0.96 of the plain stream of the same bytes.
constexpr int kAdaIdentU = 1;  // 16-B vectors per thread

template <int U, int NB>
__global__ __launch_bounds__(256) void k_ada_ident(float* __restrict__ shard, int64_t nvec, int32_t cols,
                                                   const Batch bt, int64_t stride, int K, AdaArgs ada) {
    constexpr int VEC = 4;
    const int64_t v0 = xcd_block() * (256 * U) + threadIdx.x;
    float cand_v = 0.f;
    uint64_t cand_p = kNoPos;
    int cand_key = 0;
    bool cand_ok = false;
    int64_t roff[U];
    bool on[U];
    float acc[U][VEC], dl[U][VEC], lg[U][VEC], rv[U][VEC];
    int rb[U][VEC];  // push of the element's last strict rise (-1: none)
    u32x4 raw[NB][U];
    // the loads do not wait for the predecessor check (reads only; behind an abnormal
    // predecessor nothing below is stored): a short block's data is in flight from its
    // first instructions
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = v0 + u * 256, e = v * VEC;
        on[u] = v < nvec;
        roff[u] = (e / cols) * stride + K + (e % cols) * 4;
        const u32x4 z{0u, 0u, 0u, 0u};
        unpack<float>(on[u] ? ldg16_nt((const uint8_t*)shard + v * 16) : z, acc[u]);
        unpack<float>(on[u] ? ldg16_nt((const uint8_t*)ada.delta + v * 16) : z, dl[u]);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) raw[b][u] = on[u] ? ldg16_nt(bt.base[b] + roff[u]) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            lg[u][e] = 0.f;
            rv[u][e] = 0.f;
            rb[u][e] = -1;
        }
    // k_ada_flat's upd(), pushes in order
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float g[VEC];
            unpack<float>(raw[b][u], g);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                acc[u][e] = __fadd_rn(acc[u][e], g[e]);
                const float nd = __fadd_rn(dl[u][e], __fmul_rn(g[e], g[e]));
                if (nd > dl[u][e]) { rv[u][e] = nd; rb[u][e] = b; }
                if (nd > 1.0f) lg[u][e] = nd;
                dl[u][e] = nd;
            }
        }
    const uint64_t bi0 = (uint64_t)bt.bidx[0], bi1 = NB > 1 ? (uint64_t)bt.bidx[NB > 1 ? 1 : 0] : 0,
                   bi2 = NB > 2 ? (uint64_t)bt.bidx[NB > 2 ? 2 : 0] : 0, bi3 = NB > 3 ? (uint64_t)bt.bidx[NB > 3 ? 3 : 0] : 0;
    const bool live = !(bt.prev && ctrl_abnormal(bt.prev));  // predecessor needs the host first
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!live || !on[u]) continue;
        const int64_t v = v0 + u * 256;
        stg16_nt((uint8_t*)shard + v * 16, pack<float>(acc[u]));
        stg16_nt((uint8_t*)ada.delta + v * 16, pack<float>(dl[u]));
        // alpha where the last delta a push left above 1 sets it (FloatMatrixStoreAdaGrad.java:268-272)
        float na[VEC];
        bool all_a = true, any_a = false;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            na[e] = 0.f;
            if (lg[u][e] > 1.0f) {
                na[e] = (float)((double)ada.initial_alpha / ((double)ada.factor * sqrt((double)lg[u][e])));
                if (na[e] < ada.min_alpha) na[e] = ada.min_alpha;
                any_a = true;
            } else {
                all_a = false;
            }
        }
        if (all_a) {
            stg16_nt((uint8_t*)ada.alpha + v * 16, pack<float>(na));
        } else if (any_a) {
#pragma unroll
            for (int e = 0; e < VEC; ++e)
                if (lg[u][e] > 1.0f) ada.alpha[v * VEC + e] = na[e];
        }
        // the thread's candidate in (push, vector, element) order, which is position
        // order (the pushes' columns ascend, offsets grow with u and e): the position
        // itself is formed once, for the winner
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            if (rb[u][e] < 0) continue;
            const int key = (rb[u][e] << 16) | (u << 2) | e;
            if (!cand_ok || rv[u][e] > cand_v || (rv[u][e] == cand_v && key < cand_key)) {
                cand_ok = true;
                cand_v = rv[u][e];
                cand_key = key;
            }
        }
    }
    if (cand_ok) {
        const int g = cand_key >> 16, u = (cand_key >> 2) & 0x3FFF, e = cand_key & 3;
        const uint64_t gb = g == 0 ? bi0 : g == 1 ? bi1 : g == 2 ? bi2 : bi3;  // (a select chain)
        int64_t ro = roff[0];
#pragma unroll
        for (int k = 1; k < U; ++k) ro = u == k ? roff[k] : ro;
        cand_p = pos_of(gb, (uint64_t)(ro + e * 4));
    }
    cand_block_best<4>(cand_ok, cand_v, cand_p);
    if (threadIdx.x == 0) {
        DeltaCand c;
        c.value = cand_v;
        c.valid = cand_ok;
        c.pos = cand_p;
        ada.cand[blockIdx.x] = c;
    }
}

template <int U, int NB>
static hipError_t launch_ada_ident_t(void* shard, int64_t nvec, int32_t cols, int64_t nblocks, const Batch& bt,
                                     int64_t stride, int K, const AdaArgs& ada, hipStream_t st, LaunchEv ev) {
    static const std::string kn = kname("k_ada_ident", U, NB);
    g_kernel_name = kn.c_str();
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL((k_ada_ident<U, NB>), dim3((unsigned)nblocks), dim3(256), 0, st, ev.start, ev.stop, 0,
                              (float*)shard, nvec, cols, bt, stride, K, ada);
    else
        hipLaunchKernelGGL((k_ada_ident<U, NB>), dim3((unsigned)nblocks), dim3(256), 0, st, (float*)shard, nvec, cols,
                           bt, stride, K, ada);
    return hipGetLastError();
}

// One maxDelta candidate per block: *ncand_out = the blocks launched (<= reduce_blocks(),
// the candidate buffer's size).
hipError_t launch_ada_ident(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride, int K,
                            const AdaArgs& ada, hipStream_t st, int64_t* ncand_out, LaunchEv ev) {
    if (nb <= 0 || nb > 4 || cols % 4 || (int64_t)cols * 4 >= 4096) return hipErrorInvalidValue;
    constexpr int U = kAdaIdentU;
    const int64_t nvec = rows * cols / 4, nblocks = (nvec + 256 * U - 1) / (256 * U);
    if (ncand_out) *ncand_out = nblocks;
    if (nblocks <= 0) return hipSuccess;
    switch (nb) {
        case 1: return launch_ada_ident_t<U, 1>(shard, nvec, cols, nblocks, bt, stride, K, ada, st, ev);
        case 2: return launch_ada_ident_t<U, 2>(shard, nvec, cols, nblocks, bt, stride, K, ada, st, ev);
        case 3: return launch_ada_ident_t<U, 3>(shard, nvec, cols, nblocks, bt, stride, K, ada, st, ev);
        default: return launch_ada_ident_t<U, 4>(shard, nvec, cols, nblocks, bt, stride, K, ada, st, ev);
    }
}

// JMAX 4 vectors per lane (R = 5 rows at 200 columns), two pushes per round: for
// chunks of at most 4 pushes (the exact exchange path's slices at low W) 17.3 ms
// per 10 M-row config-4 AdaGrad apply of 2 pushes against 19.1 ms for k_reduce;
// with 8 pushes k_reduce (8 pushes in flight per wave) stays ahead (2.6 vs 2.95 ms).
static hipError_t launch_ada_flat(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride,
                                  int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl, uint64_t tail_cut,
                                  const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out, LaunchEv ev) {
    return launch_ada_flat_t<4, 2, kAdaFlatWaves>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut,
                                                  ada, st, nblocks_out, ev);
}

bool reduce_clears_slots(int vtype, int mode, int32_t cols) {
    if (mode == kAdaGrad) return vtype == kF32 && cols <= 64 * 4;  // k_reduce, one chunk group per row
    if (mode != kAdd && mode != kPreReduce && mode != kAddCheckI32) return false;
    const int VEC = vtype == kF64 ? 2 : 4;
    if (cols < VEC) return false;  // k_reduce's generic path
    // k_reduce_rows clears only when one wave owns a row's every chunk (launch_auto's
    // CPW: 4 for whole 4-KiB multiples and for >= 4 chunks, else 2 or 1); the flat
    // kernel always does, but is chosen per chunk, so it is not counted on here
    const int64_t nchunks = (cols + 64 * VEC - 1) / (64 * VEC);
    const int64_t cpw = (nchunks >= 4 || cols % (64 * VEC * 4) == 0) ? 4 : nchunks >= 2 ? 2 : 1;
    return nchunks <= cpw;
}

int64_t reduce_blocks(int vtype, int64_t rows, int32_t cols) {
    // The most maxDelta candidates one AdaGrad apply writes (the candidate buffer's size):
    // k_reduce runs one row and one chunk per wave, 4 waves per block, one candidate per
    // block; k_ada_flat fewer; k_ada_ident one per block of 256·U vectors.
    const int VEC = vtype == kF64 ? 2 : 4;
    const int64_t nchunks = (cols + 64 * VEC - 1) / (64 * VEC);
    int64_t n = (rows * nchunks + 3) / 4;
    if (vtype == kF32 && cols >= 4 && cols % 4 == 0 && (int64_t)cols * 4 < 4096)
        n = std::max(n, (rows * cols / 4 + 256 * kAdaIdentU - 1) / (256 * kAdaIdentU));
    return n;
}

hipError_t launch_reduce(int vtype, int mode, void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                         int64_t stride, int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                         uint64_t tail_cut, const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out, LaunchEv ev,
                         RowMap rm) {
#define DML_A(T, M) launch_auto<T, M>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev, rm)
#define DML_F(T, M) launch_flat<T, M>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut, st, nblocks_out, ev, rm)
    if (use_flat(vtype, mode, cols, bt, nb, rm.block ? rm.rows_total : rows)) {
        if (mode == kAdaGrad)  // the AdaGrad store runs no row map (exchange path only)
            return rm.block || rm.out ? hipErrorInvalidValue
                                      : launch_ada_flat(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl,
                                                        tail_cut, ada, st, nblocks_out, ev);
        if (vtype == kF32) return mode == kAdd ? DML_F(float, kAdd) : DML_F(float, kPreReduce);
        if (vtype == kI32) return mode == kAdd ? DML_F(int32_t, kAdd) : DML_F(int32_t, kPreReduce);
        if (vtype == kF64) return mode == kAdd ? DML_F(double, kAdd) : DML_F(double, kPreReduce);
    }
#undef DML_F
    if (vtype == kF32) {
        if (mode == kAdd) return DML_A(float, kAdd);
        if (mode == kAdaGrad) return DML_A(float, kAdaGrad);
        if (mode == kPreReduce) return DML_A(float, kPreReduce);
    } else if (vtype == kI32) {
        if (mode == kAdd) return DML_A(int32_t, kAdd);
        if (mode == kAddCheckI32) return DML_A(int32_t, kAddCheckI32);
        if (mode == kPreReduce) return DML_A(int32_t, kPreReduce);
    } else if (vtype == kF64) {
        if (mode == kAdd) return DML_A(double, kAdd);
        if (mode == kPreReduce) return DML_A(double, kPreReduce);
    }
#undef DML_A
    return hipErrorInvalidValue;
}

hipError_t launch_rollback_i32(int32_t* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                               int64_t stride, int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                               uint64_t tail_cut, hipStream_t st) {
    AdaArgs none{};
    return launch_reduce_t<int32_t, kRollbackI32>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl,
                                                  tail_cut, none, st, nullptr);
}

// ---------------------------------------------------------------------------
// maxDelta finalize: reduce the per-block candidates in two launches (kMdParts
// blocks over strided slices -> cand[n .. n + kMdParts), then one block) and
// apply the reference's strict `deltas[i] > maxDelta` update
// (FloatMatrixStoreAdaGrad.java:273-277). One block over 10^5+ candidates was
// bound by a single CU's load rate.
__device__ inline void cand_scan(const DeltaCand* __restrict__ cand, int64_t i, int64_t n, int64_t step, bool& ok,
                                 float& v, uint64_t& p) {
    for (; i < n; i += step) {
        const DeltaCand c = cand[i];
        if (cand_better(c.valid != 0, c.value, c.pos, ok, v, p)) { ok = true; v = c.value; p = c.pos; }
    }
}

__global__ __launch_bounds__(256) void k_maxdelta_part(DeltaCand* __restrict__ cand, int64_t n) {
    bool ok = false;
    float v = 0.f;
    uint64_t p = kNoPos;
    cand_scan(cand, (int64_t)blockIdx.x * 256 + threadIdx.x, n, (int64_t)gridDim.x * 256, ok, v, p);
    cand_block_best<4>(ok, v, p);
    if (threadIdx.x == 0) {
        DeltaCand c;
        c.value = v; c.valid = ok; c.pos = p;
        cand[n + blockIdx.x] = c;
    }
}

__global__ __launch_bounds__(256) void k_maxdelta(const DeltaCand* __restrict__ cand, int64_t n,
                                                  MaxDelta* __restrict__ md, const Batch bt, int nb,
                                                  int64_t stride, int K, int V, int mode,
                                                  const Ctrl* __restrict__ ctrl) {
    bool ok = false;
    float v = 0.f;
    uint64_t p = kNoPos;
    cand_scan(cand, threadIdx.x, n, 256, ok, v, p);
    cand_block_best<4>(ok, v, p);
    if (threadIdx.x != 0) return;
    const DeltaCand pd = md->pend;  // the chunk's candidates so far (main reduce, earlier layers)
    if (cand_better(pd.valid != 0, pd.value, pd.pos, ok, v, p)) { ok = true; v = pd.value; p = pd.pos; }
    const bool defer = mode == kMdDefer || (mode == kMdDeferIfRepeat && ctrl && ctrl->no_dup == 0u);
    if (defer) {
        DeltaCand c;
        c.value = v; c.valid = ok; c.pos = p;
        md->pend = c;
        return;
    }
    md->pend.valid = 0;
    if (ok && v > md->value) {
        const int gb = (int)(p >> 40);
        int b = 0;
        while (b < nb - 1 && bt.bidx[b] != gb) ++b;
        const int64_t off = (int64_t)(p & kOffMask);
        const int64_t r = off / stride;
        md->value = v;
        md->row = (int32_t)ld_key(bt.base[b] + r * stride, K);  // maxDeltaRow = (int)key
        md->col = (int32_t)((off - r * stride - K) / V);
    }
}

hipError_t launch_maxdelta_finalize(DeltaCand* cand, int64_t n, MaxDelta* md, const Batch& bt, int nb,
                                    int64_t stride, int K, int V, hipStream_t st, int mode, const Ctrl* ctrl) {
    if (n > 4 * 256 * kMdParts) {
        hipLaunchKernelGGL(k_maxdelta_part, dim3(kMdParts), dim3(256), 0, st, cand, n);
        hipLaunchKernelGGL(k_maxdelta, dim3(1), dim3(256), 0, st, cand + n, (int64_t)kMdParts, md, bt, nb, stride, K,
                           V, mode, ctrl);
    } else {
        hipLaunchKernelGGL(k_maxdelta, dim3(1), dim3(256), 0, st, cand, n, md, bt, nb, stride, K, V, mode, ctrl);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Array stores (int32): undo after the first negative counter. Records
// [key][value] at stride K+VS; the ordered apply itself is the sorted leaf path
// (dml_sparse.hip).
// Undo (mod 2^32) every int32 array add positioned after the first negative.
__global__ __launch_bounds__(256) void k_array_rollback(int32_t* __restrict__ shard, int64_t rows,
                                                        const uint8_t* __restrict__ base, int64_t nrec, int b_global,
                                                        int64_t stride, int K, int64_t first, Ctrl* __restrict__ ctrl,
                                                        uint64_t tail_cut) {
    const uint64_t neg = ctrl->neg_pos;
    if (neg == kNoPos) return;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    uint64_t cut = ctrl->cutoff;
    if (tail_cut < cut) cut = tail_cut;
    const int64_t off = r * stride;
    if (pos_of((uint64_t)b_global, (uint64_t)off) >= cut) return;
    if (pos_of((uint64_t)b_global, (uint64_t)(off + K)) <= neg) return;
    const int64_t idx = row_index(ld_key(base + off, K), first, rows);
    if (idx < 0) return;
    atomicSub(&shard[idx], (int32_t)ld32(base + off + K));
}

hipError_t launch_array_rollback_i32(int32_t* shard, int64_t rows, const uint8_t* base, int64_t nrec, int b_global,
                                     int64_t stride, int K, int64_t first, Ctrl* ctrl, uint64_t tail_cut,
                                     hipStream_t st) {
    if (nrec <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_array_rollback, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, st, shard, rows, base,
                       nrec, b_global, stride, K, first, ctrl, tail_cut);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_fill(T* __restrict__ p, int64_t n, T v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
static unsigned grid_for(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}
hipError_t launch_fill(int vtype, void* p, int64_t n, double v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (vtype == kF32) hipLaunchKernelGGL(k_fill<float>, dim3(grid_for(n)), dim3(256), 0, st, (float*)p, n, (float)v);
    else if (vtype == kI32) hipLaunchKernelGGL(k_fill<int32_t>, dim3(grid_for(n)), dim3(256), 0, st, (int32_t*)p, n, (int32_t)v);
    else hipLaunchKernelGGL(k_fill<double>, dim3(grid_for(n)), dim3(256), 0, st, (double*)p, n, v);
    return hipGetLastError();
}
hipError_t launch_fill_f32(float* p, int64_t n, float v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill<float>, dim3(grid_for(n)), dim3(256), 0, st, p, n, v);
    return hipGetLastError();
}

// shard += src, element-wise (owner apply after a reduce-scatter).
template <typename T>
__global__ __launch_bounds__(256) void k_apply_dense(T* __restrict__ shard, const T* __restrict__ src, int64_t n) {
    constexpr int VEC = Elem<T>::VEC;
    const int64_t nvec = n / VEC;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
        T a[VEC], b[VEC];
        unpack<T>(((const u32x4*)shard)[i], a);
        unpack<T>(((const u32x4*)src)[i], b);
#pragma unroll
        for (int e = 0; e < VEC; ++e) a[e] = Elem<T>::add(a[e], b[e]);
        ((u32x4*)shard)[i] = pack<T>(a);
    }
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n - nvec * VEC) shard[nvec * VEC + t] = Elem<T>::add(shard[nvec * VEC + t], src[nvec * VEC + t]);
}
// int32 owner apply with IntMatrixStore's negativity check on the final counters
// (IntMatrixStore.java:174-176): the first negative element (row-major) of the
// first failing apply is kept in *neg (sticky: kNoPos until then); once it is
// set, later applies are no-ops (the reference store stops at its exception).
__global__ __launch_bounds__(256) void k_apply_dense_i32chk(int32_t* __restrict__ shard, const int32_t* __restrict__ src,
                                                            int64_t n, unsigned long long* neg) {
    if (__atomic_load_n(neg, __ATOMIC_RELAXED) != kNoPos) return;
    const int64_t nvec = n / 4;
    unsigned long long first = kNoPos;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
        int32_t a[4], b[4];
        unpack<int32_t>(((const u32x4*)shard)[i], a);
        unpack<int32_t>(((const u32x4*)src)[i], b);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            a[e] = Elem<int32_t>::add(a[e], b[e]);
            if (a[e] < 0 && first == kNoPos) first = (unsigned long long)(4 * i + e);
        }
        ((u32x4*)shard)[i] = pack<int32_t>(a);
    }
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n - nvec * 4) {
        const int64_t j = nvec * 4 + t;
        const int32_t v = Elem<int32_t>::add(shard[j], src[j]);
        shard[j] = v;
        if (v < 0 && first == kNoPos) first = (unsigned long long)j;
    }
    if (first != kNoPos) atomicMin(neg, first);
}

// The owner apply runs beside the next call's pre-reduce: a grid
// that fills every free wave slot keeps the pre-reduce's next blocks from being
// placed (its waves need most of a SIMD's VGPRs). kApplyBlocks bounds it to two
// blocks per CU; it still moves a config-2 shard's 192 MB well inside one call.
constexpr unsigned kApplyBlocks = 512;

hipError_t launch_apply_dense_i32chk(int32_t* shard, const int32_t* src, int64_t n, unsigned long long* neg,
                                     hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_dense_i32chk, dim3(kApplyBlocks), dim3(256), 0, st, shard, src, n, neg);
    return hipGetLastError();
}

hipError_t launch_apply_dense(int vtype, void* shard, const void* src, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned g = kApplyBlocks;
    if (vtype == kF32) hipLaunchKernelGGL(k_apply_dense<float>, dim3(g), dim3(256), 0, st, (float*)shard, (const float*)src, n);
    else if (vtype == kI32) hipLaunchKernelGGL(k_apply_dense<int32_t>, dim3(g), dim3(256), 0, st, (int32_t*)shard, (const int32_t*)src, n);
    else hipLaunchKernelGGL(k_apply_dense<double>, dim3(g), dim3(256), 0, st, (double*)shard, (const double*)src, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// handleFetch encode, dense-column layouts (FloatMatrixStore.java:140-153 etc.).
// One thread per (key, column). `value_slot` = bytes per column in the output
// record (4/8; 8 for AdaGrad value+alpha and FloatArrayStore's 8-byte slot).
__device__ inline void st32(uint8_t* p, uint32_t v) { *(uint32_t*)p = v; }

template <typename T>
__global__ void k_fetch(const T* __restrict__ shard, const float* __restrict__ alpha, int32_t cols,
                        const int64_t* __restrict__ keys, int64_t key_lo, int64_t n, int64_t first,
                        uint8_t* __restrict__ out, int64_t rec, int K, int value_slot) {
    const int64_t total = n * (int64_t)cols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = t / cols;
        const int32_t c = (int32_t)(t - j * cols);
        const int64_t key = keys ? keys[j] : key_lo + j;
        const int64_t idx = key - first;
        uint8_t* o = out + j * rec;
        if (c == 0) {
            st32(o, (uint32_t)key);
            if (K == 8) st32(o + 4, (uint32_t)((uint64_t)key >> 32));
        }
        uint8_t* v = o + K + (int64_t)c * value_slot;
        const T x = shard[idx * cols + c];
        if constexpr (sizeof(T) == 4) {
            st32(v, __builtin_bit_cast(uint32_t, x));
        } else {
            const uint64_t u = __builtin_bit_cast(uint64_t, x);
            st32(v, (uint32_t)u); st32(v + 4, (uint32_t)(u >> 32));
        }
        if (alpha) st32(v + 4, __float_as_uint(alpha[idx * cols + c]));
        else if (sizeof(T) == 4 && value_slot == 8) st32(v + 4, 0u);  // FloatArrayStore's zero pad
    }
}
hipError_t launch_fetch(int vtype, const void* shard, const float* alpha, int32_t cols, const int64_t* keys,
                        int64_t key_lo, int64_t n, int64_t first, uint8_t* out, int64_t rec, int K, int value_slot,
                        hipStream_t st) {
    const int64_t total = n * (int64_t)cols;
    if (total <= 0) return hipSuccess;
    const dim3 g(grid_for(total));
    if (vtype == kF32) hipLaunchKernelGGL(k_fetch<float>, g, dim3(256), 0, st, (const float*)shard, alpha, cols, keys, key_lo, n, first, out, rec, K, value_slot);
    else if (vtype == kI32) hipLaunchKernelGGL(k_fetch<int32_t>, g, dim3(256), 0, st, (const int32_t*)shard, alpha, cols, keys, key_lo, n, first, out, rec, K, value_slot);
    else hipLaunchKernelGGL(k_fetch<double>, g, dim3(256), 0, st, (const double*)shard, alpha, cols, keys, key_lo, n, first, out, rec, K, value_slot);
    return hipGetLastError();
}

// Big-endian <-> native byte swap (DataOutputStream.writeFloat/writeInt/writeDouble).
__global__ void k_bswap4(const uint32_t* __restrict__ s, uint32_t* __restrict__ d, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = __builtin_bswap32(s[i]);
}
__global__ void k_bswap8(const uint64_t* __restrict__ s, uint64_t* __restrict__ d, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = __builtin_bswap64(s[i]);
}
hipError_t launch_bswap(int V, const void* src, void* dst, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (V == 4) hipLaunchKernelGGL(k_bswap4, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)src, (uint32_t*)dst, n);
    else hipLaunchKernelGGL(k_bswap8, dim3(grid_for(n)), dim3(256), 0, st, (const uint64_t*)src, (uint64_t*)dst, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Synthetic data (DESIGN.md §Synthetic data; CPU twin: oracle/dml_oracle.c).
__device__ inline int32_t synth_grad_int(uint64_t h) {
    const int32_t s = (int32_t)(h & 0xFFFF) + (int32_t)((h >> 16) & 0xFFFF) + (int32_t)((h >> 32) & 0xFFFF) +
                      (int32_t)((h >> 48) & 0xFFFF);
    return s - 131070;
}
__device__ inline void put_value(uint8_t* p, int vtype, uint64_t h) {
    if (vtype == kF32) {
        st32(p, __float_as_uint((float)synth_grad_int(h) * 0x1p-25f));
    } else if (vtype == kF64) {
        const uint64_t u = __builtin_bit_cast(uint64_t, (double)synth_grad_int(h) * 0x1p-25);
        st32(p, (uint32_t)u); st32(p + 4, (uint32_t)(u >> 32));
    } else {
        st32(p, (uint32_t)((int32_t)(h % 5) - 2));
    }
}
__device__ inline void put_key(uint8_t* p, int K, int64_t key) {
    st32(p, (uint32_t)key);
    if (K == 8) st32(p + 4, (uint32_t)((uint64_t)key >> 32));
}

// perm: record r -> row (pa*r + pc) mod n; host guarantees pa < 2^32, r < 2^32.
__global__ void k_synth_dense(uint8_t* __restrict__ out, int K, int vtype, int64_t first, int64_t shard_rows,
                              int64_t nrec, int32_t cols, uint64_t s0, uint64_t pa, uint64_t pc) {
    const int V = vtype == kF64 ? 8 : 4;
    const int64_t stride = K + (int64_t)V * cols;
    const int64_t total = nrec * (int64_t)cols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / cols;
        const int32_t c = (int32_t)(t - r * cols);
        const uint64_t row = ((pa * (uint64_t)r) % (uint64_t)shard_rows + pc) % (uint64_t)shard_rows;
        uint8_t* rec = out + r * stride;
        if (c == 0) put_key(rec, K, first + (int64_t)row);
        put_value(rec + K + (int64_t)V * c, vtype, splitmix64_dev(s0 + row * (uint64_t)cols + (uint64_t)c));
    }
}
hipError_t launch_synth_dense(uint8_t* out, int K, int vtype, int64_t first, int64_t shard_rows, int64_t nrec,
                              int32_t cols, uint64_t s0, uint64_t pa, uint64_t pc, hipStream_t st) {
    hipLaunchKernelGGL(k_synth_dense, dim3(8192), dim3(256), 0, st, out, K, vtype, first, shard_rows, nrec, cols, s0, pa, pc);
    return hipGetLastError();
}

__global__ void k_synth_sparse(uint8_t* __restrict__ out, int K, int vtype, int value_stride, int64_t first,
                               int64_t key_space, int64_t nrec, uint64_t s0, uint64_t pa, uint64_t pc) {
    const int64_t stride = K + value_stride;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrec; r += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t i = ((pa * (uint64_t)r) % (uint64_t)key_space + pc) % (uint64_t)key_space;
        uint8_t* rec = out + r * stride;
        put_key(rec, K, first + (int64_t)i);
        for (int z = 0; z < value_stride; z += 4) st32(rec + K + z, 0u);
        put_value(rec + K, vtype, splitmix64_dev(s0 + i));
    }
}
hipError_t launch_synth_sparse(uint8_t* out, int K, int vtype, int value_stride, int64_t first, int64_t key_space,
                               int64_t nrec, uint64_t s0, uint64_t pa, uint64_t pc, hipStream_t st) {
    hipLaunchKernelGGL(k_synth_sparse, dim3(8192), dim3(256), 0, st, out, K, vtype, value_stride, first, key_space, nrec,
                       s0, pa, pc);
    return hipGetLastError();
}

__global__ void k_synth_fill(int vtype, void* p, int64_t n, uint64_t s0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = splitmix64_dev(s0 + (uint64_t)i);
        if (vtype == kF32) ((float*)p)[i] = (float)((int32_t)(h % 100) - 50) * 0x1p-17f;
        else if (vtype == kF64) ((double*)p)[i] = (double)((int32_t)(h % 100) - 50) * 0x1p-17;
        else ((int32_t*)p)[i] = 64 + (int32_t)(h % 51);
    }
}
// Streaming ceilings (diagnostic): 4 independent 16-B nt loads per lane in
// flight, contiguous 4 KiB per wave step. COPY writes what it reads; READ folds
// the loads into one word that is stored only if it hits a sentinel.
template <bool COPY>
__global__ __launch_bounds__(256) void k_stream(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                int64_t n16) {
    const int64_t lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t fold = 0;
    for (int64_t base = wave * 256; base < n16; base += nwaves * 256) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = base + j * 64 + lane;
            v[j] = ldg16_nt(src + (i < n16 ? i : 0) * 16);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = base + j * 64 + lane;
            if constexpr (COPY) {
                if (i < n16) stg16(dst + i * 16, v[j]);
            } else {
                fold ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
            }
        }
    }
    if constexpr (!COPY)
        if (fold == 0x9E3779B9u) *(uint32_t*)dst = fold;
}

// Ring reduce-scatter footprint (diagnostic, bench.py --emulate-rs): the local HBM
// traffic of one rank's ring reduce-scatter, as ONE kernel of `channels` blocks
// (RCCL runs one persistent block per channel). world - 1 steps: step s reads the
// chunk the rank sends, (rank - s - 1) mod world, plus the chunk that arrived at
// step s - 1, and writes their sum where the next rank's write would land (a local
// stand-in for the peer's write into this rank's buffer); the last step adds the
// rank's own chunk into recv. A thread owns the same vectors in every step, so the
// steps need no synchronization. Values are meaningless (no peer contributes).
template <typename T>
__global__ __launch_bounds__(256) void k_ring_rs(const T* __restrict__ part, T* __restrict__ recv,
                                                 T* __restrict__ land, int64_t chunk16, int world, int rank) {
    constexpr int VEC = Elem<T>::VEC, U = 8;  // 8 vectors per thread per step in flight, as RCCL's unrolled copies
    const uint8_t* P = (const uint8_t*)part;
    uint8_t* Lb[2] = {(uint8_t*)land, (uint8_t*)land + chunk16 * 16};
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < chunk16; i0 += nthr * U) {
        for (int s2 = 0; s2 < world; ++s2) {
            const int64_t c = s2 == world - 1 ? rank : ((rank - s2 - 1) % world + world) % world;
            u32x4 xa[U], ya[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * nthr;
                xa[u] = i < chunk16 ? ldg16_nt(P + (c * chunk16 + i) * 16) : u32x4{0u, 0u, 0u, 0u};
                ya[u] = (s2 > 0 && i < chunk16) ? ldg16_nt(Lb[s2 & 1] + i * 16) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * nthr;
                if (i >= chunk16) continue;
                T x[VEC], y[VEC];
                unpack<T>(xa[u], x);
                unpack<T>(ya[u], y);
#pragma unroll
                for (int e = 0; e < VEC; ++e) x[e] = Elem<T>::add(x[e], y[e]);
                stg16_nt((s2 == world - 1 ? (uint8_t*)recv : Lb[(s2 + 1) & 1]) + i * 16, pack<T>(x));
            }
        }
    }
}

hipError_t launch_ring_rs(int vtype, const void* part, void* recv, void* land, int64_t chunk_bytes, int world,
                          int rank, int channels, hipStream_t st) {
    const int64_t n16 = chunk_bytes / 16;
    if (n16 <= 0) return hipSuccess;
    const dim3 g((unsigned)std::max(1, channels)), blk(256);
    if (vtype == kF64)
        hipLaunchKernelGGL(k_ring_rs<double>, g, blk, 0, st, (const double*)part, (double*)recv, (double*)land, n16,
                           world, rank);
    else if (vtype == kI32)
        hipLaunchKernelGGL(k_ring_rs<int32_t>, g, blk, 0, st, (const int32_t*)part, (int32_t*)recv, (int32_t*)land,
                           n16, world, rank);
    else
        hipLaunchKernelGGL(k_ring_rs<float>, g, blk, 0, st, (const float*)part, (float*)recv, (float*)land, n16,
                           world, rank);
    return hipGetLastError();
}

// Random-RMW floor (diagnostic): one plain 4-B read-modify-write per update over a
// globally sorted index list — the best case of config 3's scatter-add (every update
// in address order, no partition), against which the leaf kernel is judged.
// Repeated indices race: the array's values are not meaningful afterwards.
__global__ __launch_bounds__(256) void k_rmw_floor(float* __restrict__ a, const uint32_t* __restrict__ idx,
                                                   const float* __restrict__ v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = idx[i];
        a[k] = a[k] + v[i];
    }
}

hipError_t launch_rmw_floor(float* a, const uint32_t* idx, const float* v, int64_t n, hipStream_t st, LaunchEv ev) {
    if (n <= 0) return hipSuccess;
    // one update per thread up to 2^28 updates (config 3: 32e6), grid-stride beyond
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)1 << 20);
    hipExtLaunchKernelGGL(k_rmw_floor, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, a, idx, v, n);
    return hipGetLastError();
}

// Row-gather floor (diagnostic, config 5): the touched rows of an int32 shard in row
// order, each read once, every record that lists it (listed in push order by the
// caller, `addr` = the record's value bytes) gathered and added, the row written once
// — the same bytes as the IntMatrixStore reduce with no key index, slot table,
// negativity check or error bookkeeping. One wave per touched row (<= 256 16-B
// vectors: cols <= 1024), four records' loads in flight, XCD-contiguous blocks as the
// product's DEPTH-3 reduce. The values are meaningful (plain wrapping int adds).
__global__ __launch_bounds__(256) void k_gather_floor(int32_t* __restrict__ shard, int32_t cols,
                                                      const int32_t* __restrict__ trow, const int32_t* __restrict__ tptr,
                                                      const uint64_t* __restrict__ addr, int64_t ntouched) {
    const int64_t w = xcd_block() * 4 + (threadIdx.x >> 6);
    if (w >= ntouched) return;
    const int lane = threadIdx.x & 63, nvec = cols / 4;
    uint8_t* rowp = (uint8_t*)(shard + (int64_t)trow[w] * cols);
    const int32_t b0 = tptr[w], b1 = tptr[w + 1];
    u32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int v = lane + 64 * j;
        acc[j] = v < nvec ? ldg16_nt(rowp + v * 16) : u32x4{0u, 0u, 0u, 0u};
    }
    for (int32_t e = b0; e < b1; e += 4) {
        u32x4 x[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t a = e + k < b1 ? uni64(addr[e + k]) : 0ull;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int v = lane + 64 * j;
                x[k][j] = (a && v < nvec) ? ldg16_nt((const uint8_t*)a + v * 16) : u32x4{0u, 0u, 0u, 0u};
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += x[k][j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int v = lane + 64 * j;
        if (v < nvec) stg16_nt(rowp + v * 16, acc[j]);
    }
}

hipError_t launch_gather_floor(int32_t* shard, int32_t cols, const int32_t* trow, const int32_t* tptr,
                               const uint64_t* addr, int64_t ntouched, hipStream_t st, LaunchEv ev) {
    if (ntouched <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((ntouched + 3) / 4);
    hipExtLaunchKernelGGL(k_gather_floor, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, shard, cols, trow, tptr,
                          addr, ntouched);
    return hipGetLastError();
}

// Dense stream floor (diagnostic, config 4 and its AdaGrad variant): the shard's
// elements in order, each read once with the same element of every full-range push
// whose records are rows in order (record r = row r, values 4 bytes after the key),
// summed in push order and written once — to `out` (the speculative second buffer,
// as k_flat_ident writes it) or in place; ADA: delta += u·u beside it (AdaGrad's
// data / delta stream, k_ada_ident's bytes). No key checks, slot tables or maxDelta
// bookkeeping: the plain stream of the same bytes, over the same allocations.
template <bool ADA>
__global__ __launch_bounds__(256) void k_dense_floor(const float* __restrict__ data, float* __restrict__ out,
                                                     float* __restrict__ delta, Batch bt, int nb, int64_t stride,
                                                     int K, int32_t cols, int64_t nvec) {
    constexpr int U = 2, D = 4;
    const int64_t v0 = xcd_block() * (256 * U) + threadIdx.x;
    int64_t off[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = v0 + u * 256, e = v * 4;
        ok[u] = v < nvec;
        off[u] = (e / cols) * stride + K + (e % cols) * 4;
    }
    u32x4 acc[U], dl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = v0 + u * 256;
        acc[u] = ok[u] ? ldg16_nt((const uint8_t*)data + v * 16) : u32x4{0u, 0u, 0u, 0u};
        if (ADA) dl[u] = ok[u] ? ldg16_nt((const uint8_t*)delta + v * 16) : u32x4{0u, 0u, 0u, 0u};
    }
    for (int b = 0; b < nb; b += D) {
        u32x4 x[D][U];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int u = 0; u < U; ++u)
                x[d][u] = (b + d < nb && ok[u]) ? ldg16_nt(bt.base[b + d] + off[u]) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (b + d >= nb) break;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float g = __uint_as_float(x[d][u][e]);
                    acc[u][e] = __float_as_uint(__fadd_rn(__uint_as_float(acc[u][e]), g));
                    if (ADA) dl[u][e] = __float_as_uint(__fadd_rn(__uint_as_float(dl[u][e]), __fmul_rn(g, g)));
                }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const int64_t v = v0 + u * 256;
        stg16_nt((uint8_t*)out + v * 16, acc[u]);
        if (ADA) stg16_nt((uint8_t*)delta + v * 16, dl[u]);
    }
}

hipError_t launch_dense_floor(const float* data, float* out, float* delta, const Batch& bt, int nb, int64_t stride,
                              int K, int32_t cols, int64_t elems, hipStream_t st, LaunchEv ev) {
    const int64_t nvec = elems / 4;
    if (nvec <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((nvec + 511) / 512);
    if (delta)
        hipExtLaunchKernelGGL(k_dense_floor<true>, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, data, out, delta,
                              bt, nb, stride, K, cols, nvec);
    else
        hipExtLaunchKernelGGL(k_dense_floor<false>, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, data, out,
                              delta, bt, nb, stride, K, cols, nvec);
    return hipGetLastError();
}

hipError_t launch_stream(bool copy, void* dst, const void* src, int64_t n16, hipStream_t st, LaunchEv ev) {
    if (n16 <= 0) return hipSuccess;
    const int64_t want = (n16 + 1023) / 1024;  // one 256-thread block per 4 wave steps
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, 256 * 16));
    if (copy)
        hipExtLaunchKernelGGL(k_stream<true>, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, (uint8_t*)dst,
                              (const uint8_t*)src, n16);
    else
        hipExtLaunchKernelGGL(k_stream<false>, dim3(grid), dim3(256), 0, st, ev.start, ev.stop, 0, (uint8_t*)dst,
                              (const uint8_t*)src, n16);
    return hipGetLastError();
}

// DataStore.rand() distributions (dml_store_rand). f32: (a/100f - 0.5f)/cols,
// a uniform in 0..99, float arithmetic as in FloatMatrixStore.java:46-47.
// f64: one thread per row, |N(0,1)| (Box-Muller) then the row over its L2 norm
// (DoubleMatrixStore.java:196-206).
__global__ void k_rand_f32(float* p, int64_t n, int32_t cols, uint64_t s0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(splitmix64_dev(s0 + (uint64_t)i) % 100u);
        p[i] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)a, 100.0f), 0.5f), (float)cols);
    }
}
__device__ inline double rand_abs_gauss(uint64_t h) {
    const double u1 = (double)((h >> 11) + 1) * 0x1p-53;                   // (0, 1]
    const double u2 = (double)(splitmix64_dev(h) >> 11) * 0x1p-53;          // [0, 1)
    return fabs(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}
__global__ void k_rand_f64_rows(double* p, int64_t rows, int32_t cols, uint64_t s0) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        double* row = p + r * cols;
        double sum = 0.0;
        for (int32_t j = 0; j < cols; ++j) {
            const double g = rand_abs_gauss(splitmix64_dev(s0 + (uint64_t)(r * cols + j)));
            row[j] = g;
            sum = __dadd_rn(sum, __dmul_rn(g, g));
        }
        sum = sqrt(sum);
        for (int32_t j = 0; j < cols; ++j) row[j] = __ddiv_rn(row[j], sum);
    }
}
hipError_t launch_rand(int vtype, void* p, int64_t rows, int32_t cols, uint64_t s0, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    if (vtype == kF32) hipLaunchKernelGGL(k_rand_f32, dim3(grid_for(rows * cols)), dim3(256), 0, st, (float*)p, rows * cols, cols, s0);
    else if (vtype == kF64) hipLaunchKernelGGL(k_rand_f64_rows, dim3(grid_for(rows)), dim3(256), 0, st, (double*)p, rows, cols, s0);
    return hipGetLastError();
}

hipError_t launch_synth_fill(int vtype, void* p, int64_t n, uint64_t s0, hipStream_t st) {
    hipLaunchKernelGGL(k_synth_fill, dim3(8192), dim3(256), 0, st, vtype, p, n, s0);
    return hipGetLastError();
}

// Row index of every record of one push (-1 outside the shard): the host's
// duplicate-row replay reads these to split the push into unique-row layers.
__global__ void k_key_rows(const uint8_t* __restrict__ base, int64_t nrec, int64_t stride, int K, int64_t first,
                           int64_t rows, int32_t* __restrict__ out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrec; r += (int64_t)gridDim.x * blockDim.x)
        out[r] = (int32_t)row_index(ld_key(base + r * stride, K), first, rows);
}
hipError_t launch_key_rows(const uint8_t* base, int64_t nrec, int64_t stride, int K, int64_t first, int64_t rows,
                           int32_t* out, hipStream_t st) {
    if (nrec <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_key_rows, dim3(grid_for(nrec)), dim3(256), 0, st, base, nrec, stride, K, first, rows, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Two-moment AdaGrad reduce-scatter: the sharded
// AdaGrad path whose xGMI bytes do not grow with the pushes per rank. Each rank
// pre-reduces its full-range pushes into Σu and Σu·u per element (fp32, push
// order; u·u rounded, then added, like the reference's delta update,
// FloatMatrixStoreAdaGrad.java:265-267), written as one [row][2 x cols] run so a
// rank's share of both is one contiguous reduce-scatter chunk; the owner applies
// row += Σu, delta += Σu², and alpha = f(final delta) where it ends above 1
// (:268-272: delta never falls, so the last push that sets alpha sees the final
// delta). The summation order is not the reference's: within 1e-6, not bit-exact.
//
// k_moments_flat: k_reduce_flat's layout (R rows per wave as one flat run of
// 16-B vectors), slot rows in LDS unless every push is identity (Batch::ident_ok).
// A call whose index met a key outside the matrix or a repeated row writes zeros
// (dml_prereduce_end reports the error; nothing of it is applied).
template <int JMAX>
__global__ __launch_bounds__(256) void k_moments_flat(int64_t ntask, int32_t cols, int32_t R, const Batch bt, int nb,
                                                      int64_t stride, int K, int32_t* __restrict__ slot,
                                                      const Ctrl* __restrict__ ctrl, RowMap rm) {
    constexpr int VEC = 4;
    constexpr int RMAX = 16;
    __shared__ int32_t s_slot[4][RMAX * kMaxW];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t t0 = (xcd_block() * 4 + wid) * R;  // first task row of the wave (XCD-contiguous, as k_reduce_flat)
    if (t0 >= ntask) return;
    const int NV = cols / VEC;
    const int nrow = (int)(ntask - t0 < (int64_t)R ? ntask - t0 : (int64_t)R);
    const int ss = slot_stride(nb);
    int32_t* const ls = s_slot[wid];
    const uint64_t ident = bt.ident_ok ? ctrl->ident : 0ull;
    const uint64_t nbm = nb >= 64 ? ~0ull : (1ull << nb) - 1ull;
    const bool all_id = (ident & nbm) == nbm;
    const bool err = ctrl->cutoff != kNoPos || ctrl->no_dup == 0u;
    const int64_t lrow = rm.row(t0 + lane);
    const uint32_t padm = (uint32_t)__ballot(lane < nrow && lrow >= rm.rows_total);
    if (!all_id) {
        // slot rows into LDS, handed back clean (-1) like k_reduce_flat's
        for (int e = lane; e < nrow * nb; e += 64) {
            const int rl = e / nb, b = e - rl * nb;
            const int64_t mr = rm.row(t0 + rl);
            int32_t v = -1;
            if (!((padm >> rl) & 1u)) {
                if ((ident >> b) & 1ull) {
                    v = mr < bt.nrec[b] ? (int32_t)mr : -1;
                } else {
                    v = slot[mr * ss + b];
                    if (v >= 0) slot[mr * ss + b] = -1;
                }
            }
            ls[rl * kMaxW + b] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    int rc[JMAX];
    uint32_t on = 0;
    float acc[JMAX][VEC], sq[JMAX][VEC];
    const int nvec = nrow * NV;
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
        const int v = j * 64 + lane;
        const int rlj = v < nvec ? v / NV : 0;
        const int cvj = v < nvec ? v - rlj * NV : 0;
        rc[j] = (rlj << 16) | cvj;
        on |= ((v < nvec && !((padm >> rlj) & 1u) && !err) ? 1u : 0u) << j;
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[j][e] = sq[j][e] = 0.f;
    }
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        const uint8_t* const bp = bt.base[b];
        int32_t rr[JMAX];
        u32x4 raw[JMAX];
#pragma unroll
        for (int j = 0; j < JMAX; ++j) {
            const int rl = rc[j] >> 16;
            rr[j] = (on >> j & 1u) ? (all_id ? (int32_t)rm.row(t0 + rl) : ls[rl * kMaxW + b]) : -1;
            raw[j] = rr[j] >= 0 ? ldg16_nt(bp + (int64_t)rr[j] * stride + K + (int64_t)(rc[j] & 0xFFFF) * 16)
                                : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < JMAX; ++j) {
            if (rr[j] < 0) continue;
            float u[VEC];
            unpack<float>(raw[j], u);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                acc[j][e] = __fadd_rn(acc[j][e], u[e]);
                sq[j][e] = __fadd_rn(sq[j][e], __fmul_rn(u[e], u[e]));
            }
        }
    }
    float* const out = (float*)rm.out;
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
        if (j * 64 + lane >= nvec) continue;
        float* const op = out + (t0 + (rc[j] >> 16)) * (int64_t)(2 * cols) + (rc[j] & 0xFFFF) * VEC;
        stg16(op, pack<float>(acc[j]));
        stg16(op + cols, pack<float>(sq[j]));
    }
}

hipError_t launch_moments(int64_t ntask, int32_t cols, const Batch& bt, int nb, int64_t stride, int K, int32_t* slot,
                          const Ctrl* ctrl, RowMap rm, hipStream_t st, LaunchEv ev) {
    constexpr int JMAX = 8;
    if (cols % 4 || cols * 4 >= 4096 || !rm.out) return hipErrorInvalidValue;  // the flat shapes
    const int NV = cols / 4;
    const int R = std::max(1, std::min(16, JMAX * 64 / NV));
    const int64_t nblocks = ((ntask + R - 1) / R + 3) / 4;
    if (nblocks <= 0) return hipSuccess;
    g_kernel_name = "dml::k_moments_flat<8>";
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL((k_moments_flat<JMAX>), dim3((unsigned)nblocks), dim3(256), 0, st, ev.start, ev.stop, 0,
                              ntask, cols, R, bt, nb, stride, K, slot, ctrl, rm);
    else
        hipLaunchKernelGGL((k_moments_flat<JMAX>), dim3((unsigned)nblocks), dim3(256), 0, st, ntask, cols, R, bt, nb,
                           stride, K, slot, ctrl, rm);
    return hipGetLastError();
}

// Owner apply of the reduce-scattered moments ([row][Σu | Σu²], rows x 2 cols):
// data += Σu, delta += Σu², alpha = f(delta) where delta ends above 1, each
// element's strict rise of delta its maxDelta candidate (ties: first in row-major
// order). One candidate per block into ada.cand.
__global__ __launch_bounds__(256) void k_ada_moments(float* __restrict__ shard, const float* __restrict__ src,
                                                     int64_t rows, int32_t cols, AdaArgs ada) {
    const int NV = cols / 4;
    const int64_t nvec = rows * NV;
    float cand_v = 0.f;
    uint64_t cand_p = kNoPos;
    bool cand_ok = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / NV;
        const int cv = (int)(i - r * NV);
        const int64_t ei = r * cols + cv * 4;
        const float* sp = src + r * (int64_t)(2 * cols) + cv * 4;
        float a[4], d[4], su[4], s2[4];
        unpack<float>(ldg16_nt((const uint8_t*)(shard + ei)), a);
        unpack<float>(ldg16_nt((const uint8_t*)(ada.delta + ei)), d);
        unpack<float>(ldg16((const uint8_t*)sp), su);
        unpack<float>(ldg16((const uint8_t*)(sp + cols)), s2);
        float na[4];
        bool all_a = true;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            a[e] = __fadd_rn(a[e], su[e]);
            const float nd = __fadd_rn(d[e], s2[e]);
            if (nd > d[e] && (!cand_ok || nd > cand_v)) {  // elements visited in row-major order per thread
                cand_ok = true;
                cand_v = nd;
                cand_p = (uint64_t)(ei + e);
            }
            d[e] = nd;
            na[e] = 0.f;
            if (nd > 1.0f) {
                na[e] = (float)((double)ada.initial_alpha / ((double)ada.factor * sqrt((double)nd)));
                if (na[e] < ada.min_alpha) na[e] = ada.min_alpha;
            } else {
                all_a = false;
            }
        }
        stg16_nt(shard + ei, pack<float>(a));
        stg16_nt(ada.delta + ei, pack<float>(d));
        if (all_a) {
            stg16_nt(ada.alpha + ei, pack<float>(na));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (d[e] > 1.0f) ada.alpha[ei + e] = na[e];
        }
    }
    cand_block_best<4>(cand_ok, cand_v, cand_p);
    if (threadIdx.x == 0) {
        DeltaCand c;
        c.value = cand_v;
        c.valid = cand_ok;
        c.pos = cand_p;
        ada.cand[blockIdx.x] = c;
    }
}

// maxDelta finalize for element-index candidates (k_ada_moments): the reference's
// strict `>` against the running maximum; row = the element's key (first + row).
__global__ __launch_bounds__(256) void k_maxdelta_elems(const DeltaCand* __restrict__ cand, int64_t n,
                                                        MaxDelta* __restrict__ md, int64_t first, int32_t cols) {
    bool ok = false;
    float v = 0.f;
    uint64_t p = kNoPos;
    cand_scan(cand, threadIdx.x, n, 256, ok, v, p);
    cand_block_best<4>(ok, v, p);
    if (threadIdx.x != 0) return;
    if (ok && v > md->value) {
        md->value = v;
        md->row = (int32_t)(first + (int64_t)(p / (uint64_t)cols));
        md->col = (int32_t)(p % (uint64_t)cols);
    }
}

hipError_t launch_ada_moments(float* shard, const float* src, int64_t rows, int32_t cols, const AdaArgs& ada,
                              MaxDelta* md, int64_t first, hipStream_t st, LaunchEv ev) {
    if (cols % 4 || rows <= 0) return hipErrorInvalidValue;
    g_kernel_name = "dml::k_ada_moments";
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL(k_ada_moments, dim3(kMomentBlocks), dim3(256), 0, st, ev.start, ev.stop, 0, shard, src,
                              rows, cols, ada);
    else
        hipLaunchKernelGGL(k_ada_moments, dim3(kMomentBlocks), dim3(256), 0, st, shard, src, rows, cols, ada);
    hipLaunchKernelGGL(k_maxdelta_elems, dim3(1), dim3(256), 0, st, ada.cand, (int64_t)kMomentBlocks, md, first, cols);
    return hipGetLastError();
}

}  // namespace dml
