"""One-off source patch (kept for the record): stream-priority knob in the store,
and a two-deep register ring (DEPTH = 2) in k_reduce_rows."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sub(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new, 1)


p = os.path.join(ROOT, "distml_amd/csrc/dml_store.hip")
s = open(p).read()
if "DML_STREAM_PRIO" not in s:
    s = sub(s, '''    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
    const size_t nbytes''', '''    hipError_t e;
    // DML_STREAM_PRIO=1: apply stream at high priority, index stream at low priority
    // (the next chunk's index then fills the wave slots the reduce leaves free).
    static const int prio_mode = getenv("DML_STREAM_PRIO") ? atoi(getenv("DML_STREAM_PRIO")) : 0;
    int prio_least = 0, prio_greatest = 0;
    if (prio_mode) (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    if ((e = prio_mode ? hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, prio_greatest)
                       : hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess)
        return fail(e, "stream");
    const size_t nbytes''')
    s = sub(s, '''    if ((e = hipStreamCreateWithFlags(&s->istream, hipStreamNonBlocking)) != hipSuccess) return fail(e, "index stream");''',
            '''    if ((e = prio_mode ? hipStreamCreateWithPriority(&s->istream, hipStreamNonBlocking, prio_least)
                       : hipStreamCreateWithFlags(&s->istream, hipStreamNonBlocking)) != hipSuccess)
        return fail(e, "index stream");''')
    open(p, "w").write(s)

p = os.path.join(ROOT, "distml_amd/csrc/dml_kernels.hip")
s = open(p).read()
if "DEPTH" not in s:
    s = sub(s, "template <typename T, int MODE, int CPW, int RPW, bool NT, bool FULL>\n__global__",
            "template <typename T, int MODE, int CPW, int RPW, bool NT, bool FULL, int DEPTH>\n__global__")
    s = sub(s, '''    const uint64_t vbase = lane < nb ? (uint64_t)bt.base[lane] : 0ull;
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {''', '''    const uint64_t vbase = lane < nb ? (uint64_t)bt.base[lane] : 0ull;
    if constexpr (DEPTH == 2) {
        static_assert(FULL, "two-deep ring: whole-vector rows only");
        // Two pushes' loads in flight (a ring of two register sets): push b+2's loads
        // are issued as soon as push b is added, so the wave never drains its loads.
        // Absent rows and pushes past the batch load a live row (an L2 hit) and add nothing.
        auto issue = [&](int b, u32x4 (&raw)[RPW][CPW], unsigned& h, int32_t (&rrb)[RPW]) {
            const int bb = b < nb ? b : (nb > 0 ? nb - 1 : 0);
            const uint8_t* bp =
                (const uint8_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vbase, bb)) |
                                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vbase >> 32), bb) << 32));
            h = 0;
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                rrb[r] = b < nb ? __builtin_amdgcn_readlane(vslot[r], bb) : -1;
                h |= (rrb[r] >= 0 ? 1u : 0u) << r;
                const uint8_t* rb = rrb[r] >= 0 ? bp + (int64_t)rrb[r] * stride + voff[0] : fbv;
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    const uint8_t* src = rb + c * 64 * VEC * (int)sizeof(T);
                    raw[r][c] = NT ? ldg16_nt(src) : ldg16(src);
                }
            }
        };
        auto consume = [&](const u32x4 (&raw)[RPW][CPW], unsigned h, const int32_t (&rrb)[RPW], int b) {
            touched |= h;
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const bool on = (h >> r) & 1u;
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    T t[VEC];
                    unpack<T>(raw[r][c], t);
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        const T sum = Elem<T>::add(acc[r][c][e], t[e]);
                        if constexpr (MODE == kAddCheckI32) {
                            if (on && sum < 0) {
                                const uint64_t p = pos_of((uint64_t)bt.bidx[b < nb ? b : 0],
                                                          (uint64_t)((int64_t)rrb[r] * stride + voff[c] + e * (int64_t)sizeof(T)));
                                negpos = p < negpos ? p : negpos;
                            }
                        }
                        acc[r][c][e] = on ? sum : acc[r][c][e];  // a select: an absent row keeps its bits (-0.0)
                    }
                }
            }
        };
        u32x4 ra[RPW][CPW], rb2[RPW][CPW];
        unsigned ha, hb;
        int32_t rra[RPW], rrb2[RPW];
        issue(0, ra, ha, rra);
        issue(1, rb2, hb, rrb2);
#pragma unroll 1
        for (int b = 0; b < nb; b += 2) {
            consume(ra, ha, rra, b);
            issue(b + 2, ra, ha, rra);
            consume(rb2, hb, rrb2, b + 1);
            issue(b + 3, rb2, hb, rrb2);
        }
    } else
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {''')
    for a in ("hipExtLaunchKernelGGL((k_reduce_rows<T, MODE, CPW, RPW, NT, FULL>)",
              "hipLaunchKernelGGL((k_reduce_rows<T, MODE, CPW, RPW, NT, FULL>)"):
        s = sub(s, a, a.replace("FULL>)", "FULL, (FULL && G == 2) ? 2 : 1>)"))
    s = sub(s, '''                case 28: return''', '''                case 30: return launch_reduce_t<float, kAdd, 2, true, 4, false, 4, 4, true>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev);
                case 31: return launch_reduce_t<float, kAdd, 2, true, 4, false, 4, 2, true>(shard, rows, cols, bt, nb, stride, K, slot, rowflag, ctrl, tail_cut, ada, st, nblocks_out, ev);
                case 28: return''')
    s = sub(s, "// 28: CPW4/RPW2 FULL (0 = auto: CPW4/RPW4 FULL for config 2).",
            "// 28: CPW4/RPW2 FULL, 30: CPW4/RPW4 FULL two-deep ring, 31: CPW4/RPW2 FULL two-deep ring\n"
            "// (0 = auto: CPW4/RPW4 FULL for config 2).")
    open(p, "w").write(s)
print("patched")
