/*
 * msssp.hip -- multi-source shared-frontier SSSP for sparse graphs (gfx950): 64 sources per
 * workgroup, one per lane, so every arc and every frontier vertex is loaded once for all 64.
 *
 * Replaces, for the eager all-pairs build, the per-source igraph Dijkstra of
 * /root/reference/src/main/routing/topology.c:1578-1814 and the per-hop path walk of :1286-1389
 * (latency sum :1364, reliability product :1308-1309 / :1365) -- for a batch of 64 sources at a
 * time.
 *
 * Layout. The graph runs in its Cuthill-McKee relabelling (build.hip), rows keep their arcs in
 * ORIGINAL neighbour order. A batch's working state is transposed: D[v][lane] (u32 quanta) and
 * R[v][lane] (f64), so one vertex is one 256-byte + one 512-byte coalesced access for all 64
 * sources. Batches are compact clusters of sources (grown breadth-first on the host), so the 64
 * distance fields are close to each other everywhere and their frontiers overlap.
 *
 * Algorithm (frontier Bellman-Ford with delta-stepping over the lane minimum). A PULL recomputes
 * a candidate vertex v from all of its in-arcs, per lane:
 *   D[v] = min over in-arcs (D[u] + w), ties broken by (D[u], u)  -- the canonical predecessor
 *          argmin (D[s][u], u) over tight in-arcs, with u in original
 *          order because a row's arcs are sorted that way;
 *   R[v] = R[pred] * r(pred, v)                                    -- the path-order product;
 *   the source lane keeps D = 0, R = 1.
 * A pull whose (D, R) changed in any lane propagates: v's out-neighbours become candidates of the
 * next pass -- once v's lane minimum is below the bucket bound T; otherwise v waits in the
 * pending set until T passes it (T advances by delta when no candidate is left). The unique fixed
 * point of these equations (positive weights) is the exact distance, the canonical predecessor
 * and the left-to-right reliability product, i.e. what the per-source Dijkstra settles: every
 * change of a vertex schedules a re-pull of each out-neighbour after a barrier, so when no
 * candidate and no pending vertex is left, every vertex was last pulled from the final states of
 * its in-neighbours. Reads of a neighbour being rewritten in the same pass (torn D/R) are
 * corrected by that same rule. tools/msssp_sim.c models this and checks it against oracle/.
 *
 * Frontier bookkeeping is in LDS: candidate bitmaps (this pass / next pass) and the pending
 * bitmap. A batch starts by setting its D rows to INF (R is read only where D is finite, so it
 * needs no initialisation): a neighbour row is then always a real upper bound, never stale data
 * of the previous batch, which would break the monotone convergence above. A pass compacts the
 * candidate bitmap into an LDS list (wave scan of popcounts, one LDS atomic per wave) and the 16
 * waves pull its entries; a changed vertex sets its
 * out-neighbours' bits in the next pass's bitmap right away (undirected: from the arcs it just
 * loaded). Output: the rows are transposed into lat[row][t] / rel[row][t] in original vertex
 * order with coalesced stores.
 */
#include <type_traits>

#include "srt_device.h"

#define MS_L 64     /* sources per batch (lanes) */
#define MS_WG 512   /* threads per workgroup (two batches per CU) */
#define MS_NWAVE (MS_WG / MS_L)
#define MS_LCAP 2048 /* LDS candidate list (a longer pass is processed in chunks) */
#define MS_G 4       /* candidates a wave pulls together */
#define MS_AC 16     /* arcs per candidate and chunk (MS_G x MS_AC lanes) */
#define MS_AK 8      /* arcs per candidate whose distance rows are loaded together */

static __device__ __forceinline__ uint32_t ms_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ uint32_t ms_ld(const uint16_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ double ms_ld(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ int ms_scan_excl(int v, int lane, int* total) {
    int x = v;
#pragma unroll
    for (int off = 1; off < MS_L; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, MS_L - 1);
    return x - v;
}
static __device__ __forceinline__ uint32_t ms_wave_min(uint32_t x) {
#pragma unroll
    for (int off = 32; off; off >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, off));
    return x;
}
static __device__ __forceinline__ bool ms_bit(const uint32_t* bm, uint32_t v) {
    return (bm[v >> 5] >> (v & 31)) & 1u;
}
static __device__ __forceinline__ void ms_set(uint32_t* bm, uint32_t v) {
    atomicOr(&bm[v >> 5], 1u << (v & 31));
}

/* Compacts the set bits of bm (nw words) into list (up to MS_LCAP entries, ascending within a
 * wave's words); consumed bits are cleared, bits that did not fit stay and set *more. */
static __device__ __forceinline__ void ms_compact(uint32_t* bm, int nw, int* list, int* cnt,
                                                  int* more, int tid, int lane) {
    for (int w0 = 0; w0 < nw; w0 += MS_WG) {
        const int wi = w0 + tid;
        const uint32_t word = wi < nw ? bm[wi] : 0u;
        const int pc = __popc(word);
        int tot;
        const int ex = ms_scan_excl(pc, lane, &tot);
        int base = 0;
        if (tot) {
            if (lane == 0) base = atomicAdd(cnt, tot);
            base = __shfl(base, 0);
        }
        if (pc) {
            int pos = base + ex;
            uint32_t rem = word;
            while (rem && pos < MS_LCAP) {
                list[pos++] = wi * 32 + (__ffs((int)rem) - 1);
                rem &= rem - 1u;
            }
            if (rem != word) bm[wi] = rem;
            if (rem) *more = 1;
        }
    }
}

/* One workgroup per batch of 64 sources (persistent over batches). orp/ocw: out-rows (begin,
 * end) and out-arcs (head, w), relabelled -- the expansion; irp/icw/ir: in-rows, in-arcs (tail,
 * w, tails in original order within a row) and their reliabilities -- the pull (the same arrays
 * for undirected graphs); inv[original] = relabelled; bsrc / brow: per batch and lane the
 * relabelled source and the output row (-1 = empty lane); ws: per slot D (n x 64 u32), R (n x 64
 * f64) and the lane minimum of every vertex (n u32). */
template <bool DIRECTED, typename DT>
__global__ __launch_bounds__(MS_WG, 4) void msssp_kernel(
    int n, const int2* __restrict__ orp, const uint2* __restrict__ ocw,
    const int2* __restrict__ irp, const uint2* __restrict__ icw, const double* __restrict__ ir,
    const int32_t* __restrict__ inv, int nbatch, const int32_t* __restrict__ bsrc,
    const int32_t* __restrict__ brow, uint32_t* __restrict__ lat, double* __restrict__ rel,
    size_t ldo, uint32_t* __restrict__ ws, size_t slot_words, uint32_t delta) {
    extern __shared__ uint32_t sm[];
    __shared__ int s_list[MS_LCAP];
    __shared__ int s_cnt, s_more;
    __shared__ uint32_t s_pmin;
    const int nw = (n + 31) >> 5;
    uint32_t* const bmA = sm;
    uint32_t* const bmB = sm + nw;
    uint32_t* const pend = sm + 2 * nw;
    const int tid = threadIdx.x, lane = tid & (MS_L - 1), wave = tid >> 6;
    /* DT: u32 quanta, or u16 when every finite distance is below 0xFFFF (the caller's bound);
     * DINF marks an unreached lane, and a u16 candidate saturates at DINF - 1 -- still an upper
     * bound of the true distance (<= the bound), so the fixed point is unchanged */
    constexpr uint32_t DINF = sizeof(DT) == 2 ? 0xFFFFu : SRT_INF;
    uint32_t* const wsb = ws + (size_t)blockIdx.x * slot_words;
    DT* const D = reinterpret_cast<DT*>(wsb);
    double* const R = reinterpret_cast<double*>(wsb + (size_t)n * MS_L);
    uint32_t* const mind = wsb + (size_t)n * MS_L * 3;

    for (int b = blockIdx.x; b < nbatch; b += gridDim.x) {
        for (int i = tid; i < 3 * nw; i += MS_WG) sm[i] = 0u;
        {
            uint4* d4 = reinterpret_cast<uint4*>(D);
            const uint32_t iw = sizeof(DT) == 2 ? 0xFFFFFFFFu : SRT_INF;
            const uint4 inf4 = make_uint4(iw, iw, iw, iw);
            for (size_t i = tid; i < (size_t)n * MS_L * sizeof(DT) / 16; i += MS_WG) d4[i] = inf4;
        }
        __syncthreads();
        const int mysrc = bsrc[(size_t)b * MS_L + lane];
        /* sources: D = 0 / R = 1 in the source's own lane; its out-neighbours are the first
         * pass's candidates */
        for (int l = wave; l < MS_L; l += MS_NWAVE) {
            const int s = bsrc[(size_t)b * MS_L + l];
            if (s < 0) continue;
            if (lane == l) {
                D[(size_t)s * MS_L + l] = (DT)0;
                R[(size_t)s * MS_L + l] = 1.0;
            }
            const int2 be = orp[s];
            for (int k = be.x + lane; k < be.y; k += MS_L) ms_set(bmA, ocw[k].x);
        }
        __syncthreads();
        if (tid < MS_L && mysrc >= 0) mind[mysrc] = 0u;
        uint32_t* cur = bmA;
        uint32_t* nxt = bmB;
        uint32_t T = delta;
        for (;;) {
            int found = 0;
            for (;;) { /* chunks of this pass's candidate list */
                if (tid == 0) {
                    s_cnt = 0;
                    s_more = 0;
                }
                __syncthreads();
                ms_compact(cur, nw, s_list, &s_cnt, &s_more, tid, lane);
                __syncthreads();
                const int cnt = min(s_cnt, MS_LCAP);
                const int more = s_more;
                found += cnt;
                /* a wave pulls MS_G consecutive list entries together, so their row, arc and
                 * distance loads share round trips: lane j < MS_G loads candidate j's in-row,
                 * lanes j * MS_AC + a its arcs a, a + MS_AC, ..., and the 64-lane distance rows
                 * of MS_G x MS_AK arcs are loaded back to back */
                /* this lane's arc slot: candidate lane / MS_AC, arc lane % MS_AC of a chunk */
                const int aj = lane / MS_AC, aa = lane % MS_AC;
                /* software pipeline: the next group's list entries, in-rows and first arc chunk
                 * are loaded while this group's distance rows are in flight, so a group's chain
                 * is its distance rows, then its reliability gathers */
                constexpr int GS = MS_NWAVE * MS_G;
                /* a lane's arc of a chunk: the (col, w) pair (one packed word measured slower: the
                 * scalar split sits on the address chain, C3 26.4 vs 25.2 ms) */
                using arc_t = uint2;
                auto arc_at = [&](int k) -> arc_t { return icw[k]; };
                auto arc_none = []() -> arc_t { return make_uint2(0u, 0u); };
                int vl_n = 0;
                int2 bel_n = make_int2(0, 0);
                arc_t ea_n = arc_none();
                {
                    const int g1 = wave * MS_G;
                    if (g1 < cnt && lane < min(MS_G, cnt - g1)) {
                        vl_n = s_list[g1 + lane];
                        bel_n = irp[vl_n];
                    }
                    const int bx1 = __shfl(bel_n.x, aj), dg1 = __shfl(bel_n.y, aj) - bx1;
                    if (aa < dg1) ea_n = arc_at(bx1 + aa);
                }
                for (int g0 = wave * MS_G; g0 < cnt; g0 += GS) {
                    const int ng = min(MS_G, cnt - g0);
                    const int vl = vl_n;
                    const int2 bel = bel_n;
                    const arc_t ea0 = ea_n;
                    {
                        const int g1 = g0 + GS;
                        vl_n = 0;
                        bel_n = make_int2(0, 0);
                        if (g1 < cnt && lane < min(MS_G, cnt - g1)) {
                            vl_n = s_list[g1 + lane];
                            bel_n = irp[vl_n];
                        }
                    }
                    uint32_t v[MS_G], od[MS_G];
                    int bx[MS_G], dg[MS_G];
                    int maxdeg = 0;
#pragma unroll
                    for (int j = 0; j < MS_G; j++) {
                        v[j] = (uint32_t)__builtin_amdgcn_readlane(vl, j);
                        bx[j] = __builtin_amdgcn_readlane(bel.x, j);
                        dg[j] = j < ng ? __builtin_amdgcn_readlane(bel.y, j) - bx[j] : 0;
                        maxdeg = max(maxdeg, dg[j]);
                        od[j] = ms_ld(D + (size_t)v[j] * MS_L + lane);
                    }
                    const int abx = __shfl(bel.x, aj), adg = aj < ng ? __shfl(bel.y, aj) - abx : 0;
                    uint32_t bc[MS_G], bdu[MS_G], bu[MS_G];
                    int bk[MS_G];
#pragma unroll
                    for (int j = 0; j < MS_G; j++) {
                        bc[j] = DINF;
                        bdu[j] = DINF;
                        bu[j] = 0u;
                        bk[j] = -1;
                    }
                    /* the arc in slot j * MS_AC + h of the chunk: its column and weight, as
                     * wave-uniform values (one lane read, the split is scalar) */
                    auto arc_of = [&](const arc_t& e, int slot, uint32_t& col, uint32_t& w) {
                        col = (uint32_t)__builtin_amdgcn_readlane((int)e.x, slot);
                        w = (uint32_t)__builtin_amdgcn_readlane((int)e.y, slot);
                    };
                    arc_t ea = ea0;
                    for (int c0 = 0; c0 < maxdeg; c0 += MS_AC) {
                        if (c0 > 0) ea = aa + c0 < adg ? arc_at(abx + c0 + aa) : arc_none();
#pragma unroll
                        for (int h = 0; h < MS_AC; h += MS_AK) {
                            if (c0 + h >= maxdeg) break;
                            uint32_t du[MS_G][MS_AK];
#pragma unroll
                            for (int j = 0; j < MS_G; j++)
#pragma unroll
                                for (int a = 0; a < MS_AK; a++) {
                                    uint32_t col, w;
                                    arc_of(ea, j * MS_AC + h + a, col, w);
                                    du[j][a] = ms_ld(D + (size_t)col * MS_L + lane);
                                }
#pragma unroll
                            for (int j = 0; j < MS_G; j++)
#pragma unroll
                                for (int a = 0; a < MS_AK; a++) {
                                    const int k = c0 + h + a;
                                    if (k >= dg[j] || du[j][a] >= DINF) continue;
                                    uint32_t col, w;
                                    arc_of(ea, j * MS_AC + h + a, col, w);
                                    const uint32_t c =
                                        sizeof(DT) == 2 ? min(du[j][a] + w, DINF - 1u) : du[j][a] + w;
                                    if (c < bc[j] || (c == bc[j] && du[j][a] < bdu[j])) {
                                        bc[j] = c;
                                        bdu[j] = du[j][a];
                                        bk[j] = bx[j] + k;
                                        bu[j] = col;
                                    }
                                }
                        }
                    }
                    {   /* the next group's first arc chunk (its in-rows arrived meanwhile) */
                        const int bx1 = __shfl(bel_n.x, aj), dg1 = __shfl(bel_n.y, aj) - bx1;
                        ea_n = aa < dg1 ? arc_at(bx1 + aa) : arc_none();
                    }
                    uint32_t nd[MS_G];
                    double nr[MS_G], orl[MS_G];
#pragma unroll
                    for (int j = 0; j < MS_G; j++) {
                        /* the old reliability rides with the predecessor gathers */
                        orl[j] = ms_ld(R + (size_t)v[j] * MS_L + lane);
                        nd[j] = DINF;
                        nr[j] = 0.0;
                        if ((int)v[j] == mysrc) {
                            nd[j] = 0u;
                            nr[j] = 1.0;
                        } else if (bk[j] >= 0) {
                            nd[j] = bc[j];
                            nr[j] = ms_ld(R + (size_t)bu[j] * MS_L + lane) * ir[bk[j]];
                        }
                    }
#pragma unroll
                    for (int j = 0; j < MS_G; j++) {
                        if (j >= ng) break;
                        /* an unreached lane's R is not initialised: it reads as 0 */
                        const double ol = od[j] < DINF ? orl[j] : 0.0;
                        const bool ch = nd[j] != od[j] ||
                                        __double_as_longlong(nr[j]) != __double_as_longlong(ol);
                        if (!__ballot(ch)) continue;
                        const uint32_t vj = v[j];
                        D[(size_t)vj * MS_L + lane] = (DT)nd[j];
                        R[(size_t)vj * MS_L + lane] = nr[j];
                        const uint32_t mn = ms_wave_min(nd[j]);
                        if (lane == 0) mind[vj] = mn;
                        if (mn < T) {
                            if (lane == 0 && ms_bit(pend, vj))
                                atomicAnd(&pend[vj >> 5], ~(1u << (vj & 31)));
                            if (DIRECTED) {
                                const int2 ob = orp[vj];
                                for (int k = ob.x + lane; k < ob.y; k += MS_L) ms_set(nxt, ocw[k].x);
                            } else if (maxdeg <= MS_AC) { /* the arcs of the (only) chunk */
                                if (aj == j && aa < dg[j]) {
                                    ms_set(nxt, ea.x);
                                }
                            } else {
                                for (int k = bx[j] + lane; k < bx[j] + dg[j]; k += MS_L)
                                    ms_set(nxt, icw[k].x);
                            }
                        } else if (lane == 0) {
                            ms_set(pend, vj);
                        }
                    }
                }
                __syncthreads();
                if (!more) break;
            }
            if (found) {
                uint32_t* const t = cur;
                cur = nxt;
                nxt = t;
                continue;
            }
            /* no candidate left: advance T past the smallest pending lane minimum */
            if (tid == 0) s_pmin = SRT_INF;
            __syncthreads();
            uint32_t pm = SRT_INF;
            for (int wi = tid; wi < nw; wi += MS_WG) {
                const uint32_t word = pend[wi];
                if (!word) continue;
                /* every pending vertex's minimum loaded at once (predicated, unrolled) */
#pragma unroll
                for (int bt = 0; bt < 32; bt++)
                    if ((word >> bt) & 1u) pm = min(pm, ms_ld(mind + wi * 32 + bt));
            }
            pm = ms_wave_min(pm);
            if (lane == 0 && pm < SRT_INF) atomicMin(&s_pmin, pm);
            __syncthreads();
            const uint32_t pmin = s_pmin;
            if (pmin >= SRT_INF) break;
            T = (pmin / delta + 1u) * delta;
            /* pending vertices below T propagate now */
            for (int wi = tid; wi < nw; wi += MS_WG) {
                const uint32_t word = pend[wi];
                if (!word) continue;
                uint32_t mv[32];
#pragma unroll
                for (int bt = 0; bt < 32; bt++)
                    mv[bt] = (word >> bt) & 1u ? ms_ld(mind + wi * 32 + bt) : SRT_INF;
                uint32_t keep = word;
#pragma unroll
                for (int bt = 0; bt < 32; bt++) {
                    if (!((word >> bt) & 1u) || mv[bt] >= T) continue;
                    keep &= ~(1u << bt);
                    const int2 ob = orp[wi * 32 + bt];
                    for (int k = ob.x; k < ob.y; k++) ms_set(cur, ocw[k].x);
                }
                pend[wi] = keep;
            }
            __syncthreads();
        }
        /* output rows in original vertex order: lane j takes target t0 + j and reads its 64-lane
         * rows in 16-byte pieces (4 sources each); each source's row segment is one coalesced
         * store */
        const int32_t* br = brow + (size_t)b * MS_L;
        for (int t0 = wave * MS_L; t0 < n; t0 += MS_WG) {
            const int t = t0 + lane;
            const bool ok = t < n;
            const uint32_t v = ok ? (uint32_t)inv[t] : 0u;
            /* E lanes per 16-byte piece of the D row: 4 (u32) or 8 (u16) */
            constexpr int E = 16 / (int)sizeof(DT);
            const uint4* d4 = reinterpret_cast<const uint4*>(D + (size_t)v * MS_L);
            const double2* r2 = reinterpret_cast<const double2*>(R + (size_t)v * MS_L);
#pragma unroll 2
            for (int q = 0; q < MS_L / E; q++) {
                const uint4 dq = d4[q];
                const uint32_t w4[4] = {dq.x, dq.y, dq.z, dq.w};
                uint32_t dd[E];
                double rr[E];
#pragma unroll
                for (int i = 0; i < E; i++) {
                    dd[i] = sizeof(DT) == 2 ? (w4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu : w4[i];
                    if (dd[i] >= DINF) dd[i] = SRT_INF;
                }
#pragma unroll
                for (int i = 0; i < E; i += 2) {
                    const double2 x = r2[(q * E + i) >> 1];
                    rr[i] = x.x;
                    rr[i + 1] = x.y;
                }
#pragma unroll
                for (int i = 0; i < E; i++) {
                    const int row = br[q * E + i];
                    if (row < 0 || !ok) continue;
                    lat[(size_t)row * ldo + t] = dd[i];
                    rel[(size_t)row * ldo + t] = dd[i] < SRT_INF ? rr[i] : 0.0;
                }
            }
        }
        __syncthreads();
    }
}

/* LDS bytes of the kernel's three bitmaps for n vertices (dynamic part) */
static size_t ms_lds_bytes(int n) { return (size_t)3 * (size_t)((n + 31) >> 5) * sizeof(uint32_t); }

int srt_msssp_max_n(void) {
    /* three bitmaps beside the 8-KB list and the statics, within 160 KB */
    return (int)((((size_t)150 << 10) / 3 / 4) * 32);
}

/* Rows of the sources grouped in nbatch batches of 64 lanes (bsrc / brow: device arrays of
 * nbatch x 64 relabelled sources and output rows, -1 = empty lane); graph arrays as for the
 * kernel. Rows get the distances (u32 quanta, SRT_INF unreached) and the path-order reliability;
 * the diagonal is the caller's (srt_sparse_diag). */
/* the working rows stay allocated between builds (per device or virtual-rank slot): a fresh
 * multi-GB allocation per call costs milliseconds of mapping */
static uint32_t* g_ms_ws[SRT_STATE_SLOTS];
static size_t g_ms_cap[SRT_STATE_SLOTS];

int srt_msssp_rows(int n, int directed, const int2* orp, const uint2* ocw, const int2* irp,
                   const uint2* icw, const double* ir, const int32_t* inv,
                   uint32_t delta, int nbatch, const int32_t* bsrc, const int32_t* brow,
                   uint32_t* lat, double* rel, size_t ldo, int d16, hipStream_t st) {
    if (n > srt_msssp_max_n()) {
        srt_set_error("msssp: %d vertices exceed the LDS bitmaps (%d)", n, srt_msssp_max_n());
        return SRT_E_ARG;
    }
    if (nbatch <= 0) return SRT_OK;
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* D (u32-sized slots; a u16 row uses half), R and the lane minimum, rounded to 16 bytes */
    const size_t slot_words = ((size_t)n * MS_L * 3 + (size_t)n + 3) & ~(size_t)3;
    const size_t per_slot = slot_words * sizeof(uint32_t);
    const int fs = srt_form_int("ms_slots", 0); /* tests: one or a few persistent slots */
    size_t slots = fs > 0 ? (size_t)fs : 2 * (size_t)cus;
    if (slots > (size_t)nbatch) slots = nbatch;
    const int sl = srt_state_slot();
    if (g_ms_cap[sl] < slots * per_slot) {
        size_t budget = (size_t)16 << 30, free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > ((size_t)8 << 30)) {
            budget = free_b + g_ms_cap[sl] - ((size_t)8 << 30);
            if (budget > ((size_t)64 << 30)) budget = (size_t)64 << 30;
        }
        if (slots * per_slot > budget) slots = budget / per_slot;
        if (slots < 1) slots = 1;
        if (g_ms_ws[sl] && g_ms_cap[sl] < slots * per_slot) {
            SRT_HIPCHK(hipStreamSynchronize(st));
            SRT_HIPCHK(hipFree(g_ms_ws[sl]));
            g_ms_ws[sl] = NULL;
            g_ms_cap[sl] = 0;
        }
        if (!g_ms_ws[sl]) {
            if (hipMalloc((void**)&g_ms_ws[sl], slots * per_slot) != hipSuccess) {
                (void)hipGetLastError();
                g_ms_ws[sl] = NULL;
                srt_set_error("msssp: workspace of %zu MiB failed", (slots * per_slot) >> 20);
                return SRT_E_NOMEM;
            }
            g_ms_cap[sl] = slots * per_slot;
        }
    }
    if (slots * per_slot > g_ms_cap[sl]) slots = g_ms_cap[sl] / per_slot;
    uint32_t* ws = g_ms_ws[sl];
    const uint32_t dl = delta < 1 ? 1u : delta;
    const size_t dyn = ms_lds_bytes(n);
#define SRT_MSSSP_LAUNCH(DIR, DT)                                                                \
    do {                                                                                         \
        SRT_HIPCHK(hipFuncSetAttribute((const void*)msssp_kernel<DIR, DT>,                        \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));    \
        msssp_kernel<DIR, DT><<<(unsigned)slots, MS_WG, dyn, st>>>(                               \
            n, orp, ocw, irp, icw, ir, inv, nbatch, bsrc, brow, lat, rel, ldo, ws, slot_words,    \
            dl);                                                                                 \
    } while (0)
    if (directed && d16) SRT_MSSSP_LAUNCH(true, uint16_t);
    else if (directed) SRT_MSSSP_LAUNCH(true, uint32_t);
    else if (d16) SRT_MSSSP_LAUNCH(false, uint16_t);
    else SRT_MSSSP_LAUNCH(false, uint32_t);
#undef SRT_MSSSP_LAUNCH
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* rows computed elsewhere (the single-source kernels, for sources too scattered to share a batch)
 * copied to their output rows: row i of (tl, tr) to row rows[i] of (lat, rel) */
__global__ void ms_scatter_kernel(int n, const int32_t* __restrict__ rows,
                                  const uint32_t* __restrict__ tl, const double* __restrict__ tr,
                                  uint32_t* __restrict__ lat, double* __restrict__ rel, size_t ldo) {
    const int i = blockIdx.y;
    const size_t o = (size_t)rows[i] * ldo;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        lat[o + t] = tl[(size_t)i * n + t];
        rel[o + t] = tr[(size_t)i * n + t];
    }
}

int srt_ms_scatter_rows(int nr, int n, const int32_t* rows, const uint32_t* tl, const double* tr,
                        uint32_t* lat, double* rel, size_t ldo, hipStream_t st) {
    if (nr <= 0) return SRT_OK;
    const int bx = srt_ceil_div(n, 256) < 16 ? srt_ceil_div(n, 256) : 16;
    ms_scatter_kernel<<<dim3((unsigned)bx, (unsigned)nr), 256, 0, st>>>(n, rows, tl, tr, lat, rel, ldo);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}
