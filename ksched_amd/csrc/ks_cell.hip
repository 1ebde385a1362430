// ks_cell.hip — the whole ε-scaling push-relabel solve of a small graph inside
// one 1024-thread workgroup (ks_cell.h). Same algorithm as the
// multi-kernel engine (ks_engine.hip): phases ε ← ε/α, each
// starting by saturating every arc of negative reduced cost, then alternating a
// global price update (Bellman-Ford from the deficits over lengths
// floor(rc/ε)+1, prices p ← p − ε·min(d, L)) with bursts of push/relabel sweeps
// against a price snapshot; price refinement at ε = 1 certifies optimality.
// What changes is where it runs:
//
//   control   the phase loop, every decision and every termination test run on
//             the device; a step (one sweep, one Bellman-Ford round) ends at a
//             workgroup barrier — ~1 µs instead of a ~10 µs dependent launch.
//   LDS       the cell's prices (int64) and Bellman-Ford distances (int32,
//             saturating at 2^30: any cap keeps the triangle inequality the
//             update needs) live in LDS, 12 B per node, so the random gather of
//             a relaxation or an arc scan is an LDS read; only the 32-B
//             residual positions (streamed along each node's segment) and the
//             excess words come from L2.
//   frontier  per-class lists: a node enters the next frontier once, through a
//             test-and-set in an LDS bitmap, appended at its class's slice of a
//             list buffer in HBM; the next step takes lane groups of 4…64 lanes
//             per node (classes ≤ 64 positions), one wave per node (≤ 512) or
//             the whole workgroup (the cluster aggregator).
//   snapshot  sweeps read one price array and defer relabels to the end of the
//             sweep (a pending list applied after the barrier) — the snapshot
//             semantics of the engine's double-buffered prices (at
//             most one endpoint of a pair pushes in a sweep, so residuals are two
//             plain stores; the relabel minimum covers arcs a concurrent push may
//             make residual).
//
// Every loop is bounded (round and sweep caps, and a 100 MHz wall-clock limit
// read by one thread and broadcast through LDS), so a workgroup always exits.
#include "ks_cell.h"

namespace ks {
namespace {

constexpr int CT = CELL_THREADS;
constexpr int NW = CT / 64;
constexpr int DINF = 0x7fffffff;           // not reached by the update
constexpr long long DCAP = 1LL << 30;      // distances saturate here
constexpr long long DNEG = -(1LL << 30);   // price refinement below this: treated as a negative cycle
constexpr long long INF64 = 0x3fffffffffffffffLL;
constexpr size_t LDS_LIMIT = 163840;       // one workgroup may declare all 160 KiB on gfx950

enum { OP_SWEEP = 0, OP_BF = 1, OP_PR = 2, OP_SAT = 3 };
enum { F_INFEAS = 1, F_NEG = 2 };

struct St {
    int cnt[2][8];        // frontier list lengths per buffer and class
    int cbs[8];           // the cell's class bounds (dynamically indexed)
    int rl_cnt[2];        // pending relabels, by sweep parity
    int flag;             // F_INFEAS | F_NEG
    int stop;             // the wall-clock limit was hit
    long long red[NW];
};

// LDS: the static block and the dynamic region — prices (int64 × maxn), then
// distances (int32 × maxn), then two frontier bitmaps (W words each). Accessed
// by name (never through a pointer kept in a struct) so every access stays an
// LDS instruction.
__shared__ St s_;
extern __shared__ long long dyn_[];

// Per-workgroup scalars and per-thread counters. Global pointers are read from
// the kernel argument itself (A), which keeps them global-address-space loads.
struct K {
    int x0, N, W, maxn;
    int c1, c2, c3, c4, c5, c6;
    long long eps;
    int eps_shift;        // log2 ε when ε is a power of two (the cell ladder's are), else −1
    int sp;               // sweep parity (pending-relabel buffer)
};

// Work counters (ks_result units), counted per wave where the work happens: one
// ballot and, when any lane did work, one LDS add by lane 0 (the ballot must be
// taken at a point where the whole wave is converged).
enum { C_SCAN = 0, C_VISIT = 1, C_PUSH = 2, C_RELABEL = 3, C_GUSCAN = 4, NCTR = 5 };
__shared__ unsigned long long ctr_[NCTR];
__device__ __forceinline__ int lane();
__device__ __forceinline__ void wcount(int i, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m && lane() == 0) atomicAdd(&ctr_[i], (unsigned long long)__popcll(m));
}
// Thread-per-node work counts per thread, summed over the wave by DPP (no LDS
// round trips) and added to the workgroup's counters once per step.
struct Tc {
    unsigned c[NCTR] = {0, 0, 0, 0, 0};
};
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ unsigned dpp_add(unsigned v) {
    return v + (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {   // the sum lands in lane 63
    v = dpp_add<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xf>(v);   // row_half_mirror
    v = dpp_add<0x140, 0xf>(v);   // row_mirror
    v = dpp_add<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
    v = dpp_add<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3
    return v;
}
__device__ __forceinline__ void flush(const Tc& t) {
#pragma unroll
    for (int i = 0; i < NCTR; ++i) {
        const unsigned w = wave_sum_u32(t.c[i]);
        if (lane() == 63 && w) atomicAdd(&ctr_[i], (unsigned long long)w);
    }
}

__device__ __forceinline__ long long* prc() { return dyn_; }
__device__ __forceinline__ int* dst(const K& k) { return reinterpret_cast<int*>(dyn_ + k.maxn); }
__device__ __forceinline__ unsigned* bmp(const K& k) {
    return reinterpret_cast<unsigned*>(dyn_ + k.maxn + (k.maxn + 1) / 2);
}

// The lane id comes from volatile asm: recomputed where used, never hoisted out
// of the kernel's operation loop (hoisted lane-index and lane-mask values of
// every inlined shuffle otherwise stay live across the whole solve and spill).
__device__ __forceinline__ int lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ __forceinline__ int wid() { return (int)(threadIdx.x >> 6); }
__device__ __forceinline__ size_t ni(long long x) { return 4 * (size_t)x; }

__device__ __forceinline__ long long ld_ex(const CellArgs& A, int v) {
    return __hip_atomic_load(&A.excess[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void add_ex(const CellArgs& A, int v, long long d) {
    __hip_atomic_fetch_add(&A.excess[v], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ Pos ld_pos(const Pos* p) {
    const longlong2 a = reinterpret_cast<const longlong2*>(p)[0];   // cost, rcap
    const longlong2 b = reinterpret_cast<const longlong2*>(p)[1];   // ucap, head | rev << 32
    Pos r;
    r.cost = a.x;
    r.rcap = a.y;
    r.ucap = b.x;
    r.head = (int)(unsigned)((unsigned long long)b.y & 0xffffffffULL);
    r.rev = (int)(unsigned)((unsigned long long)b.y >> 32);
    return r;
}
__device__ __forceinline__ void seg(const CellArgs& A, int x, int& b0, int& b1) {
    const unsigned long long w = (unsigned long long)A.nd[ni(x) + 3];
    b0 = (int)(unsigned)(w & 0xffffffffULL);
    b1 = (int)(unsigned)(w >> 32);
}
__device__ __forceinline__ long long floordiv(long long a, long long b) {   // b > 0
    long long q = a / b;
    if ((a % b) != 0 && a < 0) --q;
    return q;
}

// 64-bit lane exchange by byte index (ds_bpermute: a lane outside the wave wraps,
// callers ignore those values)
__device__ __forceinline__ long long bperm64(int idx, long long x) {
    const int lo = __builtin_amdgcn_ds_bpermute(idx << 2, (int)(unsigned long long)x);
    const int hi = __builtin_amdgcn_ds_bpermute(idx << 2, (int)((unsigned long long)x >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// Lane-group (G lanes, aligned) collectives: xor partners o < G stay in the group.
template <int G>
__device__ __forceinline__ long long g_incl_scan(long long x) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        const int ln = lane();
        const long long y = bperm64(ln - o, x);
        if ((ln & (G - 1)) >= o) x += y;
    }
    return x;
}
template <int G>
__device__ __forceinline__ long long g_last(long long x) {   // the group's last lane's value
    return bperm64(lane() | (G - 1), x);
}
template <int G>
__device__ __forceinline__ long long g_min(long long x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x = min(x, bperm64(lane() ^ o, x));
    return x;
}
template <int G>
__device__ __forceinline__ long long g_sum(long long x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += bperm64(lane() ^ o, x);
    return x;
}
template <int G>
__device__ __forceinline__ long long g_max(long long x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x = max(x, bperm64(lane() ^ o, x));
    return x;
}

// ------------------------------------------------------- block collectives ---
// Each starts with a barrier (the previous user of red[] has read it) and ends
// with the value in every thread.
__device__ __forceinline__ long long blk_sum(long long x) {
    x = g_sum<64>(x);
    __syncthreads();
    if (lane() == 0) s_.red[wid()] = x;
    __syncthreads();
    long long t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += s_.red[i];
    return t;
}
__device__ __forceinline__ long long blk_max(long long x) {
    x = g_max<64>(x);
    __syncthreads();
    if (lane() == 0) s_.red[wid()] = x;
    __syncthreads();
    long long t = s_.red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = max(t, s_.red[i]);
    return t;
}
__device__ __forceinline__ long long blk_min(long long x) {
    x = g_min<64>(x);
    __syncthreads();
    if (lane() == 0) s_.red[wid()] = x;
    __syncthreads();
    long long t = s_.red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = min(t, s_.red[i]);
    return t;
}
// exclusive prefix over the workgroup; *total = the workgroup's sum
__device__ __forceinline__ long long blk_excl_scan(long long x, long long* total) {
    const long long incl = g_incl_scan<64>(x);
    __syncthreads();
    if (lane() == 63) s_.red[wid()] = incl;
    __syncthreads();
    long long off = 0, tot = 0;
    const int w = wid();
    for (int i = 0; i < w; ++i) off += s_.red[i];
#pragma unroll
    for (int i = 0; i < NW; ++i) tot += s_.red[i];
    *total = tot;
    return off + incl - x;
}

// ------------------------------------------------------------- frontiers ---
__device__ __forceinline__ int cls_of(const K& k, int x) {
    return (x >= k.c1) + (x >= k.c2) + (x >= k.c3) + (x >= k.c4) + (x >= k.c5) + (x >= k.c6);
}
// x joins frontier buffer nb once (LDS bitmap test-and-set), at its class's slice.
__device__ __forceinline__ void mark(const CellArgs& A, const K& k, int nb, int x) {
    const int l = x - k.x0;
    const unsigned bit = 1u << (l & 31);
    if (atomicOr(&bmp(k)[nb * k.W + (l >> 5)], bit) & bit) return;
    const int c = cls_of(k, x);
    const int i = atomicAdd(&s_.cnt[nb][c], 1);
    A.lists[(size_t)nb * A.nn + s_.cbs[c] + i] = x;
}
// src 0 / 1: a frontier buffer; 2: every node of the cell (dense pass)
__device__ __forceinline__ int count_of(int src, int c) {
    return src == 2 ? s_.cbs[c + 1] - s_.cbs[c] : s_.cnt[src][c];
}
__device__ __forceinline__ int node_at(const CellArgs& A, int src, int c, int j) {
    return src == 2 ? s_.cbs[c] + j : A.lists[(size_t)src * A.nn + s_.cbs[c] + j];
}
__device__ __forceinline__ int total_of(int b) {
    int t = 0;
#pragma unroll
    for (int c = 0; c < CELL_NCLS; ++c) t += s_.cnt[b][c];
    return t;
}
// empty both buffers (callers put a barrier after it)
__device__ __forceinline__ void reset_lists(const K& k) {
    if (threadIdx.x < 16) (&s_.cnt[0][0])[threadIdx.x] = 0;
    unsigned* bm = bmp(k);
    for (int w = threadIdx.x; w < 2 * k.W; w += CT) bm[w] = 0;
}

// ------------------------------------------------------------ push/relabel ---
__device__ __forceinline__ void push(const CellArgs& A, const K& k, int nb, int a, int w, long long r, long long d,
                                     int rv, long long uc) {
    A.pos[a].rcap = r - d;
    A.pos[rv].rcap = uc - (r - d);
    add_ex(A, w, d);
    mark(A, k, nb, w);
}
// the relabel of v takes effect after the sweep (price snapshot)
__device__ __forceinline__ void relabel(const CellArgs& A, const K& k, int v, long long np) {
    const int i = atomicAdd(&s_.rl_cnt[k.sp], 1);
    A.rl_node[k.x0 + i] = v;
    A.rl_p[k.x0 + i] = np;
}

// One node per G-lane group (G = 64 loops over 64-position chunks): the excess
// is spread over the admissible arcs by an in-group prefix sum; a node that
// saturates all of them relabels to p − (minc + ε), minc over residual arcs and
// over arcs of reduced cost in (0, ε] (ks_engine.hip sweep_group).
template <int G>
__device__ __forceinline__ void sweep_grp(const CellArgs& A, K& k, int nb, int v) {
    const long long* P = prc();
    const int lig = lane() & (G - 1);
    long long e = 0, pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        e = ld_ex(A, v);
        pv = P[v - k.x0];
        seg(A, v, b0, en);
    }
    const bool act = e > 0;
    if (!act) en = b0;
    wcount(C_VISIT, act && lig == 0);
    long long rem = e, minc = INF64;
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        const bool valid = a < en;
        long long r = 0, cr = 0, uc = 0;
        int w = 0, rv = 0;
        if (valid) {
            const Pos q = ld_pos(A.pos + a);
            r = q.rcap;
            w = q.head;
            rv = q.rev;
            uc = q.ucap;
            cr = q.cost + pv - P[w - k.x0];
        }
        wcount(C_SCAN, valid);
        const long long adm = (valid && cr < 0 && r > 0) ? r : 0;
        const long long incl = g_incl_scan<G>(adm);
        const long long total = g_last<G>(incl);
        long long d = rem - (incl - adm);
        d = d < 0 ? 0 : (d > adm ? adm : d);
        if (d > 0) push(A, k, nb, a, w, r, d, rv, uc);
        wcount(C_PUSH, d > 0);
        if (valid) {
            if (cr < 0) {
                if (r - d > 0) minc = min(minc, cr);
            } else if (r > 0 || cr <= k.eps) {
                minc = min(minc, cr);
            }
        }
        rem -= total < rem ? total : rem;
        if (G == 64 && rem == 0) break;
    }
    minc = g_min<G>(minc);
    wcount(C_RELABEL, act && lig == 0 && rem > 0);
    if (act && lig == 0) {
        const long long pushed = e - rem;
        if (pushed) add_ex(A, v, -pushed);
        if (rem > 0) {
            if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
            else relabel(A, k, v, pv - (minc + k.eps));
            mark(A, k, nb, v);
        }
    }
}

// The same for a node above 512 positions: the whole workgroup, 1024 positions
// per pass, the excess spread by a workgroup-wide prefix sum. v is uniform.
__device__ __forceinline__ void sweep_hub(const CellArgs& A, K& k, int nb, int v) {
    const long long* P = prc();
    const long long e = ld_ex(A, v);
    const long long pv = P[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    if (e <= 0) return;
    wcount(C_VISIT, threadIdx.x == 0);
    long long rem = e, minc = INF64;
    for (int base = b0; base < en; base += CT) {
        const int a = base + (int)threadIdx.x;
        const bool valid = a < en;
        long long r = 0, cr = 0, uc = 0;
        int w = 0, rv = 0;
        if (valid) {
            const Pos q = ld_pos(A.pos + a);
            r = q.rcap;
            w = q.head;
            rv = q.rev;
            uc = q.ucap;
            cr = q.cost + pv - P[w - k.x0];
        }
        wcount(C_SCAN, valid);
        const long long adm = (valid && cr < 0 && r > 0) ? r : 0;
        long long tot;
        const long long excl = blk_excl_scan(adm, &tot);
        long long d = rem - excl;
        d = d < 0 ? 0 : (d > adm ? adm : d);
        if (d > 0) push(A, k, nb, a, w, r, d, rv, uc);
        wcount(C_PUSH, d > 0);
        if (valid) {
            if (cr < 0) {
                if (r - d > 0) minc = min(minc, cr);
            } else if (r > 0 || cr <= k.eps) {
                minc = min(minc, cr);
            }
        }
        rem -= tot < rem ? tot : rem;
        if (rem == 0) break;
    }
    minc = blk_min(minc);
    wcount(C_RELABEL, threadIdx.x == 0 && rem > 0);
    if (threadIdx.x == 0) {
        const long long pushed = e - rem;
        if (pushed) add_ex(A, v, -pushed);
        if (rem > 0) {
            if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
            else relabel(A, k, v, pv - (minc + k.eps));
            mark(A, k, nb, v);
        }
    }
}

// ---------------------------------------------------------- Bellman-Ford ---
// In-arc (u → v) = the reverse of v's position a; its residual is ucap − rcap
// and its reduced cost −(cost(a) + p(v) − p(u)). PR: price refinement (ε = 1,
// negative lengths allowed, no clamp at 0).
template <bool PR>
__device__ __forceinline__ void relax(const CellArgs& A, const K& k, int nb, int a, int dv, long long pv) {
    const Pos q = ld_pos(A.pos + a);
    if (q.ucap - q.rcap <= 0) return;
    const int lu = q.head - k.x0;
    const long long pu = prc()[lu];
    int* D = dst(k);
    const long long x = pu - q.cost - pv;
    long long len = PR ? x + 1 : (k.eps_shift >= 0 ? (x >> k.eps_shift) : floordiv(x, k.eps)) + 1;
    if (!PR) len = len < 0 ? 0 : (len > DCAP ? DCAP : len);
    else len = len > DCAP ? DCAP : (len < DNEG ? DNEG : len);
    long long cand = (long long)dv + len;
    if (cand > DCAP) cand = DCAP;
    if (PR && cand < DNEG) {
        cand = DNEG;
        atomicOr(&s_.flag, F_NEG);
    }
    if (cand < (long long)D[lu]) {
        const int old = atomicMin(&D[lu], (int)cand);
        if (cand < (long long)old) mark(A, k, nb, q.head);
    }
}

template <int G, bool PR>
__device__ __forceinline__ void bf_grp(const CellArgs& A, K& k, int nb, int v) {
    const int lig = lane() & (G - 1);
    int dv = DINF;
    long long pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        dv = dst(k)[v - k.x0];
        pv = prc()[v - k.x0];
        seg(A, v, b0, en);
    }
    if (!PR && dv >= DINF) en = b0;
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        if (a < en) relax<PR>(A, k, nb, a, dv, pv);
        wcount(C_GUSCAN, a < en);
    }
}

template <bool PR>
__device__ __forceinline__ void bf_hub(const CellArgs& A, K& k, int nb, int v) {
    const int dv = dst(k)[v - k.x0];
    const long long pv = prc()[v - k.x0];
    if (!PR && dv >= DINF) return;
    int b0, en;
    seg(A, v, b0, en);
    for (int base = b0; base < en; base += CT) {   // (a uniform trip count: the ballot needs the whole wave)
        const int a = base + (int)threadIdx.x;
        if (a < en) relax<PR>(A, k, nb, a, dv, pv);
        wcount(C_GUSCAN, a < en);
    }
}

// -------------------------------------------------------------- saturate ---
// Goldberg's refine start: every residual arc of reduced cost below −thr is
// saturated (thr = ε after a failed refinement or on a warm start).
template <int G>
__device__ __forceinline__ void sat_grp(const CellArgs& A, K& k, int v, long long thr) {
    const long long* P = prc();
    const int lig = lane() & (G - 1);
    long long pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        pv = P[v - k.x0];
        seg(A, v, b0, en);
    }
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;
    long long tot = 0;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        bool pushed = false;
        if (a < en) {
            const Pos q = ld_pos(A.pos + a);
            if (q.rcap > 0 && q.cost + pv - P[q.head - k.x0] < -thr) {
                A.pos[a].rcap = 0;
                A.pos[q.rev].rcap = q.ucap;
                add_ex(A, q.head, q.rcap);
                tot += q.rcap;
                pushed = true;
            }
        }
        wcount(C_PUSH, pushed);
    }
    tot = g_sum<G>(tot);
    if (v >= 0 && lig == 0 && tot) add_ex(A, v, -tot);
}

__device__ __forceinline__ void sat_hub(const CellArgs& A, K& k, int v, long long thr) {
    const long long* P = prc();
    const long long pv = P[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    long long tot = 0;
    for (int base = b0; base < en; base += CT) {
        const int a = base + (int)threadIdx.x;
        bool pushed = false;
        if (a < en) {
            const Pos q = ld_pos(A.pos + a);
            if (q.rcap > 0 && q.cost + pv - P[q.head - k.x0] < -thr) {
                A.pos[a].rcap = 0;
                A.pos[q.rev].rcap = q.ucap;
                add_ex(A, q.head, q.rcap);
                tot += q.rcap;
                pushed = true;
            }
        }
        wcount(C_PUSH, pushed);
    }
    tot = blk_sum(tot);
    if (threadIdx.x == 0 && tot) add_ex(A, v, -tot);
}

// ------------------------------------------------ one thread per node ---
// Classes of ≤ 32 positions (tasks, PUs, machines): a node per thread, its
// positions loaded CH at a time (independent loads in flight), the excess spread
// along them in order — the same distribution as the lane-group prefix sum, with
// no cross-lane exchange, and 64 nodes per wave instead of 64/G.
constexpr int CH = 4;

__device__ __forceinline__ void sweep_thr(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const long long* P = prc();
    long long e = 0, pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        e = ld_ex(A, v);
        pv = P[v - k.x0];
        seg(A, v, b0, en);
    }
    if (e <= 0) return;
    ++t.c[C_VISIT];
    long long rem = e, minc = INF64;
    for (int a0 = b0; a0 < en; a0 += CH) {
        Pos q[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (a0 + u < en) q[u] = ld_pos(A.pos + a0 + u);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            if (a0 + u >= en) break;
            ++t.c[C_SCAN];
            const long long r = q[u].rcap;
            const long long cr = q[u].cost + pv - P[q[u].head - k.x0];
            long long d = 0;
            if (cr < 0 && r > 0) {
                d = rem < r ? rem : r;
                if (d > 0) {
                    push(A, k, nb, a0 + u, q[u].head, r, d, q[u].rev, q[u].ucap);
                    ++t.c[C_PUSH];
                    rem -= d;
                }
                if (r - d > 0) minc = min(minc, cr);
            } else if (r > 0 || cr <= k.eps) {
                minc = min(minc, cr);
            }
        }
        if (rem == 0) break;
    }
    const long long pushed = e - rem;
    if (pushed) add_ex(A, v, -pushed);
    if (rem > 0) {
        if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
        else relabel(A, k, v, pv - (minc + k.eps));
        ++t.c[C_RELABEL];
        mark(A, k, nb, v);
    }
}

template <bool PR>
__device__ __forceinline__ void bf_thr(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    int dv = DINF;
    long long pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        dv = dst(k)[v - k.x0];
        pv = prc()[v - k.x0];
        seg(A, v, b0, en);
    }
    if (!PR && dv >= DINF) return;
    for (int a0 = b0; a0 < en; a0 += CH) {
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (a0 + u < en) {
                relax<PR>(A, k, nb, a0 + u, dv, pv);
                ++t.c[C_GUSCAN];
            }
    }
}

__device__ __forceinline__ void sat_thr(const CellArgs& A, K& k, int v, long long thr, Tc& t) {
    const long long* P = prc();
    long long pv = 0;
    int b0 = 0, en = 0;
    if (v >= 0) {
        pv = P[v - k.x0];
        seg(A, v, b0, en);
    }
    long long tot = 0;
    for (int a0 = b0; a0 < en; a0 += CH) {
        Pos q[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (a0 + u < en) q[u] = ld_pos(A.pos + a0 + u);
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (a0 + u < en && q[u].rcap > 0 && q[u].cost + pv - P[q[u].head - k.x0] < -thr) {
                A.pos[a0 + u].rcap = 0;
                A.pos[q[u].rev].rcap = q[u].ucap;
                add_ex(A, q[u].head, q[u].rcap);
                tot += q[u].rcap;
                ++t.c[C_PUSH];
            }
    }
    if (tot) add_ex(A, v, -tot);
}

// ------------------------------------------------------------------ step ---
// An item: 64 nodes of a class ≤ 32 positions (one per thread), or one node of
// the ≤ 64 / ≤ 512-position classes (the wave).
template <int OP, int C>
__device__ __forceinline__ void item(const CellArgs& A, K& k, int src, int nb, int j, int n, long long thr, Tc& t) {
    if (C < 4) {
        const int idx = j * 64 + lane();
        const int v = idx < n ? node_at(A, src, C, idx) : -1;
        if (OP == OP_SWEEP) sweep_thr(A, k, nb, v, t);
        else if (OP == OP_BF) bf_thr<false>(A, k, nb, v, t);
        else if (OP == OP_PR) bf_thr<true>(A, k, nb, v, t);
        else sat_thr(A, k, v, thr, t);
        return;
    }
    const int v = __builtin_amdgcn_readfirstlane(node_at(A, src, C, j));
    if (OP == OP_SWEEP) sweep_grp<64>(A, k, nb, v);
    else if (OP == OP_BF) bf_grp<64, false>(A, k, nb, v);
    else if (OP == OP_PR) bf_grp<64, true>(A, k, nb, v);
    else sat_grp<64>(A, k, v, thr);
}

// One step over frontier src (2: every node) into buffer nb: the workgroup-
// sized nodes one after another with every thread, then the rest as items
// (a batch of 64/G nodes of one class, or one ≤ 512-position node) dealt to the
// 16 waves. The caller's barrier completes buffer nb; step_post then empties src.
template <int OP>
__device__ __forceinline__ void step(const CellArgs& A, K& k, int src, int nb, long long thr) {
    const int n6 = count_of(src, 6);
    for (int j = 0; j < n6; ++j) {
        const int v = node_at(A, src, 6, j);
        __syncthreads();   // the previous node's pushes and marks are in
        if (OP == OP_SWEEP) sweep_hub(A, k, nb, v);
        else if (OP == OP_BF) bf_hub<false>(A, k, nb, v);
        else if (OP == OP_PR) bf_hub<true>(A, k, nb, v);
        else sat_hub(A, k, v, thr);
    }
    const int n0 = count_of(src, 0), n1 = count_of(src, 1), n2 = count_of(src, 2), n3 = count_of(src, 3),
              n4 = count_of(src, 4), n5 = count_of(src, 5);
    const int e0 = (n0 + 63) >> 6;
    const int e1 = e0 + ((n1 + 63) >> 6);
    const int e2 = e1 + ((n2 + 63) >> 6);
    const int e3 = e2 + ((n3 + 63) >> 6);
    const int e4 = e3 + n4;
    const int e5 = e4 + n5;
    Tc t;
    for (int it = wid(); it < e5; it += NW) {
        if (it < e0) item<OP, 0>(A, k, src, nb, it, n0, thr, t);
        else if (it < e1) item<OP, 1>(A, k, src, nb, it - e0, n1, thr, t);
        else if (it < e2) item<OP, 2>(A, k, src, nb, it - e1, n2, thr, t);
        else if (it < e3) item<OP, 3>(A, k, src, nb, it - e2, n3, thr, t);
        else if (it < e4) item<OP, 4>(A, k, src, nb, it - e3, n4, thr, t);
        else item<OP, 5>(A, k, src, nb, it - e4, n5, thr, t);
    }
    flush(t);
}

// After a step's barrier: src emptied; a sweep's relabels take effect; the
// pending-relabel counter of the NEXT sweep's parity is reset (it was last read
// before the previous barrier).
template <int OP>
__device__ __forceinline__ void step_post(const CellArgs& A, const K& k, int src) {
    if (src < 2) {
        if (threadIdx.x < 8) s_.cnt[src][threadIdx.x] = 0;
        unsigned* bm = bmp(k);
        for (int w = threadIdx.x; w < k.W; w += CT) bm[src * k.W + w] = 0;
    }
    if (OP == OP_SWEEP) {
        long long* P = prc();
        const int nr = s_.rl_cnt[k.sp];
        for (int i = threadIdx.x; i < nr; i += CT) P[A.rl_node[k.x0 + i] - k.x0] = A.rl_p[k.x0 + i];
        if (threadIdx.x == 0) s_.rl_cnt[k.sp ^ 1] = 0;
    }
}

// ---------------------------------------------------------- control ---
// The solve is a state machine: thread 0 decides the next operation from the
// control block in LDS (the phase loop of ks_engine.hip Engine::solve, run on
// the device), and the whole workgroup executes one operation per iteration of
// the kernel's loop. Every operation starts and ends at a barrier, so no
// register state lives across operations.
enum Op { O_SAT, O_GUINIT, O_BF, O_GUFIN, O_SWEEP, O_PRINIT, O_PR, O_PRFIN, O_DONE };
enum Next { N_PHASE_LOOP = 0, N_RECOVERY = 1 };

struct Ctl {
    int op, src, nb, sp;
    long long thr;            // saturation threshold of the running phase
    long long eps;            // ε the current operation uses
    long long eps_ph;         // ε of the running phase
    unsigned long long t0;
    int phases, pr_failed, early, status;
    int peak, cyc_sweeps, upd_rounds, pr_rounds, pr_cap, pr_ok_now, pr_next, nexc;
    int updates, pr_ok, pr_tries, ended_at_one;
    unsigned long long phase_sweeps, sweeps, rounds;
    unsigned long long t_op;                // when the running operation started
    unsigned long long op_ticks[O_DONE];    // 100 MHz ticks per operation kind (incl. its barriers)
    unsigned op_n[O_DONE];
};
__shared__ Ctl c_;

__device__ __forceinline__ int total_any(int src) { return total_of(src); }

// thread 0 only: a phase of ε = eps_ph begins (DESIGN §3 ε schedule)
__device__ __forceinline__ void begin_phase(const CellArgs& A) {
    Ctl& c = c_;
    ++c.phases;
    c.thr = (c.phases == 1 && A.warm) ? A.sat_thr0 : (c.pr_failed ? c.eps_ph : 0LL);
    c.pr_failed = 0;
    const bool last = c.eps_ph / A.alpha < 1 || c.eps_ph <= 1 || (A.use_pr && c.eps_ph * A.pr_div < A.mult);
    c.early = last ? 0 : 1;
    c.eps = c.eps_ph;
    c.peak = 0;
    c.phase_sweeps = 0;
    c.op = O_SAT;
    c.src = 2;
    c.nb = 0;
}
__device__ __forceinline__ void finish(int status) {
    c_.status = status;
    c_.op = O_DONE;
}
// after a phase: price refinement where it may certify, then the next phase
__device__ __forceinline__ void phase_end(const CellArgs& A) {
    Ctl& c = c_;
    if (A.use_pr && c.eps_ph > 1 && c.eps_ph * A.pr_div < A.mult) {
        c.op = O_PRINIT;
        c.pr_cap = A.pr_cap;
        c.pr_next = N_PHASE_LOOP;
        return;
    }
    if (c.eps_ph > 1) {
        c.eps_ph = c.eps_ph / A.alpha > 1 ? c.eps_ph / A.alpha : 1;
        begin_phase(A);
    } else {
        c.ended_at_one = 1;
        finish(CS_OK);
    }
}

__device__ __forceinline__ void control(const CellArgs& A, int N) {
    Ctl& c = c_;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    c.op_ticks[c.op] += now - c.t_op;
    ++c.op_n[c.op];
    c.t_op = now;
    if (now - c.t0 > A.timeout_ticks) return finish(CS_TIMEOUT);
    switch (c.op) {
        case O_SAT:
            c.op = O_GUINIT;
            return;
        case O_GUINIT:
            c.upd_rounds = 0;
            c.src = 0;
            c.nb = 1;
            c.op = total_any(0) ? O_BF : O_GUFIN;
            return;
        case O_BF:
            ++c.upd_rounds;
            ++c.rounds;
            c.src = c.nb;
            c.nb ^= 1;
            if (!total_any(c.src)) c.op = O_GUFIN;
            else if (c.upd_rounds > 4 * N + 64) finish(CS_NOCONV);
            return;
        case O_GUFIN: {
            ++c.updates;
            if (s_.flag & F_INFEAS) return finish(CS_INFEASIBLE);
            const int n = c.nexc;
            if (n == 0) return phase_end(A);
            c.peak = max(c.peak, n);
            if (c.early && n <= A.phase_exit && (long long)n * A.phase_frac <= c.peak) return phase_end(A);
            c.cyc_sweeps = 0;
            c.src = 0;
            c.nb = 1;
            c.op = O_SWEEP;
            return;
        }
        case O_SWEEP:
            ++c.sweeps;
            ++c.phase_sweeps;
            ++c.cyc_sweeps;
            c.sp ^= 1;
            c.src = c.nb;
            c.nb ^= 1;
            if (s_.flag & F_INFEAS) return finish(CS_INFEASIBLE);
            if (!total_any(c.src)) return phase_end(A);   // no node holds excess
            if (c.phase_sweeps > 64ULL * ((unsigned long long)N + 64)) return finish(CS_NOCONV);
            if (c.cyc_sweeps >= A.gi) c.op = O_GUINIT;
            return;
        case O_PRINIT:
            ++c.pr_tries;
            c.eps = 1;
            c.pr_rounds = 0;
            c.src = 2;
            c.nb = 0;
            c.op = O_PR;
            return;
        case O_PR:
            ++c.rounds;
            ++c.pr_rounds;
            if (s_.flag & F_NEG) c.pr_ok_now = 0;
            else if (!total_any(c.nb)) c.pr_ok_now = 1;
            else if (c.pr_rounds >= c.pr_cap) c.pr_ok_now = 0;
            else {
                c.src = c.nb;
                c.nb ^= 1;
                return;
            }
            c.op = O_PRFIN;
            return;
        case O_PRFIN:
            c.eps = c.eps_ph;
            if (c.pr_ok_now) ++c.pr_ok;
            if (c.pr_next == N_RECOVERY) {
                if (c.pr_ok_now) {
                    c.ended_at_one = 1;
                    return finish(CS_OK);
                }
                // one more ε = 1 phase from the flow in place, saturating only the
                // arcs that violate 1-optimality
                c.eps_ph = 1;
                ++c.phases;
                c.thr = 1;
                c.early = 0;
                c.eps = 1;
                c.peak = 0;
                c.phase_sweeps = 0;
                c.pr_next = N_PHASE_LOOP;
                c.op = O_SAT;
                c.src = 2;
                c.nb = 0;
                return;
            }
            if (c.pr_ok_now) {
                c.ended_at_one = 1;
                return finish(CS_OK);
            }
            c.pr_failed = 1;
            if (c.eps_ph > 1) {
                c.eps_ph = c.eps_ph / A.alpha > 1 ? c.eps_ph / A.alpha : 1;
                begin_phase(A);
            } else {
                c.ended_at_one = 1;
                finish(CS_OK);
            }
            return;
        default:
            return;
    }
}

// ------------------------------------------------------------ operations ---
// dense: D = 0 at deficits, unreached elsewhere; the deficits are buffer 0
__device__ __forceinline__ void gu_init(const CellArgs& A, const K& k) {
    int* D = dst(k);
    for (int l = threadIdx.x; l < k.N; l += CT) {
        const int x = k.x0 + l;
        const long long e = ld_ex(A, x);
        D[l] = e < 0 ? 0 : DINF;
        if (e < 0) mark(A, k, 0, x);
    }
}
// L = the largest finite distance; p ← p − ε·min(d, L); the excess nodes are
// buffer 0 (an excess node the update did not reach: infeasible)
__device__ __forceinline__ void gu_fin(const CellArgs& A, const K& k) {
    int* D = dst(k);
    long long* P = prc();
    long long L = 0;
    for (int l = threadIdx.x; l < k.N; l += CT)
        if (D[l] < DINF) L = max(L, (long long)D[l]);
    L = blk_max(L);
    const long long lim = (1LL << 60) / k.eps;
    if (L > lim) L = lim;
    int nexc = 0;
    for (int l = threadIdx.x; l < k.N; l += CT) {
        const int x = k.x0 + l;
        const long long d = D[l];
        const long long e = ld_ex(A, x);
        P[l] -= k.eps * (d < L ? d : L);
        if (e > 0) {
            if (d >= DINF) atomicOr(&s_.flag, F_INFEAS);
            mark(A, k, 0, x);
            ++nexc;
        }
    }
    const int n = (int)blk_sum(nexc);
    if (threadIdx.x == 0) c_.nexc = n;
}

__global__ __launch_bounds__(CT) void k_cell(CellArgs A) {
    const CellDesc cd = A.cells[blockIdx.x];
    const int N = cd.cb[CELL_NCLS] - cd.cb[0];
    if (threadIdx.x < 8) s_.cbs[threadIdx.x] = A.cells[blockIdx.x].cb[threadIdx.x];
    if (threadIdx.x < NCTR) ctr_[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        s_.rl_cnt[0] = s_.rl_cnt[1] = 0;
        s_.flag = 0;
        s_.stop = 0;
        Ctl& c = c_;
        c = Ctl{};
        c.t0 = __builtin_amdgcn_s_memrealtime();
        c.t_op = c.t0;
        c.eps_ph = A.eps_start;
        c.eps = 1;
        if (N == 0) {
            c.ended_at_one = 1;
            finish(CS_OK);
        } else if (A.mode == 0) {
            c.eps_ph = A.eps_start / A.alpha > 1 ? A.eps_start / A.alpha : 1;
            begin_phase(A);
        } else {   // certificate recovery: refinement at ε = 1 first
            c.eps_ph = 1;
            c.op = O_PRINIT;
            c.pr_cap = 4 * A.pr_cap;
            c.pr_next = N_RECOVERY;
        }
    }
    {
        K k;
        k.x0 = cd.cb[0];
        k.N = N;
        k.maxn = A.max_nodes;
        k.W = (N + 31) / 32;
        reset_lists(k);
        long long* P = prc();
        int* D = dst(k);
        for (int l = threadIdx.x; l < N; l += CT) {
            P[l] = A.nd[ni(k.x0 + l)];
            D[l] = DINF;
        }
    }
    __syncthreads();
    // one operation per iteration: its body, a barrier, the post-work of steps
    // with the controller's decision (thread 0), a barrier
    for (;;) {
        const int op = c_.op;
        if (op == O_DONE) break;
        K k;
        k.x0 = cd.cb[0];
        k.N = N;
        k.maxn = A.max_nodes;
        k.W = (N + 31) / 32;
        k.c1 = cd.cb[1];
        k.c2 = cd.cb[2];
        k.c3 = cd.cb[3];
        k.c4 = cd.cb[4];
        k.c5 = cd.cb[5];
        k.c6 = cd.cb[6];
        k.eps = c_.eps;
        k.eps_shift = (k.eps & (k.eps - 1)) == 0 ? __builtin_ctzll((unsigned long long)k.eps) : -1;
        k.sp = c_.sp;
        const int src = c_.src, nb = c_.nb;
        switch (op) {
            case O_SAT:
                step<OP_SAT>(A, k, 2, 0, c_.thr);
                break;
            case O_GUINIT:
                reset_lists(k);
                __syncthreads();
                gu_init(A, k);
                break;
            case O_BF:
                step<OP_BF>(A, k, src, nb, 0);
                break;
            case O_GUFIN:
                reset_lists(k);
                __syncthreads();
                gu_fin(A, k);
                break;
            case O_SWEEP:
                step<OP_SWEEP>(A, k, src, nb, 0);
                break;
            case O_PRINIT: {
                int* D = dst(k);
                reset_lists(k);
                for (int l = threadIdx.x; l < N; l += CT) D[l] = 0;
                if (threadIdx.x == 0) s_.flag &= ~F_NEG;
                break;
            }
            case O_PR:
                step<OP_PR>(A, k, src, nb, 0);
                break;
            case O_PRFIN:
                if (c_.pr_ok_now) {
                    long long* P = prc();
                    const int* D = dst(k);
                    for (int l = threadIdx.x; l < N; l += CT) P[l] -= (long long)D[l];
                }
                reset_lists(k);
                break;
            default:
                break;
        }
        __syncthreads();
        if (op == O_BF) step_post<OP_BF>(A, k, src);
        else if (op == O_SWEEP) step_post<OP_SWEEP>(A, k, src);
        else if (op == O_PR) step_post<OP_PR>(A, k, src);
        if (threadIdx.x == 0) control(A, N);
        __syncthreads();
    }
    {
        const long long* P = prc();
        const int x0 = cd.cb[0];
        for (int l = threadIdx.x; l < N; l += CT) {
            const long long p = P[l];
            A.nd[ni(x0 + l)] = p;
            A.nd[ni(x0 + l) + 2] = p;
        }
    }
    if (threadIdx.x == 0) {
        const Ctl& c = c_;
        CellOut o{};
        o.status = c.status;
        o.phases = c.phases;
        o.updates = c.updates;
        o.pr_ok = c.pr_ok;
        o.pr_tries = c.pr_tries;
        o.last_eps = c.ended_at_one;
        o.sweeps = c.sweeps;
        o.bf_rounds = c.rounds;
        o.scans = ctr_[C_SCAN];
        o.visits = ctr_[C_VISIT];
        o.pushes = ctr_[C_PUSH];
        o.relabels = ctr_[C_RELABEL];
        o.gu_scans = ctr_[C_GUSCAN];
        o.ticks = __builtin_amdgcn_s_memrealtime() - c.t0;
        for (int i = 0; i < CELL_NOPS; ++i) {
            o.op_ticks[i] = c.op_ticks[i];
            o.op_n[i] = c.op_n[i];
        }
        A.out[blockIdx.x] = o;
    }
}

}  // namespace

size_t cell_lds_bytes(int n) {
    if (n < 0) return 0;
    const size_t w = ((size_t)n + 31) / 32;
    // prices 8n, distances 4n rounded up to whole 8-byte words, two bitmaps
    const size_t b = 8 * (size_t)n + 8 * (((size_t)n + 1) / 2) + 2 * 4 * w;
    const size_t dyn = (b + 15) / 16 * 16;
    return dyn + sizeof(St) + sizeof(Ctl) + 64 <= LDS_LIMIT ? dyn : 0;
}

int cell_max_nodes() {
    int lo = 0, hi = 1 << 16;
    while (hi - lo > 1) {
        const int mid = (lo + hi) / 2;
        if (cell_lds_bytes(mid)) lo = mid;
        else hi = mid;
    }
    return lo;
}

hipError_t cell_launch(const CellArgs& a, hipStream_t st) {
    const size_t lds = cell_lds_bytes(a.max_nodes);
    if (!lds || a.ncells <= 0) return hipErrorInvalidValue;
    // (per device and cheap: set on every launch)
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cell),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cell, dim3(a.ncells), dim3(CT), lds, st, a);
    return hipGetLastError();
}

}  // namespace ks
