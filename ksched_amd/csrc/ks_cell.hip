// ks_cell.hip — the whole ε-scaling push-relabel solve of a small graph inside
// one 1024-thread workgroup (ks_cell.h). Same algorithm as the
// multi-kernel engine (ks_engine.hip): phases ε ← ε/α, each
// starting by saturating every arc of negative reduced cost, then alternating a
// global price update (Bellman-Ford from the deficits over lengths
// floor(rc/ε)+1, prices p ← p − ε·min(d, L)) with bursts of push/relabel sweeps
// against a price snapshot; price refinement at ε = 1 certifies optimality. By
// default the final phase is replaced by the engine's cycle-cancelling finish
// (the phase before it drains; a refinement with parent keys, whose parent
// graph's negative cycles are found by pointer doubling and cancelled:
// cyc_search). What changes is where it runs:
//
//   control   the phase loop, every decision and every termination test run on
//             the device; a step (one sweep, one Bellman-Ford round) ends at a
//             workgroup barrier — ~1 µs instead of a ~10 µs dependent launch.
//   LDS       the cell's prices (int64) and Bellman-Ford distances (int32,
//             saturating at 2^30: any cap keeps the triangle inequality the
//             update needs) live in LDS, 12 B per node, so the random gather of
//             a relaxation or an arc scan is an LDS read; only the 16-B compact
//             residual positions (CellPos, streamed along each node's segment),
//             the segment table and the excess words come from L2.
//   frontier  per-class lists: a node enters the next frontier once, through a
//             test-and-set in an LDS bitmap, appended at its class's slice of a
//             list buffer in HBM. Waves take items from an LDS counter, the
//             costliest classes first: the whole workgroup per node above 512
//             positions (the cluster aggregator, the sink), one wave per node
//             (≤ 512), a 16- or 32-lane group per node (≤ 32: machines), one
//             thread per node (≤ 8: tasks, PUs — a bitmask of the positions that
//             need a push / relaxation / saturation, then only those).
//   latency   a solve issues 29 % of its CU's VALU ceiling (PMC: 7.5e7 wave64 VALU
//             instructions over 1.3e8 cycles, against 2 per cycle): it is bound by its
//             dependent chains and barriers; batched record loads are issued unconditionally and
//             pinned (a load in a lane-conditional branch waits there), lane-group
//             scans are DPP with the group's last lane as leader.
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

#include <algorithm>

namespace ks {
namespace {

constexpr int CT = CELL_THREADS;
constexpr int NW = CT / 64;
constexpr int DINF = 0x7fffffff;           // not reached by the update
constexpr long long DCAP = 1LL << 30;      // distances saturate here
constexpr long long DNEG = -(1LL << 30);   // price refinement below this: treated as a negative cycle
constexpr long long INF64 = 0x3fffffffffffffffLL;
constexpr int BXC = 256;                   // updates with at most this many excess nodes are bounded
// cycle-cancelling finish (cyc_search)
constexpr int CYC_LOG = 10;                 // cycles of up to 1,024 arcs
constexpr int CYC_WALK = 1 << CYC_LOG;
constexpr int CYC_EVERY = 16;               // refinement rounds between searches (8 and 32: no better)
constexpr int CYC_IDB = 15;                 // bits of a local node id in the packed word (cells ≤ 32k nodes)
constexpr int CYC_IDM = (1 << CYC_IDB) - 1;
constexpr int CYC_ON = 1 << 30;             // marked: on a cycle

enum { OP_SWEEP = 0, OP_BF = 1, OP_PR = 2, OP_SAT = 3 };
enum { F_INFEAS = 1, F_NEG = 2 };

struct St {
    int cnt[2][8];        // frontier list lengths per buffer and class
    int cbs[8];           // the cell's class bounds (dynamically indexed)
    int rl_cnt[2];        // pending relabels, by sweep parity
    int flag;             // F_INFEAS | F_NEG
    int stop;             // the wall-clock limit was hit
    int next;             // the step's next item (waves take items dynamically)
    int bnd;              // bounded update: offers at or above this distance are dropped (DINF: none)
    int nbx;              // excess nodes listed by gu_init (more than BXC: the update is unbounded)
    int bx[BXC];          // their local indices
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
    int pb;               // the cell's first position (compact records address reverses from it)
    int c1, c2, c3, c4, c5, c6;
    long long eps;
    int eps_shift;        // log2 ε when ε is a power of two (the cell ladder's are), else −1
    int sp;               // sweep parity (pending-relabel buffer)
    int bnd;              // s_.bnd at the step's start
    int prc;              // the refinement records parents (the cycle-cancelling finish)
};

// Work counters (ks_result units): counted per lane in registers, summed over the
// wave by DPP (no LDS round trips) and added to the workgroup's counters once per
// step.
enum { C_SCAN = 0, C_VISIT = 1, C_PUSH = 2, C_RELABEL = 3, C_GUSCAN = 4, NCTR = 5 };
__shared__ unsigned long long ctr_[NCTR];
__shared__ unsigned long long t_items_, t_first_;   // diagnostics: last / first wave's items done
__shared__ unsigned long long cls_t_[4][8];          // diagnostics: item ticks by step kind × node class
__shared__ unsigned cls_n_[4][8];                    //              and items
__device__ __forceinline__ int lane();
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
// A compact position (ks_cell.h CellPos) decoded into the engine's field names:
// scaled cost, residual, pair capacity, absolute head and reverse position.
constexpr long long DEAD_SCALED = 1LL << 60;
__device__ __forceinline__ int4 ld_raw(const CellArgs& A, int a) { return *reinterpret_cast<const int4*>(A.cp + a); }
__device__ __forceinline__ Pos dec(const CellArgs& A, const K& k, int4 w) {
    Pos r;
    r.rcap = w.x;
    r.ucap = w.y;
    r.cost = w.z == CELL_DEAD ? DEAD_SCALED : (long long)w.z;
    r.head = k.x0 + (int)((unsigned)w.w & ((1u << CELL_HEAD_BITS) - 1));
    r.rev = k.pb + (int)((unsigned)w.w >> CELL_HEAD_BITS);
    return r;
}
__device__ __forceinline__ Pos ld_cp(const CellArgs& A, const K& k, int a) { return dec(A, k, ld_raw(A, a)); }
// Pins a batch's loaded records in VGPRs at this point (one wait for the whole
// batch): without it the compiler sinks a load into the branch of its only use,
// where it gets its own s_waitcnt and the batch runs one load at a time.
template <int N>
__device__ __forceinline__ void pin(int4 (&q)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(q[i].x), "+v"(q[i].y), "+v"(q[i].z), "+v"(q[i].w));
}
__device__ __forceinline__ void st_rcap(const CellArgs& A, int a, long long v) { A.cp[a].rcap = (int)v; }

// a node's positions [first[x], first[x+1]): 4 B per node, so a cell's segment
// table is 48 KB of L2 instead of its 388 KB of 32-B node records (config 5, eight
// cells sharing each XCD's L2: 65.0 → 62.3 ms in an interleaved A/B)
__device__ __forceinline__ void seg(const CellArgs& A, int x, int& b0, int& b1) {
    b0 = A.first[x];
    b1 = A.first[x + 1];
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

// DPP lane-group scans (G = 4…64, aligned groups): row_shr within 16-lane rows,
// then row_bcast:15 / :31 across rows. The inclusive result of the group's LAST
// lane is the group total (sum) or minimum (min): leaf groups lead from that lane,
// so no broadcast is needed.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, false);
}
// l = lane & (G − 1), computed once by the caller: lane() is a volatile asm, a
// scheduling barrier that would keep a batch's loads apart.
template <int G>
__device__ __forceinline__ int gs_add(int x, int l) {
    int y = dpp_i32<0x111, 0xf>(x);   // row_shr:1
    if (l >= 1) x += y;
    y = dpp_i32<0x112, 0xf>(x);       // row_shr:2
    if (l >= 2) x += y;
    if (G > 4) {
        y = dpp_i32<0x114, 0xf>(x);   // row_shr:4
        if (l >= 4) x += y;
    }
    if (G > 8) {
        y = dpp_i32<0x118, 0xf>(x);   // row_shr:8
        if (l >= 8) x += y;
    }
    if (G > 16) x += dpp_i32<0x142, 0xa>(x);   // row_bcast:15 → rows 1, 3
    if (G > 32) x += dpp_i32<0x143, 0xc>(x);   // row_bcast:31 → rows 2, 3
    return x;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ long long dpp_i64(long long v, long long fill) {
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned long long)fill, (int)(unsigned long long)v, CTRL,
                                               ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)((unsigned long long)fill >> 32),
                                               (int)((unsigned long long)v >> 32), CTRL, ROW_MASK, 0xf, false);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// inclusive prefix minimum over the group (64-bit); the last lane holds the group min
template <int G>
__device__ __forceinline__ long long gs_min(long long x, int l) {
    long long y = dpp_i64<0x111, 0xf>(x, INF64);
    if (l >= 1) x = min(x, y);
    y = dpp_i64<0x112, 0xf>(x, INF64);
    if (l >= 2) x = min(x, y);
    if (G > 4) {
        y = dpp_i64<0x114, 0xf>(x, INF64);
        if (l >= 4) x = min(x, y);
    }
    if (G > 8) {
        y = dpp_i64<0x118, 0xf>(x, INF64);
        if (l >= 8) x = min(x, y);
    }
    if (G > 16) x = min(x, dpp_i64<0x142, 0xa>(x, INF64));
    if (G > 32) x = min(x, dpp_i64<0x143, 0xc>(x, INF64));
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
    st_rcap(A, a, r - d);
    st_rcap(A, rv, uc - (r - d));
    add_ex(A, w, d);
    mark(A, k, nb, w);
}
// the relabel of v takes effect after the sweep (price snapshot)
__device__ __forceinline__ void relabel(const CellArgs& A, const K& k, int v, long long np) {
    const int i = atomicAdd(&s_.rl_cnt[k.sp], 1);
    A.rl_node[k.x0 + i] = v;
    A.rl_p[k.x0 + i] = np;
}

// Wave- and workgroup-sized nodes walk their positions UC chunks at a time: every
// chunk's record loads are issued before the first is used (one chunk per round
// trip left a 450-position aggregator eight dependent L2 latencies per visit).
constexpr int UC = 4;

__device__ __forceinline__ long long uni64(long long x) {   // a wave-uniform copy (x is the same in every lane)
    const unsigned long long u = (unsigned long long)x;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ long long lane63_64(long long x) {
    const unsigned long long u = (unsigned long long)x;
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// The relabel minimum over v's positions: residual arcs (admissible ones only when
// the push left residual) and arcs of reduced cost in (0, ε] (ks_engine.hip
// sweep_group).
__device__ __forceinline__ void minc_acc(long long& minc, bool valid, long long cr, int r, int d, long long eps) {
    if (!valid) return;
    if (cr < 0) {
        if (r - d > 0) minc = min(minc, cr);
    } else if (r > 0 || cr <= eps) {
        minc = min(minc, cr);
    }
}

// One node per wave (classes of ≤ 64 and ≤ 512 positions; v uniform): the excess
// is spread over the admissible arcs in position order by a wave prefix sum; a
// node that saturates all of them relabels to p − (minc + ε).
__device__ __forceinline__ void sweep_wave(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const long long* P = prc();
    const long long e = uni64(ld_ex(A, v));
    if (e <= 0) return;
    const long long pv = P[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    const int ln = lane();
    t.c[C_VISIT] += ln == 0;
    long long rem = e, minc = INF64;
    for (int base = b0; base < en; base += 64 * UC) {
        int4 qr[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const int a = base + 64 * u + ln;
            qr[u] = ld_raw(A, a < en ? a : b0);
        }
        pin(qr);
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const Pos Q = dec(A, k, qr[u]);
            const int a = base + 64 * u + ln;
            const bool valid = a < en;
            int r = 0;
            long long cr = 0;
            if (valid) {
                r = (int)Q.rcap;
                cr = Q.cost + pv - P[Q.head - k.x0];
            }
            t.c[C_SCAN] += valid;
            const int adm = (valid && cr < 0 && r > 0) ? r : 0;
            const int incl = gs_add<64>(adm, ln);
            const int tot = __builtin_amdgcn_readlane(incl, 63);
            const long long ex = rem - (incl - adm);
            const int d = ex <= 0 ? 0 : (ex < adm ? (int)ex : adm);
            if (d > 0) {
                push(A, k, nb, a, Q.head, r, d, Q.rev, Q.ucap);
                ++t.c[C_PUSH];
            }
            minc_acc(minc, valid, cr, r, d, k.eps);
            rem -= tot < rem ? tot : rem;
        }
        if (rem == 0) break;
    }
    if (rem > 0) minc = lane63_64(gs_min<64>(minc, ln));   // (rem is uniform: only a relabel needs it)
    if (ln == 63) {
        const long long pushed = e - rem;
        if (pushed) add_ex(A, v, -pushed);
        if (rem > 0) {
            ++t.c[C_RELABEL];
            if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
            else relabel(A, k, v, pv - (minc + k.eps));
            mark(A, k, nb, v);
        }
    }
}

// The same for a node above 512 positions: the whole workgroup, each thread UC
// consecutive positions (position order kept), one workgroup prefix sum per
// CT·UC positions. v is uniform.
__device__ __forceinline__ void sweep_hub(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const long long* P = prc();
    const long long e = ld_ex(A, v);
    const long long pv = P[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    if (e <= 0) return;
    t.c[C_VISIT] += threadIdx.x == 0;
    long long rem = e, minc = INF64;
    for (int base = b0; base < en; base += CT * UC) {
        const int a0 = base + (int)threadIdx.x * UC;
        int4 qr[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) qr[u] = ld_raw(A, a0 + u < en ? a0 + u : b0);
        pin(qr);
        long long cr[UC];
        int adm[UC], my = 0;
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const Pos Q = dec(A, k, qr[u]);
            const bool valid = a0 + u < en;
            cr[u] = valid ? Q.cost + pv - P[Q.head - k.x0] : 0;
            adm[u] = (valid && cr[u] < 0 && Q.rcap > 0) ? (int)Q.rcap : 0;
            my += adm[u];
            t.c[C_SCAN] += valid;
        }
        long long tot;
        long long before = blk_excl_scan(my, &tot);
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const Pos Q = dec(A, k, qr[u]);
            const int r = (int)Q.rcap;
            long long d = rem - before;
            d = d < 0 ? 0 : (d > adm[u] ? adm[u] : d);
            before += adm[u];
            if (d > 0) {
                push(A, k, nb, a0 + u, Q.head, r, d, Q.rev, Q.ucap);
                ++t.c[C_PUSH];
            }
            minc_acc(minc, a0 + u < en, cr[u], r, (int)d, k.eps);
        }
        rem -= tot < rem ? tot : rem;
        if (rem == 0) break;
    }
    if (rem > 0) minc = blk_min(minc);   // (uniform over the workgroup)
    if (threadIdx.x == 0) {
        const long long pushed = e - rem;
        if (pushed) add_ex(A, v, -pushed);
        if (rem > 0) {
            ++t.c[C_RELABEL];
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
// the finish's parent keys: offer (biased into 32 bits) above the parent arc's position
constexpr unsigned long long PKEY_NONE = ~0ULL;
__device__ __forceinline__ unsigned long long pkey(long long d, int a) {
    return ((unsigned long long)(d + (1LL << 31)) << 32) | (unsigned)a;   // d in [DNEG, DCAP]
}
__device__ __forceinline__ int key_pos(unsigned long long k) {
    return k == PKEY_NONE ? -1 : (int)(unsigned)(k & 0xffffffffULL);
}
// (the keys change only by atomics, performed in L2: read them there, not from L1)
__device__ __forceinline__ int key_at(const unsigned long long* key, int l) {
    return key_pos(__hip_atomic_load(key + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <bool PR>
__device__ __forceinline__ void relax_q(const CellArgs& A, const K& k, int nb, const Pos& q, int dv, long long pv) {
    if (q.ucap - q.rcap <= 0) return;
    const int lu = q.head - k.x0;
    const long long pu = prc()[lu];
    int* D = dst(k);
    const long long x = pu - q.cost - pv;
    if (!PR) {
        // global update, in 32 bits past the price difference: len = clamp(⌊x/ε⌋ + 1,
        // 0, DCAP) and a reached dv ≤ DCAP, so dv + len ≤ 2^31 fits an unsigned word
        const long long lq = k.eps_shift >= 0 ? (x >> k.eps_shift) : floordiv(x, k.eps);
        const unsigned len = lq < 0 ? 0u : (lq >= DCAP - 1 ? (unsigned)DCAP : (unsigned)lq + 1u);
        unsigned c = (unsigned)dv + len;
        c = c > (unsigned)DCAP ? (unsigned)DCAP : c;
        const int cand = (int)c;
        if (cand >= k.bnd) return;   // bounded update: beyond every excess node
        if (cand < D[lu]) {
            const int old = atomicMin(&D[lu], cand);
            if (cand < old) mark(A, k, nb, q.head);
        }
        return;
    }
    long long len = x + 1;
    len = len > DCAP ? DCAP : (len < DNEG ? DNEG : len);
    long long cand = (long long)dv + len;
    if (cand > DCAP) cand = DCAP;
    if (cand < DNEG) {
        cand = DNEG;
        atomicOr(&s_.flag, F_NEG);
    }
    if (cand < (long long)D[lu]) {
        const int old = atomicMin(&D[lu], (int)cand);
        if (cand < (long long)old) {
            mark(A, k, nb, q.head);
            // the parent arc (head → v, the reverse of q) for the finish's cycle search:
            // the least offer's, as the engine's packed keys (a 64-bit key in global
            // memory, offer above the position: the minimum is the final distance's arc)
            if (k.prc) atomicMin(reinterpret_cast<unsigned long long*>(A.rl_p) + q.head, pkey(cand, q.rev));
        }
    }
}

// One node's in-arcs by one wave (W = 64, v uniform) or the workgroup (W = CT).
template <int W, bool PR>
__device__ __forceinline__ void bf_node(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const int dv = dst(k)[v - k.x0];
    if (!PR && dv >= k.bnd) return;   // (k.bnd ≤ DINF: unreached nodes too)
    const int me = W == 64 ? lane() : (int)threadIdx.x;
    const long long pv = prc()[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    for (int base = b0 + me; base < en; base += W * UC) {
        int4 qr[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u)
            qr[u] = ld_raw(A, base + W * u < en ? base + W * u : base);
        pin(qr);
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const Pos Q = dec(A, k, qr[u]);
            if (base + W * u < en) {
                relax_q<PR>(A, k, nb, Q, dv, pv);
                ++t.c[C_GUSCAN];
            }
        }
    }
}

// -------------------------------------------------------------- saturate ---
// Goldberg's refine start: every residual arc of reduced cost below −thr is
// saturated (thr = ε after a failed refinement or on a warm start). W as bf_node.
template <int W>
__device__ __forceinline__ void sat_node(const CellArgs& A, K& k, int v, long long thr, Tc& t) {
    const long long* P = prc();
    const long long pv = P[v - k.x0];
    int b0, en;
    seg(A, v, b0, en);
    const int me = W == 64 ? lane() : (int)threadIdx.x;
    long long tot = 0;
    for (int base = b0 + me; base < en; base += W * UC) {
        int4 qr[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u)
            qr[u] = ld_raw(A, base + W * u < en ? base + W * u : base);
        pin(qr);
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const Pos Q = dec(A, k, qr[u]);
            const int a = base + W * u;
            if (a < en && Q.rcap > 0 && Q.cost + pv - P[Q.head - k.x0] < -thr) {
                st_rcap(A, a, 0);
                st_rcap(A, Q.rev, Q.ucap);
                add_ex(A, Q.head, Q.rcap);
                tot += Q.rcap;
                ++t.c[C_PUSH];
            }
        }
    }
    if (W == 64) {
        tot = lane63_64(g_sum<64>(tot));
        if (lane() == 0 && tot) add_ex(A, v, -tot);
    } else {
        tot = blk_sum(tot);
        if (threadIdx.x == 0 && tot) add_ex(A, v, -tot);
    }
}

// ------------------------------------------------ leaf classes, U at a time ---
// Classes of ≤ 32 positions (PUs, tasks, machines): one node per G-lane group, one
// position per lane (a task's eight 16-B records are one coalesced line), and U
// batches of 64/G nodes in flight per wave: every batch's list, segment and
// position loads are issued before any of them is used (one batch per wave left
// each wave one dependent chain at a time — latency-bound at ~1.5 µs per batch).
template <int G>
struct LeafU {
    static constexpr int U = G <= 16 ? 4 : 2;
};

// A batch's segment and record loads, all unconditional (indices clamped to the
// cell's first node / position 0, masked after): a load inside a lane-conditional
// branch gets its own s_waitcnt there, which serialises the batch.
template <int G, int U>
__device__ __forceinline__ void leaf_load(const CellArgs& A, const K& k, int lig, const int (&v)[U], int (&b0)[U],
                                          int (&en)[U], int4 (&qr)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        seg(A, v[u] >= 0 ? v[u] : k.x0, b0[u], en[u]);
        if (v[u] < 0) en[u] = b0[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int a = b0[u] + lig;
        qr[u] = ld_raw(A, a < en[u] ? a : 0);
    }
    pin(qr);
}

template <int G, int U>
__device__ __forceinline__ void sweep_leaf(const CellArgs& A, K& k, int nb, const int (&v)[U], Tc& t) {
    const long long* P = prc();
    const int lig = lane() & (G - 1);
    const bool lead = lig == G - 1;
    long long e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = ld_ex(A, v[u] >= 0 ? v[u] : k.x0);
    int b0[U], en[U];
    int4 qr[U];
    leaf_load<G, U>(A, k, lig, v, b0, en, qr);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v[u] < 0) e[u] = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const Pos Q = dec(A, k, qr[u]);
        const bool act = e[u] > 0;
        const int a = b0[u] + lig;
        const bool valid = act && a < en[u];
        const long long pv = v[u] >= 0 ? P[v[u] - k.x0] : 0;
        int r = 0;
        long long cr = 0;
        if (valid) {
            r = (int)Q.rcap;
            cr = Q.cost + pv - P[Q.head - k.x0];
        }
        t.c[C_SCAN] += valid;
        t.c[C_VISIT] += act && lead;
        const int adm = (valid && cr < 0 && r > 0) ? r : 0;
        const int incl = gs_add<G>(adm, lig);                       // the last lane: the group's admissible total
        const long long ex = e[u] - (incl - adm);              // what is left when this arc's turn comes
        const int d = ex <= 0 ? 0 : (ex < adm ? (int)ex : adm);
        if (d > 0) {
            push(A, k, nb, a, Q.head, r, d, Q.rev, Q.ucap);
            ++t.c[C_PUSH];
        }
        long long minc = INF64;
        if (valid) {
            if (cr < 0) {
                if (r - d > 0) minc = cr;
            } else if (r > 0 || cr <= k.eps) {
                minc = cr;
            }
        }
        // the group minimum (at the last lane) — only when some node of the wave
        // keeps excess and relabels: a node that pushed it all does not need it
        if (__ballot(act && lead && e[u] > incl)) minc = gs_min<G>(minc, lig);
        if (act && lead) {
            const long long rem = e[u] > incl ? e[u] - incl : 0;
            const long long pushed = e[u] - rem;
            if (pushed) add_ex(A, v[u], -pushed);
            if (rem > 0) {
                ++t.c[C_RELABEL];
                if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
                else relabel(A, k, v[u], pv - (minc + k.eps));
                mark(A, k, nb, v[u]);
            }
        }
    }
}

template <int G, int U, bool PR>
__device__ __forceinline__ void bf_leaf(const CellArgs& A, K& k, int nb, const int (&v)[U], Tc& t) {
    const int lig = lane() & (G - 1);
    int b0[U], en[U];
    int4 qr[U];
    leaf_load<G, U>(A, k, lig, v, b0, en, qr);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const Pos Q = dec(A, k, qr[u]);
        if (b0[u] + lig >= en[u]) continue;
        const int dv = dst(k)[v[u] - k.x0];
        if (!PR && dv >= k.bnd) continue;
        relax_q<PR>(A, k, nb, Q, dv, prc()[v[u] - k.x0]);
        ++t.c[C_GUSCAN];
    }
}

template <int G, int U>
__device__ __forceinline__ void sat_leaf(const CellArgs& A, K& k, const int (&v)[U], long long thr, Tc& t) {
    const long long* P = prc();
    const int lig = lane() & (G - 1);
    int b0[U], en[U];
    int4 qr[U];
    leaf_load<G, U>(A, k, lig, v, b0, en, qr);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const Pos Q = dec(A, k, qr[u]);
        const int a = b0[u] + lig;
        int tot = 0;
        if (a < en[u]) {
            const long long pv = P[v[u] - k.x0];
            if (Q.rcap > 0 && Q.cost + pv - P[Q.head - k.x0] < -thr) {
                st_rcap(A, a, 0);
                st_rcap(A, Q.rev, Q.ucap);
                add_ex(A, Q.head, Q.rcap);
                tot = (int)Q.rcap;
                ++t.c[C_PUSH];
            }
        }
        tot = gs_add<G>(tot, lig);
        if (v[u] >= 0 && lig == G - 1 && tot) add_ex(A, v[u], -(long long)tot);
    }
}

// ------------------------------------------------ one thread per node ---
// Classes of ≤ 4 and ≤ 8 positions (PUs, tasks): a node per thread, 64 per wave.
// A cheap pass over all of a node's records (loaded at once, unconditionally)
// builds a bitmask of the positions that need the expensive path — a push, a
// relaxation, a saturation — and a ctz loop then takes only those, re-reading the
// record (an L1 hit). A task has about one such position, so a wave runs the
// expensive path about once per 64 tasks instead of once per position index
// (fewer VALU instructions per wave, and fewer lanes idle in the expensive path).
template <int MAXP>
__device__ __forceinline__ int thr_load(const CellArgs& A, const K& k, int v, int& b0, int4 (&qr)[MAXP]) {
    int en;
    seg(A, v >= 0 ? v : k.x0, b0, en);
    const int cnt = v >= 0 ? en - b0 : 0;
#pragma unroll
    for (int i = 0; i < MAXP; ++i) qr[i] = ld_raw(A, i < cnt ? b0 + i : 0);
    pin(qr);
    return cnt;
}

template <int MAXP>
__device__ __forceinline__ void sweep_thr(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const long long* P = prc();
    const long long e0 = ld_ex(A, v >= 0 ? v : k.x0);
    int b0;
    int4 qr[MAXP];
    const int cnt = thr_load<MAXP>(A, k, v, b0, qr);
    const long long e = v >= 0 ? e0 : 0;
    if (e <= 0) return;
    const long long pv = P[v - k.x0];
    ++t.c[C_VISIT];
    t.c[C_SCAN] += cnt;
    long long rem = e, minc = INF64;
    unsigned pm = 0;   // positions that receive a push
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
        if (i >= cnt) break;
        const Pos Q = dec(A, k, qr[i]);
        const int r = (int)Q.rcap;
        const long long cr = Q.cost + pv - P[Q.head - k.x0];
        if (cr < 0) {   // admissible when residual (the relabel minimum as in sweep_leaf)
            if (r > 0) {
                const long long d = rem < r ? rem : r;
                if (d > 0) pm |= 1u << i;
                rem -= d;
                if (r - d > 0) minc = min(minc, cr);
            }
        } else if (r > 0 || cr <= k.eps) {
            minc = min(minc, cr);
        }
    }
    long long left = e;
    while (pm) {   // in position order: the same amounts as above (an admissible arc is
                   // not changed by another node's push within the sweep)
        const int i = __builtin_ctz(pm);
        pm &= pm - 1;
        const int a = b0 + i;
        const Pos Q = ld_cp(A, k, a);
        const int r = (int)Q.rcap;
        const int d = left < r ? (int)left : r;
        left -= d;
        push(A, k, nb, a, Q.head, r, d, Q.rev, Q.ucap);
        ++t.c[C_PUSH];
    }
    const long long pushed = e - rem;
    if (pushed) add_ex(A, v, -pushed);
    if (rem > 0) {
        ++t.c[C_RELABEL];
        if (minc >= INF64) atomicOr(&s_.flag, F_INFEAS);
        else relabel(A, k, v, pv - (minc + k.eps));
        mark(A, k, nb, v);
    }
}

template <int MAXP, bool PR>
__device__ __forceinline__ void bf_thr(const CellArgs& A, K& k, int nb, int v, Tc& t) {
    const int vc = v >= 0 ? v : k.x0;
    const int dv = dst(k)[vc - k.x0];
    int b0;
    int4 qr[MAXP];
    int cnt = thr_load<MAXP>(A, k, v, b0, qr);
    if (!PR && dv >= k.bnd) cnt = 0;
    t.c[C_GUSCAN] += cnt;
    unsigned m = 0;   // positions whose reverse (an in-arc of v) is residual
#pragma unroll
    for (int i = 0; i < MAXP; ++i)
        if (i < cnt && qr[i].y - qr[i].x > 0) m |= 1u << i;
    if (!m) return;
    const long long pv = prc()[vc - k.x0];
    while (m) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        relax_q<PR>(A, k, nb, ld_cp(A, k, b0 + i), dv, pv);
    }
}

template <int MAXP>
__device__ __forceinline__ void sat_thr(const CellArgs& A, K& k, int v, long long thr, Tc& t) {
    const long long* P = prc();
    int b0;
    int4 qr[MAXP];
    const int cnt = thr_load<MAXP>(A, k, v, b0, qr);
    if (!cnt) return;
    const long long pv = P[v - k.x0];
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
        if (i >= cnt) break;
        const Pos Q = dec(A, k, qr[i]);
        if (Q.rcap > 0 && Q.cost + pv - P[Q.head - k.x0] < -thr) m |= 1u << i;
    }
    long long tot = 0;
    while (m) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        const int a = b0 + i;
        const Pos Q = ld_cp(A, k, a);
        st_rcap(A, a, 0);
        st_rcap(A, Q.rev, Q.ucap);
        add_ex(A, Q.head, Q.rcap);
        tot += Q.rcap;
        ++t.c[C_PUSH];
    }
    if (tot) add_ex(A, v, -tot);
}

// ------------------------------------------------------------------ step ---
constexpr int THR_CLASSES = 2;   // classes 0, 1: a node per thread; 2, 3: a lane group per node
__host__ __device__ constexpr int items_per_wave(int c) {   // leaf nodes per item
    return c < THR_CLASSES ? 64 : c < 4 ? (64 / (4 << c)) * ((4 << c) <= 16 ? 4 : 2) : 1;
}

// An item: a batch of leaf-class nodes, or one node of the ≤ 64 / ≤ 512-position
// classes (the wave).
template <int OP, int C>
__device__ __forceinline__ void item(const CellArgs& A, K& k, int src, int nb, int j, int n, long long thr, Tc& t) {
    if (C < THR_CLASSES) {
        const int idx = j * 64 + lane();
        int v;
        if (src == 2) v = idx < n ? s_.cbs[C] + idx : -1;
        else {
            const int x = A.lists[(size_t)src * A.nn + s_.cbs[C] + (idx < n ? idx : 0)];
            v = idx < n ? x : -1;
        }
        constexpr int MAXP = 4 << C;
        if (OP == OP_SWEEP) sweep_thr<MAXP>(A, k, nb, v, t);
        else if (OP == OP_BF) bf_thr<MAXP, false>(A, k, nb, v, t);
        else if (OP == OP_PR) bf_thr<MAXP, true>(A, k, nb, v, t);
        else sat_thr<MAXP>(A, k, v, thr, t);
        return;
    }
    if (C < 4) {
        constexpr int G = 4 << C;
        constexpr int U = LeafU<G>::U;
        int v[U];
        const int grp = lane() / G;
        if (src == 2) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int idx = (j * U + u) * (64 / G) + grp;
                v[u] = idx < n ? s_.cbs[C] + idx : -1;
            }
        } else {   // the list loads unconditional and outside any per-batch branch (see leaf_load)
            const int* L = A.lists + (size_t)src * A.nn + s_.cbs[C];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int idx = (j * U + u) * (64 / G) + grp;
                const int x = L[idx < n ? idx : 0];
                v[u] = idx < n ? x : -1;
            }
        }
        if (OP == OP_SWEEP) sweep_leaf<G, U>(A, k, nb, v, t);
        else if (OP == OP_BF) bf_leaf<G, U, false>(A, k, nb, v, t);
        else if (OP == OP_PR) bf_leaf<G, U, true>(A, k, nb, v, t);
        else sat_leaf<G, U>(A, k, v, thr, t);
        return;
    }
    const int v = __builtin_amdgcn_readfirstlane(node_at(A, src, C, j));
    if (OP == OP_SWEEP) sweep_wave(A, k, nb, v, t);
    else if (OP == OP_BF) bf_node<64, false>(A, k, nb, v, t);
    else if (OP == OP_PR) bf_node<64, true>(A, k, nb, v, t);
    else sat_node<64>(A, k, v, thr, t);
}

// One step over frontier src (2: every node) into buffer nb: the workgroup-
// sized nodes one after another with every thread, then the rest as items
// (a batch of 64/G nodes of one class, or one ≤ 512-position node) dealt to the
// 16 waves. The caller's barrier completes buffer nb; step_post then empties src.
template <int OP>
__device__ __forceinline__ void step(const CellArgs& A, K& k, int src, int nb, long long thr) {
    Tc t;
    const int n6 = count_of(src, 6);
    for (int j = 0; j < n6; ++j) {
        const int v = node_at(A, src, 6, j);
        __syncthreads();   // the previous node's pushes and marks are in
        const unsigned long long h0 = A.diag ? __builtin_amdgcn_s_memrealtime() : 0;
        if (OP == OP_SWEEP) sweep_hub(A, k, nb, v, t);
        else if (OP == OP_BF) bf_node<CT, false>(A, k, nb, v, t);
        else if (OP == OP_PR) bf_node<CT, true>(A, k, nb, v, t);
        else sat_node<CT>(A, k, v, thr, t);
        if (A.diag && threadIdx.x == 0) {
            atomicAdd(&cls_t_[OP][6], __builtin_amdgcn_s_memrealtime() - h0);
            atomicAdd(&cls_n_[OP][6], 1u);
        }
    }
    const int n0 = count_of(src, 0), n1 = count_of(src, 1), n2 = count_of(src, 2), n3 = count_of(src, 3),
              n4 = count_of(src, 4), n5 = count_of(src, 5);
    constexpr int p0 = items_per_wave(0), p1 = items_per_wave(1), p2 = items_per_wave(2), p3 = items_per_wave(3);
    // the costliest items first (an aggregator per wave, then machines, then
    // batches of tasks), taken dynamically: the step's tail is its cheapest items
    const int e5 = n5;
    const int e4 = e5 + n4;
    const int e3 = e4 + (n3 + p3 - 1) / p3;
    const int e2 = e3 + (n2 + p2 - 1) / p2;
    const int e1 = e2 + (n1 + p1 - 1) / p1;
    const int e0 = e1 + (n0 + p0 - 1) / p0;
    for (;;) {
        int it0 = 0;
        if (lane() == 0) it0 = atomicAdd(&s_.next, 1);
        const int it = __builtin_amdgcn_readfirstlane(it0);
        if (it >= e0) break;
        const unsigned long long i0 = A.diag ? __builtin_amdgcn_s_memrealtime() : 0;
        const int cl = it < e5 ? 5 : it < e4 ? 4 : it < e3 ? 3 : it < e2 ? 2 : it < e1 ? 1 : 0;
        if (it < e5) item<OP, 5>(A, k, src, nb, it, n5, thr, t);
        else if (it < e4) item<OP, 4>(A, k, src, nb, it - e5, n4, thr, t);
        else if (it < e3) item<OP, 3>(A, k, src, nb, it - e4, n3, thr, t);
        else if (it < e2) item<OP, 2>(A, k, src, nb, it - e3, n2, thr, t);
        else if (it < e1) item<OP, 1>(A, k, src, nb, it - e2, n1, thr, t);
        else item<OP, 0>(A, k, src, nb, it - e1, n0, thr, t);
        if (A.diag && lane() == 0) {
            atomicAdd(&cls_t_[OP][cl], __builtin_amdgcn_s_memrealtime() - i0);
            atomicAdd(&cls_n_[OP][cl], 1u);
        }
    }
    flush(t);
    if (A.diag && lane() == 0) {   // when this wave's items were done (diagnostics: item span vs barrier tail)
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        atomicMax(&t_items_, now);
        atomicMin(&t_first_, now);
    }
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
enum Op { O_SAT, O_GUINIT, O_BF, O_GUFIN, O_SWEEP, O_PRINIT, O_PR, O_PRFIN, O_CYC, O_DONE };
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
    int drain;                // this phase drains: the cycle-cancelling finish follows it
    int prc, prc_tried;       // the finish's refinement is running / was tried
    int cycles, searches;     // cycles it cancelled, parent-graph searches
    int rejected;             // leader walks that did not close a cycle
    unsigned cyc_dbg[4];
    unsigned long long phase_sweeps, sweeps, rounds;
    unsigned long long t_op;                // when the running operation started
    unsigned long long op_ticks[O_DONE];    // 100 MHz ticks per operation kind (incl. its barriers)
    unsigned op_n[O_DONE];
    unsigned long long item_ticks[O_DONE];  // op start → the last wave's items done
    unsigned long long first_ticks[O_DONE]; // op start → the first wave's items done
    int fsz;                                // diagnostics: the running step's frontier size
    unsigned long long hist_t[12];          //              sweep / BF ticks by frontier size (≤16, 64, 256, 1k, 4k, more)
    unsigned hist_n[12];
    unsigned long long phase_ticks[8];      //              ticks by phase (slot 7: later phases, refinements)
    unsigned long long t_phase;             //              when the running phase (or refinement) began
};
__shared__ Ctl c_;

__device__ __forceinline__ int total_any(int src) { return total_of(src); }

// thread 0 only: a phase of ε = eps_ph begins (DESIGN §3 ε schedule)
__device__ __forceinline__ void phase_tick(unsigned long long now) {   // diagnostics
    Ctl& c = c_;
    const int slot = c.op == O_PR || c.op == O_PRINIT || c.op == O_PRFIN ? 7 : min(7, max(0, c.phases - 1));
    c.phase_ticks[slot] += now - c.t_phase;
    c.t_phase = now;
}
__device__ __forceinline__ void begin_phase(const CellArgs& A) {
    Ctl& c = c_;
    ++c.phases;
    c.thr = (c.phases == 1 && A.warm) ? A.sat_thr0 : ((c.pr_failed || A.warm >= 2) ? c.eps_ph : 0LL);
    c.pr_failed = 0;
    const bool last = c.eps_ph / A.alpha < 1 || c.eps_ph <= 1 || (A.use_pr && c.eps_ph * A.pr_div < A.mult);
    c.early = last ? 0 : 1;
    // the phase before the last drains when the cycle-cancelling finish replaces the
    // last one
    const long long nx = c.eps_ph / A.alpha > 1 ? c.eps_ph / A.alpha : 1;
    const bool before_last = !last && (nx / A.alpha < 1 || nx <= 1 || (A.use_pr && nx * A.pr_div < A.mult));
    c.drain = A.use_prc && before_last && !c.prc_tried;
    if (c.drain) c.early = 0;
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
    if (c.drain) {   // the drained flow: refinement with parents, cancelling the cycles it meets
        c.drain = 0;
        c.prc_tried = 1;
        c.prc = 1;
        c.op = O_PRINIT;
        c.pr_cap = A.prc_cap;
        c.pr_next = N_PHASE_LOOP;
        return;
    }
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

__device__ __forceinline__ void control_body(const CellArgs& A, int N, unsigned long long now);
// One clock read per operation (a scalar-memory round trip on thread 0, between
// the workgroup's two barriers): the operation's time, the timeout, the next start.
__device__ __forceinline__ void control(const CellArgs& A, int N) {
    Ctl& c = c_;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (c.op == O_SWEEP || c.op == O_BF) {
        const int f = c.fsz;
        const int b = f <= 16 ? 0 : f <= 64 ? 1 : f <= 256 ? 2 : f <= 1024 ? 3 : f <= 4096 ? 4 : 5;
        const int h = (c.op == O_BF ? 6 : 0) + b;
        c.hist_t[h] += now - c.t_op;
        ++c.hist_n[h];
    }
    control_body(A, N, now);
    c.fsz = c.src < 2 ? total_any(c.src) : N;
}
__device__ __forceinline__ void control_body(const CellArgs& A, int N, unsigned long long now) {
    Ctl& c = c_;
    s_.next = 0;   // the next step's item dispenser (read after the barrier that follows)
    c.op_ticks[c.op] += now - c.t_op;
    if (t_items_ > c.t_op) c.item_ticks[c.op] += t_items_ - c.t_op;
    if (t_first_ > c.t_op && t_first_ != ~0ULL) c.first_ticks[c.op] += t_first_ - c.t_op;
    ++c.op_n[c.op];
    t_items_ = 0;
    t_first_ = ~0ULL;
    c.t_op = now;
    if (now - c.t0 > A.timeout_ticks) return finish(CS_TIMEOUT);
    if (A.diag) phase_tick(now);
    // TESTS ONLY: one cell gives up part-way, as a step cap would (the host then
    // re-solves that cell alone on the engine)
    if ((int)blockIdx.x == A.fault_cell) {
        unsigned ops = 0;
        for (int i = 0; i < O_DONE; ++i) ops += c.op_n[i];
        if ((int)ops >= A.fault_ops) return finish(CS_NOCONV);
    }
    switch (c.op) {
        case O_SAT:
            s_.bnd = DINF;
            s_.nbx = 0;
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
            s_.bnd = DINF;   // the next update lists its excess nodes afresh
            s_.nbx = 0;
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
                if (c.prc && c.pr_rounds % CYC_EVERY == 0) c.op = O_CYC;   // not converged yet: search
                return;
            }
            c.op = O_PRFIN;
            return;
        case O_CYC:
            ++c.searches;
            c.op = O_PR;
            return;
        case O_PRFIN:
            c.prc = 0;
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
        if (A.bound && e > 0) {
            const int i = atomicAdd(&s_.nbx, 1);
            if (i < BXC) s_.bx[i] = l;
        }
    }
}
// Bounded update (the engine's k_gu_max bound): once every listed excess
// node is reached, B = their largest tentative distance, and offers at or above B
// are dropped. Every node below B is still exact (lengths are ≥ 0), excess nodes
// included, and gu_fin caps L at B, so min(d, L) keeps the triangle inequality.
// B only falls, so a stale copy read during a round is safe. After a step's barrier.
__device__ __forceinline__ void gu_bound(const K& k) {
    if (threadIdx.x >= 64) return;
    const int n = s_.nbx;
    if (n == 0 || n > BXC) return;
    const int ln = (int)threadIdx.x;
    long long d = 0;
    for (int i = ln; i < n; i += 64) d = max(d, (long long)dst(k)[s_.bx[i]]);
    const long long b = g_max<64>(d);
    if (ln == 0 && b < (long long)s_.bnd) s_.bnd = (int)b;
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
    if (L > (long long)k.bnd) L = k.bnd;
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

// ------------------------------------------------ cycle-cancelling finish ---
// The engine's finish (ks_engine.hip k_cyc_*) inside the workgroup. The
// phase before the last drains; price refinement from d ≡ 0 then records each
// improved node's parent arc with its least offer (a 64-bit key per node in rl_p,
// free while no sweep runs), and every CYC_EVERY rounds that have not converged the
// parent graph is searched: one word per node packs the node 2^k steps ahead and the
// least id over those steps (pointer doubling in place, in rl_node's slice, free
// likewise — a word is read and
// written whole, so a reader never pairs a new jump with an old minimum); after
// CYC_LOG steps every node a window ahead of another lies on a cycle (marked), and
// each cycle's least id walks it — its arcs residual, every node agreeing on the
// least id (a cycle longer than the window has nodes that disagree), the cost
// negative — and pushes the bottleneck around it. Cycles of the parent graph are
// node-disjoint (one parent per node), so the walkers never share an arc. The
// cycle's nodes rejoin the next round's frontier; the refinement certifies once
// its frontier drains. Giving up (prc_cap rounds) leaves a feasible flow to the
// final phase.

__device__ __forceinline__ void cyc_search(const CellArgs& A, const K& k, int src, int nb) {
    // N words each: jump | least id << CYC_IDB, double-buffered (every step reads the
    // previous step's words only: in place, the jumps of a cycle's nodes can fold onto
    // one node, and a cycle must be every node's destination to be found)
    int* Wb[2] = {A.rl_node + k.x0, A.lists + (size_t)nb * A.nn + k.x0};   // (buffer nb is empty until the next round)
    int* W = Wb[0];
    const unsigned long long* key = reinterpret_cast<const unsigned long long*>(A.rl_p) + k.x0;
    unsigned dbg[4] = {0, 0, 0, 0};
    for (int l = threadIdx.x; l < k.N; l += CT) {
        const int a = key_at(key, l);
        const int j = a >= 0 ? ld_cp(A, k, a).head - k.x0 : l;
        W[l] = j | (l << CYC_IDB);
        dbg[0] += a >= 0;
    }
    __syncthreads();
    const int lg = A.cyc_lg;   // CYC_LOG (a shorter window only under fault_inject bit 7)
    for (int d = 0; d < lg; ++d) {
        const int* Wi = Wb[d & 1];
        int* Wo = Wb[(d & 1) ^ 1];
        for (int l = threadIdx.x; l < k.N; l += CT) {
            const int w = Wi[l];
            const int wx = Wi[w & CYC_IDM];   // 2^d steps ahead of l, then 2^d more
            Wo[l] = (wx & CYC_IDM) | (min(w >> CYC_IDB, wx >> CYC_IDB) << CYC_IDB);
        }
        __syncthreads();
    }
    W = Wb[lg & 1];
    for (int l = threadIdx.x; l < k.N; l += CT) {
        const int x = W[l] & CYC_IDM;
        if (key_at(key, x) >= 0 && !(atomicOr(&W[x], CYC_ON) & CYC_ON)) ++dbg[1];
    }
    __syncthreads();
    // A leader's walk is the whole check: a marked node whose window minimum is itself
    // but which lies on a chain (longer than the window) walks up into a cycle and never
    // returns to itself, so nothing is pushed (counted in rejected)
    int found = 0, rejected = 0;
    for (int l = threadIdx.x; l < k.N; l += CT) {
        const int w = W[l];
        if (!(w & CYC_ON) || ((w & ~CYC_ON) >> CYC_IDB) != l) continue;
        ++dbg[2];
        long long cost = 0;
        int cap = 0x7fffffff, x = l;
        bool ok = false;
        for (int st = 0; st < CYC_WALK; ++st) {
            const int a = key_at(key, x);
            if (a < 0) break;
            const Pos q = ld_cp(A, k, a);
            const int wx = W[x];
            if (q.rcap <= 0 || !(wx & CYC_ON) || ((wx & ~CYC_ON) >> CYC_IDB) != l) break;
            cost += q.cost;
            cap = min(cap, (int)q.rcap);
            x = q.head - k.x0;
            if (x == l) {
                ok = true;
                break;
            }
        }
        dbg[3] += ok;
        rejected += !ok;
        if (!ok || cost >= 0) continue;
        x = l;
        do {
            const int a = key_at(key, x);
            const Pos q = ld_cp(A, k, a);
            st_rcap(A, a, q.rcap - cap);
            st_rcap(A, q.rev, q.ucap - (q.rcap - cap));
            mark(A, k, src, x + k.x0);
            x = q.head - k.x0;
        } while (x != l);
        ++found;
    }
    if (found) atomicAdd(&c_.cycles, found);
    if (rejected) atomicAdd(&c_.rejected, rejected);
    for (int i = 0; i < 4; ++i)
        if (dbg[i]) atomicAdd(&c_.cyc_dbg[i], dbg[i]);
}

__global__ __launch_bounds__(CT) void k_cell(CellArgs A) {
    const CellDesc cd = A.cells[blockIdx.x];
    const int N = cd.cb[CELL_NCLS] - cd.cb[0];
    const int pb = A.first[cd.cb[0]];
    if (threadIdx.x < 8) s_.cbs[threadIdx.x] = A.cells[blockIdx.x].cb[threadIdx.x];
    if (threadIdx.x < NCTR) ctr_[threadIdx.x] = 0;
    if (*A.bad) {   // a position the compact record cannot hold: nothing is touched
        if (threadIdx.x == 0) {
            CellOut o{};
            o.status = CS_RANGE;
            A.out[blockIdx.x] = o;
        }
        return;
    }
    if (threadIdx.x == 0) {
        s_.rl_cnt[0] = s_.rl_cnt[1] = 0;
        s_.flag = 0;
        s_.stop = 0;
        s_.next = 0;
        s_.bnd = DINF;
        s_.nbx = 0;
        Ctl& c = c_;
        c = Ctl{};
        c.t0 = __builtin_amdgcn_s_memrealtime();
        c.t_op = c.t0;
        c.t_phase = c.t0;
        t_items_ = 0;
        t_first_ = ~0ULL;
        for (int i = 0; i < 32; ++i) {
            (&cls_t_[0][0])[i] = 0;
            (&cls_n_[0][0])[i] = 0;
        }
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
        k.pb = pb;
        k.c1 = cd.cb[1];
        k.c2 = cd.cb[2];
        k.c3 = cd.cb[3];
        k.c4 = cd.cb[4];
        k.c5 = cd.cb[5];
        k.c6 = cd.cb[6];
        k.eps = c_.eps;
        k.eps_shift = (k.eps & (k.eps - 1)) == 0 ? __builtin_ctzll((unsigned long long)k.eps) : -1;
        k.sp = c_.sp;
        k.bnd = s_.bnd;
        k.prc = c_.prc;
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
                if (c_.prc)   // no parents yet
                    for (int l = threadIdx.x; l < N; l += CT)
                        reinterpret_cast<unsigned long long*>(A.rl_p)[k.x0 + l] = PKEY_NONE;
                if (threadIdx.x == 0) s_.flag &= ~F_NEG;
                break;
            }
            case O_PR:
                step<OP_PR>(A, k, src, nb, 0);
                break;
            case O_CYC:
                cyc_search(A, k, src, nb);
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
        if (op == O_BF) {
            step_post<OP_BF>(A, k, src);
            gu_bound(k);
        }
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
        o.cycles = c.cycles;
        o.searches = c.searches;
        o.rejected = c.rejected;
        for (int i = 0; i < 4; ++i) o.cyc_dbg[i] = c.cyc_dbg[i];
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
            o.item_ticks[i] = c.item_ticks[i];
            o.first_ticks[i] = c.first_ticks[i];
        }
        for (int i = 0; i < 32; ++i) {
            o.cls_ticks[i] = (&cls_t_[0][0])[i];
            o.cls_n[i] = (&cls_n_[0][0])[i];
        }
        for (int i = 0; i < 12; ++i) {
            o.hist_t[i] = c.hist_t[i];
            o.hist_n[i] = c.hist_n[i];
        }
        for (int i = 0; i < 8; ++i) o.phase_ticks[i] = c.phase_ticks[i];
        A.out[blockIdx.x] = o;
    }
}

// Grid-wide, before the cell launch: every position's compact record. The head's
// cell (a binary search over the cells' first ids) gives the local head index and
// the base of the reverse's offset. A value the record cannot hold flags *bad, and
// the cells then return CS_RANGE without touching anything (the host falls back
// to the multi-kernel engine).
__global__ void k_cell_pack(CellArgs A, int* bad) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < A.m2; p += (long long)gridDim.x * blockDim.x) {
        const Pos q = ld_pos(A.pos + p);
        int lo = 0, hi = A.ncells;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (A.cells[mid].cb[0] <= q.head) lo = mid;
            else hi = mid;
        }
        const int x0 = A.cells[lo].cb[0];
        const long long pb = A.first[x0];
        CellPos c;
        const bool dead = q.cost >= DEAD_SCALED;
        const long long cs = dead ? 0 : q.cost;   // scaled: the decode needs no multiply
        const long long hl = q.head - x0, rr = q.rev - pb;
        if (q.ucap > CELL_MAX_CAP || q.rcap > CELL_MAX_CAP || cs > CELL_MAX_COST || cs < -CELL_MAX_COST ||
            hl >= (1LL << CELL_HEAD_BITS) || rr < 0 || rr >= CELL_MAX_POS)
            atomicOr(bad, 1);
        c.rcap = (int)q.rcap;
        c.ucap = (int)q.ucap;
        c.cost = dead ? CELL_DEAD : (int)cs;
        c.hr = (unsigned)hl | ((unsigned)rr << CELL_HEAD_BITS);
        A.cp[p] = c;
    }
}

// After the cell launch: the residuals back into the engine's positions.
__global__ void k_cell_unpack(CellArgs A, const int* bad) {
    if (*bad) return;
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < A.m2; p += (long long)gridDim.x * blockDim.x)
        A.pos[p].rcap = A.cp[p].rcap;
}

}  // namespace

size_t cell_lds_bytes(int n, size_t limit) {
    if (n < 0) return 0;
    const size_t w = ((size_t)n + 31) / 32;
    // prices 8n, distances 4n rounded up to whole 8-byte words, two bitmaps
    const size_t b = 8 * (size_t)n + 8 * (((size_t)n + 1) / 2) + 2 * 4 * w;
    const size_t dyn = (b + 15) / 16 * 16;
    return dyn + sizeof(St) + sizeof(Ctl) + 64 + sizeof(cls_t_) + sizeof(cls_n_) <= limit ? dyn : 0;
}

int cell_max_nodes(size_t limit) {
    int lo = 0, hi = 1 << CELL_HEAD_BITS;   // (the compact record's local head field)
    while (hi - lo > 1) {
        const int mid = (lo + hi) / 2;
        if (cell_lds_bytes(mid, limit)) lo = mid;
        else hi = mid;
    }
    return lo;
}

hipError_t cell_launch(const CellArgs& a, int* bad, size_t lds_limit, hipStream_t st, bool* refused) {
    *refused = false;
    const size_t lds = cell_lds_bytes(a.max_nodes, lds_limit);
    if (!lds || a.ncells <= 0) {
        *refused = true;
        return hipErrorInvalidValue;
    }
    // (per device and cheap: set on every launch)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cell),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) {
        *refused = e == hipErrorInvalidValue;   // the device will not give k_cell that much LDS
        return e;
    }
    if ((e = hipMemsetAsync(bad, 0, sizeof(int), st)) != hipSuccess) return e;
    const int pg = (int)std::min<long long>(4096, (a.m2 + 255) / 256 > 0 ? (a.m2 + 255) / 256 : 1);
    hipLaunchKernelGGL(k_cell_pack, dim3(pg), dim3(256), 0, st, a, bad);
    CellArgs b = a;
    b.bad = bad;
    hipLaunchKernelGGL(k_cell, dim3(a.ncells), dim3(CT), lds, st, b);
    hipLaunchKernelGGL(k_cell_unpack, dim3(pg), dim3(256), 0, st, a, (const int*)bad);
    return hipGetLastError();
}

}  // namespace ks
