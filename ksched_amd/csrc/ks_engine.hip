// ks_engine.hip — gfx950 ε-scaling push-relabel min-cost flow engine.
//
// Replaces the Flowlessly solve behind ksched's placement.Solver
// (scheduling/flow/placement/solver.go:30-34, 60-90). Algorithm and data
// layout: DESIGN.md §3-§4. Summary:
//
//   build      Nodes are RENUMBERED internally: classed by residual degree into
//              lane GROUPS of 4/8/16/32/64 lanes per node (one residual arc per
//              lane: a node costs one short dependent chain, not a serial arc
//              loop), each class a contiguous id range padded to whole 64-node
//              blocks, heavy hubs (degree > 4096; cluster aggregator, sink) last.
//              The residual CSR over the new ids comes from a radix sort of the
//              2m (tail, slot) keys (hipcub over rocPRIM). Every arc also keeps
//              its pair capacity ucap = rcap(a) + rcap(rev a), so the reverse
//              residual is ucap − rcap (no gather) and a push is two stores.
//   phases     ε ← ε/α: saturate every residual arc with negative reduced cost,
//              then alternate a GLOBAL PRICE UPDATE (Bellman-Ford from the
//              deficits) with a short burst of push/relabel SWEEPS until no node
//              holds excess. Once ε is below a small fraction of a cost unit the
//              flow is tested by PRICE REFINEMENT at ε = 1 (Bellman-Ford on the
//              difference constraints of 1-optimality); success proves the flow
//              optimal and ends the solve early.
//   finish     (default) the final phase is replaced: the phase before it drains,
//              then the refinement's Bellman-Ford records each node's parent arc
//              (packed keys) and every 8 rounds the parent graph is searched by
//              pointer doubling; its negative cycles are cancelled in parallel
//              until the refinement certifies (k_cyc_*). A near-optimal
//              flow (config 4's churn rounds) takes the finish a phase earlier.
//   layout     the solve's hot kernels read 16-B compact positions (CPos + a
//              reverse array) when the graph's values fit 32 bits (PL<CP>).
//   frontier   sweeps and Bellman-Ford rounds only touch the ACTIVE frontier:
//              one flag byte per node (three rotating buffers) plus per-hub
//              flags. Producers store 1 (idempotent: no counters, no returning
//              atomics); a wave owns a window of one or two lane-group batches,
//              ballots its flags, clears what it reads and hands the active
//              nodes to its groups. Dense passes take every node.
//   sweep      every frontier node discharges once against a price SNAPSHOT
//              (double-buffered prices: read P[ni(q)], write P[ni(q^1)]); a node
//              relabels only if it saturated all of its own admissible arcs, and
//              the relabel also covers arcs that may gain residual capacity from
//              concurrent pushes in the same sweep (reduced cost in (0, ε]) —
//              ε-optimality without locks.
//   control    the host enqueues one CYCLE per round trip: [global-update init]
//              [k Bellman-Ford rounds] [max] [apply] [g sweeps]; kernels read
//              device-side flags and exit early once their stage is finished,
//              so a cycle costs one host synchronisation.
//   heavy hubs pushes into a hub are wave-aggregated into a 16-way sharded
//              inbox; hub chunks claim excess with a CAS and the last-arriving
//              chunk finalises the relabel. Bellman-Ford relaxations into a hub
//              are min-reduced in LDS per workgroup.
//   tail       once an update leaves ≤ 64 nodes with excess, each sends its
//              units down the update's distances (k_augment walks; k_aug_hub
//              hands a hub's excess on in parallel) instead of one hop per
//              sweep over dozens of cycles; the update itself is bounded at the
//              excess nodes' largest distance. In a coarse phase the tail runs
//              FORWARD updates instead (k_fs_*): a search from the excess nodes
//              to the nearest deficit, the successive-shortest-path dual step,
//              and one unit per deficit pushed back along the search's parent
//              arcs — no global recompute.
//   verify     on-device: conservation, capacity, and 1-optimality of the final
//              prices in scaled units (costs × (n+1), so 1-optimal ⇒ optimal);
//              the total cost is reduced in int64.
//
// All in-kernel cross-workgroup communication uses device-scope RMW atomics or
// idempotent flag stores; everything else is handed over at kernel boundaries.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ks_cell.h"
#include "ks_engine.h"
#include "ks_sched.h"

namespace ks {
namespace {

constexpr int BLK = 256;
constexpr int WAVE = 64;
constexpr int WPB = BLK / WAVE;
constexpr int NGC = 6;             // group classes: 4, 8, 16, 32, 64 lanes; 64 lanes × several chunks
constexpr int HEAVY_MIN = 4096;    // degree > 4096: hub, chunked over workgroups
constexpr int CHUNK = 1024;        // heavy hubs: 1024 residual arcs per workgroup
constexpr int PER_T = CHUNK / 256; // arcs per thread in a hub chunk
constexpr int HSPLIT = 4;          // Bellman-Ford: workgroups per hub chunk (one arc per thread at 4)
constexpr int BF_PER_T = PER_T / HSPLIT;
static_assert(PER_T % HSPLIT == 0, "a hub chunk splits into whole arcs per thread");
constexpr int WPW = 2;             // windows per wave in sparse (grid-stride) passes
constexpr int SHARDS = 16;         // inbox shards per heavy hub
constexpr int MAXB = 64;           // max sweeps per cycle
constexpr int HUB_LDS = 16;        // hubs whose Bellman-Ford minima are reduced in LDS
constexpr int CYC_SLOTS = 2;       // control snapshots / timing events rotate over two cycles
constexpr int NCTR = 10;
constexpr int CTR_SHARDS = 64;
constexpr long long INF64 = 0x3fffffffffffffffLL;
constexpr long long LEN_CAP = 1LL << 40;   // global-update arc length clamp
constexpr double kSolveWallLimitS = 120.0; // host-side guard against a non-converging solve
constexpr double kCellLimitS = 20.0;       // the cell solver's in-kernel wall-clock limit (every workgroup exits)

enum { C_SCAN = 0, C_VISIT = 1, C_PUSH = 2, C_RELABEL = 3, C_GUSCAN = 4, C_BFROUND = 5, C_AUGWALK = 6, C_AUGHOP = 7,
       C_FSSCAN = 8, C_GULEAF = 9 };
constexpr int AUG_KMAX = 4096;     // most excess nodes a tail's walkers start from (ks_opts.tail_nodes)
constexpr int BX_CAP = 64;         // global updates with at most this many excess nodes are bounded
// Forward tail update: a node's search key (in its record's dist slot) packs the
// distance from the excess nodes above the position of the arc that set it.
constexpr int FS_PB = 26;
constexpr long long FS_NONE = (1LL << FS_PB) - 1;    // no parent (an excess node)
constexpr long long FS_DMAX = 1LL << 36;             // distances beyond are not searched
constexpr int FDEF_CAP = 64;       // deficits one forward update traces paths to
constexpr int FS_LIST_BLOCKS = 128;
constexpr int FWD_UPD = 4;         // forward updates per cycle once a search finished within its rounds (2: ~1 ms slower on config 4)

struct Ctl {
    long long eps;
    long long gu_L;        // max finite distance of the current global update
    long long gu_X;        // max distance of a node holding excess (−1: none)
    int infeasible;
    int bf_done;           // Bellman-Ford frontier drained (update converged)
    int verify_bad;
    int cp_bad;            // k_pack_pos: a value the 16-B record cannot hold (the solve reads Pos)
    int cyc_done;          // cycle-cancelling refinement: cycles cancelled
    int cyc_rej;           //   marked nodes k_cyc_check found with other than one member pointing at them
    int bf_count;          // Bellman-Ford rounds that did work (whole solve)
    int bfa[3];            // Bellman-Ford flag buffer k holds at least one flag
    int apply_act;         // the global-update apply seeded a non-empty frontier
    int sweep_act[MAXB];   // sweep pos left a non-empty frontier
    int gu_pending;        // the last cycle's update did not converge: the next cycle continues it
    int n_exc;             // nodes the last apply found holding excess
    int bf_r0;             // bf_count when the running update started
    int bf_seq0;           // sequence number of the running update's first (dense) round
    int aug_reached;       // walks of this cycle that reached a deficit / stopped short
    int aug_short;
    int n_xl2;             // nodes fed by this cycle's hub distribution
    int dbg_x[4];          // diagnostics (KS_CYCLE_LOG): the first listed excess nodes, their excess at the apply
    int dbg_e[4];
    int n_bx;              // excess nodes k_gu_init listed for the distance bound (> BX_CAP: no bound)
    long long bf_bound;    // Bellman-Ford prune bound: max tentative distance of the listed excess nodes
    long long gu_B;        // the converged bounded update's cap: max distance of the listed excess nodes
    // forward tail update (k_fs_*): a search from the excess nodes
    long long fs_D;        // least distance of a deficit found by the running search (INF64: none yet)
    int fs_cnt[3];         // frontier list lengths (rotating like the flag buffers)
    int fs_done;           // the search's frontier drained
    int fs_fail;           // list overflow or no deficit in range: the next cycle is a backward update
    int fs_pending;        // a search is running: the next init continues it (set by its first round)
    int fs_rounds;         // rounds of the running search that had a frontier
    int n_fdef;            // deficits at distance D listed for the trace
    int fs_moved;          // units the trace moved
    long long u_exc;       // excess units the last apply (backward) / init (forward) found
    int fs_maxcnt;         // the running search's widest frontier (nodes; hubs count 1024 each)
    int n_exc_rep;         // excess nodes / units the last completed forward update's init found
    long long u_exc_rep;
    int fs_completed;      // forward updates completed (whole solve)
    int fs_moved_cyc;      // units the traces of this cycle moved
    // device-clock timing (s_memrealtime, 100 MHz) where a HIP event between two
    // kernels would cost a ~5.7 µs gap of its own (profiles/r06_*_gaps):
    unsigned long long t_sw0;       // the cycle's first sweep started
    unsigned long long t_end;       // k_cycle_end started (= the last sweep ended)
    unsigned long long t_srch;      // the finish's running parent-graph search started (0: none)
    unsigned long long srch_ticks;  // the finish's searches so far (subtracted from its batches' spans)
};

struct HItem {
    int node, hid, begin, end;
};

__host__ __device__ constexpr int class_lanes(int c) { return c < 4 ? (4 << c) : 64; }
__host__ __device__ inline int degree_class(int d) {
    return d <= 4 ? 0 : d <= 8 ? 1 : d <= 16 ? 2 : d <= 32 ? 3 : d <= 64 ? 4 : d <= HEAVY_MIN ? 5 : NGC;
}
constexpr int CCLS = 5;            // chunked class: Bellman-Ford splits its nodes into 64-arc waves

struct CItem {                     // one 64-arc chunk of a chunked-class node
    int node, begin, end, lead;    // lead = 1 for the node's first chunk
};
// A wave owns one window: win_batches(c) batches of 64/G consecutive node ids.
// classes below 4 (≤ 16 lanes per node) own two batches per window, the rest one
__host__ __device__ constexpr int win_batches(int c) { return c < 4 ? 2 : 1; }
static_assert(NGC == 6, "KS_BY_CLASS dispatches six classes");
__host__ __device__ constexpr int win_slots(int c) { return win_batches(c) * (64 / class_lanes(c)); }

// One frontier buffer: a flag byte per (non-hub) node, a flag per hub.
struct Front {
    unsigned char* flag;   // [hub_base]
    int* hub;              // [nheavy]
};

struct DG {
    int n;                 // internal node ids: [0, hub_base) grouped nodes, then hubs
    int m;
    int hub_base;
    int expand;            // Bellman-Ford: relax low-degree targets two hops per round
    const int* first;
    Pos* pos;              // residual positions: cost, rcap, ucap = rcap(a) + rcap(rev a), head, rev
    CPos* cp;              // compact solve: 16-B copies of the positions (nullptr: the solve reads pos)
    int* crev;             // compact solve: reverse position of each position
    long long* excess;
    long long* p0;         // node records (stride 4, index with ni()): p0 at +0, dist at +1, p1 at +2
    long long* p1;
    long long* dist;
    long long* inbox;
    int wbeg[NGC + 1];     // windows of class c: [wbeg[c], wbeg[c+1])
    int obeg[NGC + 1];     // first node id of class c
    int oend[NGC];         // one past the last real node of class c
    const HItem* hitems;
    int nhitems;
    int nheavy;
    const CItem* citems;   // chunks of the chunked class
    int ncitems;
    int ncls_c;            // nodes of the chunked class
    int sw_clsb;           // sweep blocks striding the class windows (after the hub blocks)
    const int* hnchunks;
    int* xl;               // excess nodes listed by the last apply (the first aug_k)
    int aug_k;             // a phase's tail: ≤ aug_k excess nodes (ks_opts.tail_nodes)
    int* xl2;              // nodes fed by k_aug_hub (the first AUG_K2)
    int* bx;               // excess nodes of the running update (the first BX_CAP; k_gu_init)
    int* fl;               // forward search: 3 rotating frontier lists of fl_cap node ids
    int fl_cap;
    int fs_wide;           // a forward frontier wider than this fails its search as wide
    int npos;              // residual positions (m2cap)
    int* fdef;             // forward search: deficits at the found distance (FDEF_CAP)
    int bound;             // 1: prune Bellman-Ford offers at ctl->bf_bound (ks_opts.bf_bound >= 0)
    long long* aug_req;    // per hub: excess claimed by its k_aug_hub chunks
    long long* q_req;      // claim slots: hubs [0, nheavy), then chunked nodes
    long long* q_taken;
    long long* q_min;
    int* q_unsat;
    int* q_arrive;
    Front sf[3];   // sweep frontiers
    Front bf[3];   // Bellman-Ford frontiers
    Ctl* ctl;
    unsigned long long* ctr;
};

// Node records: p0, dist, p1 and the node's segment bounds (first[x], first[x+1]
// packed) share one 32-B record, so a Bellman-Ford tail gather (price, distance,
// and a leaf's segment) or a sweep's node load (price, segment) is one cache line.
__host__ __device__ __forceinline__ size_t ni(long long x) { return 4 * (size_t)x; }
constexpr int ND_SEG = 3;   // record slot of the packed segment bounds

__device__ __forceinline__ void seg_of(const long long* nd, int x, int& b0, int& b1) {
    const unsigned long long w = (unsigned long long)nd[ni(x) + ND_SEG];
    b0 = (int)(unsigned)(w & 0xffffffffULL);
    b1 = (int)(unsigned)(w >> 32);
}

// ---------------------------------------------------------------- atomics ---
__device__ __forceinline__ void atom_add(long long* p, long long v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long atom_add_ret(long long* p, long long v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long atom_exch(long long* p, long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int atom_exch_i(int* p, int v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long atom_min_ret(long long* p, long long v) {
    return __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void atom_min(long long* p, long long v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// excess and dist are only ever changed by atomics (performed beyond the issuing
// XCD's L2). Every load of them that hands data across workgroups or kernels is
// an agent-scope load: a plain load can hit a stale copy in another XCD's L2
// when a node's owner moves to a different XCD between launches (observed when
// several solves share the GPU: over-pushes, lost distance updates).
__device__ __forceinline__ long long atom_load(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int atom_load_i(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One residual position (ks_pos.h) in two 16-byte loads issued together.
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

// Position access of the solve's hot kernels, by record layout:
// PL<false> reads the 32-B Pos records, PL<true> the 16-B CPos copies (32-bit
// residual, pair capacity, scaled cost, head) plus the separate reverse array.
// Every hot kernel is instantiated for both; the host launches the compact one when
// the graph's scaled costs and capacities fit 32 bits (ks_opts.compact_pos).
template <bool CP>
struct PL;
template <>
struct PL<false> {
    static __device__ __forceinline__ Pos ld(const DG& g, int a) { return ld_pos(g.pos + a); }
    // the record without its reverse position (Bellman-Ford): the same loads here
    static __device__ __forceinline__ Pos ld_nr(const DG& g, int a) { return ld_pos(g.pos + a); }
    static __device__ __forceinline__ void set_rc(const DG& g, int a, long long v) { g.pos[a].rcap = v; }
    static __device__ __forceinline__ long long rc_atomic(const DG& g, int a) { return atom_load(&g.pos[a].rcap); }
    static __device__ __forceinline__ bool cas_rc(const DG& g, int a, long long& exp, long long v) {
        return __hip_atomic_compare_exchange_strong(&g.pos[a].rcap, &exp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    }
    static __device__ __forceinline__ void add_rc(const DG& g, int a, long long v) { atom_add(&g.pos[a].rcap, v); }
    static __device__ __forceinline__ int head(const DG& g, int a) { return g.pos[a].head; }
    static __device__ __forceinline__ int rev(const DG& g, int a) { return g.pos[a].rev; }
};
template <>
struct PL<true> {
    static __device__ __forceinline__ Pos ld(const DG& g, int a) {
        const int4 w = reinterpret_cast<const int4*>(g.cp)[a];
        const int rv = g.crev[a];   // issued with the record (independent address)
        Pos r;
        r.rcap = w.x;
        r.ucap = w.y;
        r.cost = w.z;   // CPOS_DEAD for inert positions: never residual, reduced cost > ε
        r.head = w.w;
        r.rev = rv;
        return r;
    }
    static __device__ __forceinline__ Pos ld_nr(const DG& g, int a) {
        const int4 w = reinterpret_cast<const int4*>(g.cp)[a];
        Pos r;
        r.rcap = w.x;
        r.ucap = w.y;
        r.cost = w.z;
        r.head = w.w;
        r.rev = -1;
        return r;
    }
    static __device__ __forceinline__ void set_rc(const DG& g, int a, long long v) { g.cp[a].rcap = (int)v; }
    static __device__ __forceinline__ long long rc_atomic(const DG& g, int a) {
        return __hip_atomic_load(&g.cp[a].rcap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    static __device__ __forceinline__ bool cas_rc(const DG& g, int a, long long& exp, long long v) {
        int e = (int)exp;
        const bool ok = __hip_atomic_compare_exchange_strong(&g.cp[a].rcap, &e, (int)v, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        exp = e;
        return ok;
    }
    static __device__ __forceinline__ void add_rc(const DG& g, int a, long long v) {
        __hip_atomic_fetch_add(&g.cp[a].rcap, (int)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    static __device__ __forceinline__ int head(const DG& g, int a) { return g.cp[a].head; }
    static __device__ __forceinline__ int rev(const DG& g, int a) { return g.crev[a]; }
};

// ------------------------------------------------------------ wave helpers ---
__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }
__device__ __forceinline__ long long wave_sum(long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ long long wave_min(long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, (long long)__shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ long long wave_max(long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (long long)__shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ long long wave_incl_scan(long long x, int lane) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}
// Lane-group (G lanes, aligned) collectives.
template <int G>
__device__ __forceinline__ long long g_incl_scan(long long x) {
    const int l = lane_id() & (G - 1);
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        long long y = __shfl_up(x, o, G);
        if (l >= o) x += y;
    }
    return x;
}
template <int G>
__device__ __forceinline__ long long g_min(long long x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x = min(x, (long long)__shfl_xor(x, o, G));
    return x;
}
template <int G>
__device__ __forceinline__ long long g_sum(long long x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, G);
    return x;
}
__device__ __forceinline__ long long floordiv(long long a, long long b) {  // b > 0
    long long q = a / b;
    if ((a % b) != 0 && a < 0) --q;
    return q;
}

// Mark node w active in frontier f (idempotent plain stores).
__device__ __forceinline__ void mark(const DG& g, const Front& f, int w, int& out) {
    if (w >= g.hub_base) f.hub[w - g.hub_base] = 1;
    else f.flag[w] = 1;
    out = 1;
}

// Per-lane pending hub push: wave-aggregated into the hub's sharded inbox.
struct Pend {
    int key;
    long long val;
};

struct Cnt {
    long long scan = 0, visit = 0, push = 0, relabel = 0;
};

__device__ __forceinline__ void flush_counters(const DG& g, const Cnt& c) {
    const long long s = wave_sum(c.scan), v = wave_sum(c.visit), p = wave_sum(c.push),
                    r = wave_sum(c.relabel);
    if (lane_id() == 0 && (s | v | p | r)) {
        const int sh = ((blockIdx.x * WPB) + (threadIdx.x >> 6)) & (CTR_SHARDS - 1);
        unsigned long long* c0 = g.ctr + sh * NCTR;
        if (s) atomicAdd(c0 + C_SCAN, (unsigned long long)s);
        if (v) atomicAdd(c0 + C_VISIT, (unsigned long long)v);
        if (p) atomicAdd(c0 + C_PUSH, (unsigned long long)p);
        if (r) atomicAdd(c0 + C_RELABEL, (unsigned long long)r);
    }
}

// Push d units along arc a (v → w): residuals are two plain stores (only v's
// discharge writes the pair this sweep), the excess a fire-and-forget atomic.
// Non-hub heads are marked in nf (when given); hub pushes are buffered in pd
// and flagged once per wave in flush_pending.
// rv / uc: the arc's reverse position and pair capacity when the caller loaded
// them with the arc (rv < 0: load them here, one more dependent step).
template <bool CP>
__device__ __forceinline__ void push_arc(const DG& g, const Front* nf, int a, int w, long long r, long long d,
                                         Pend& pd, int& out, int rv, long long uc) {
    PL<CP>::set_rc(g, a, r - d);
    PL<CP>::set_rc(g, rv, uc - (r - d));
    if (w < g.hub_base) {
        atom_add(&g.excess[w], d);
        if (nf) {
            nf->flag[w] = 1;
            out = 1;
        }
        return;
    }
    const int h = w - g.hub_base;
    if (pd.key == h) {
        pd.val += d;
    } else if (pd.key < 0) {
        pd.key = h;
        pd.val = d;
    } else {
        atom_add(&g.inbox[h * SHARDS + (blockIdx.x & (SHARDS - 1))], d);
        if (nf) {
            nf->hub[h] = 1;
            out = 1;
        }
    }
}

// Must be called by all 64 lanes of a wave at a converged point.
__device__ __forceinline__ void flush_pending(const DG& g, const Front* nf, Pend& pd, int& out) {
    const int lane = lane_id();
    for (;;) {
        const unsigned long long msk = __ballot(pd.key >= 0);
        if (!msk) break;
        const int leader = __ffsll((long long)msk) - 1;
        const int k = __shfl(pd.key, leader);
        const long long s = wave_sum(pd.key == k ? pd.val : 0);
        if (lane == leader) {
            atom_add(&g.inbox[k * SHARDS + (blockIdx.x & (SHARDS - 1))], s);
            if (nf) {
                nf->hub[k] = 1;
                out = 1;
            }
        }
        if (pd.key == k) pd.key = -1;
    }
}

// Drain a hub's inbox shards into its excess. Returns the drained amount.
__device__ __forceinline__ long long drain_inbox(const DG& g, int h) {
    long long s = 0;
#pragma unroll
    for (int k = 0; k < SHARDS; ++k) s += atom_exch(&g.inbox[h * SHARDS + k], 0LL);
    if (s) atom_add(&g.excess[g.hub_base + h], s);
    return s;
}

// ------------------------------------------------------------ block helpers ---
__device__ __forceinline__ long long block_sum(long long x, long long* sh) {
    x = wave_sum(x);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 0) sh[w] = x;
    __syncthreads();
    long long t = 0;
#pragma unroll
    for (int i = 0; i < WPB; ++i) t += sh[i];
    return t;
}
__device__ __forceinline__ long long block_min(long long x, long long* sh) {
    x = wave_min(x);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 0) sh[w] = x;
    __syncthreads();
    long long t = INF64;
#pragma unroll
    for (int i = 0; i < WPB; ++i) t = min(t, sh[i]);
    return t;
}
// exclusive scan across the block; returns exclusive prefix, *total = block total
__device__ __forceinline__ long long block_excl_scan(long long x, long long* sh, long long* total) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const long long incl = wave_incl_scan(x, lane);
    __syncthreads();
    if (lane == WAVE - 1) sh[w] = incl;
    __syncthreads();
    long long off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < WPB; ++i) {
        if (i < w) off += sh[i];
        tot += sh[i];
    }
    *total = tot;
    return off + incl - x;
}

// --------------------------------------------------- frontier traversal ---
// A wave owns one window of class C. It ballots the window's flags (clearing
// what it reads; dense passes take every real node) and hands the active nodes
// to its G-lane groups one batch at a time. The loop trip count is wave-uniform,
// so the group code may use wave collectives.
#define KS_WINDOW(C, ARGS, W, ...)                                                   \
    {                                                                                \
        constexpr int G_ = class_lanes(C);                                           \
        constexpr int PER_ = 64 / G_;                                                \
        constexpr int WS_ = win_slots(C);                                            \
        const int base_ = g.obeg[C] + ((W) - g.wbeg[C]) * WS_;                       \
        const int ln_ = lane_id();                                                   \
        bool on_ = false;                                                            \
        if (ln_ < WS_) {                                                             \
            if ((ARGS).dense) {                                                      \
                on_ = base_ + ln_ < g.oend[C];                                       \
            } else {                                                                 \
                on_ = (ARGS).flags[base_ + ln_] != 0;                                \
                if (on_) (ARGS).flags[base_ + ln_] = 0;                              \
            }                                                                        \
        }                                                                            \
        unsigned long long mask_ = __ballot(on_);                                    \
        const int k_ = ln_ / G_;                                                     \
        while (mask_) {                                                              \
            unsigned long long mm_ = mask_;                                          \
            for (int j_ = 0; j_ < k_; ++j_) mm_ &= mm_ - 1;                          \
            const int v = mm_ ? base_ + __ffsll((long long)mm_) - 1 : -1;            \
            __VA_ARGS__;                                                             \
            for (int j_ = 0; j_ < PER_; ++j_) mask_ &= mask_ - 1;                    \
        }                                                                            \
    }
// Dispatch on the (wave-uniform) class of window IDX.
#define KS_BY_CLASS(IDX, ARGS, CALLT)                                                \
    {                                                                                \
        const int i_ = (IDX);                                                        \
        if (i_ < g.wbeg[1]) KS_WINDOW(0, ARGS, i_, CALLT(0))                         \
        else if (i_ < g.wbeg[2]) KS_WINDOW(1, ARGS, i_, CALLT(1))                    \
        else if (i_ < g.wbeg[3]) KS_WINDOW(2, ARGS, i_, CALLT(2))                    \
        else if (i_ < g.wbeg[4]) KS_WINDOW(3, ARGS, i_, CALLT(3))                    \
        else if (i_ < g.wbeg[5]) KS_WINDOW(4, ARGS, i_, CALLT(4))                    \
        else if (i_ < g.wbeg[6]) KS_WINDOW(5, ARGS, i_, CALLT(5))                    \
    }
struct Scan {
    unsigned char* flags;   // frontier flags to consume (sparse pass)
    int dense;              // 1: every node, flags ignored
};

__device__ __forceinline__ int wave_index_in_grid(int first_block) {
    return ((int)blockIdx.x - first_block) * WPB + ((int)threadIdx.x >> 6);
}

// ===================================================================== build ===
// The residual CSR is built on device from the arc table of the store
// (ks_store.h). Every node owns a segment of CAPACITY positions: its live arcs
// (forward arcs and reverses of its in-arcs), plus slack once the graph is
// edited incrementally, so later inserts land in place. Internal ids group the
// nodes by the degree class of their capacity, hubs last; dead positions are
// inert (no capacity, head = owner, cost DEAD_COST).
__global__ void k_degree(int hi, const unsigned char* __restrict__ alive, const int* __restrict__ src,
                         const int* __restrict__ dst, int* __restrict__ deg) {
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK)
        if (alive[s]) {
            atomicAdd(&deg[src[s]], 1);
            atomicAdd(&deg[dst[s]], 1);
        }
}

// Segment capacity of a node slot. Tight after a load (its degree). Once the
// graph is edited incrementally: tasks (≤ 8 arcs: preferences, or one running
// arc after the pin) one 8-lane group — a removed task's segment is reused
// whole by the task that takes over its id (flowgraph/graph.go:169-182), and
// so are dead and spare slots; other nodes their degree +50 % (at least 4)
// rounded up to a lane group (≤ 64) or a 64-arc chunk, never less than what
// they had before (hint) unless that is 4× their need — an aggregator whose
// degree fell after the pins keeps room for the next arrivals — and twice that
// when an insert overflowed them since the last build.
__host__ __device__ inline int seg_capacity(int deg, bool alive, bool task, int slack) {
    if (!slack) return deg;
    if ((!alive || task) && deg <= 8) return 8;
    const int c = deg + (deg / 2 > 4 ? deg / 2 : 4);
    if (c <= 64) {
        int g = 4;
        while (g < c) g <<= 1;
        return g;
    }
    return (c + 63) / 64 * 64;
}

__global__ void k_capacity(int ncap, int nstore, const int* __restrict__ deg, const unsigned char* __restrict__ alive,
                           const unsigned char* __restrict__ type, int slack, int* __restrict__ hint,
                           unsigned char* __restrict__ grow, int* __restrict__ capv, unsigned char* __restrict__ cls) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        const int d = v < nstore ? deg[v] : 0;
        const bool a = v < nstore && alive[v];
        int c = seg_capacity(d, a, a && type[v] == KS_NODE_TASK, slack);
        if (slack && v < nstore) {
            const int h = hint[v];
            if (grow[v]) c = max(c, 2 * max(h, 4));
            else if (h <= 4 * c) c = max(c, h);
            else c = max(c, h / 2);
            if (c > 64) c = (c + 63) / 64 * 64;
            grow[v] = 0;
        }
        if (v < nstore) hint[v] = c;
        capv[v] = c;
        cls[v] = (unsigned char)degree_class(c);
    }
}

// perm[list[i]] = base + i (one class, or the hubs).
__global__ void k_make_perm(int cnt, int base, const int* __restrict__ list, int* __restrict__ perm) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < cnt; i += (long long)gridDim.x * BLK)
        perm[list[i]] = base + (int)i;
}

__global__ void k_capi(int ncap, const int* __restrict__ perm, const int* __restrict__ capv, int* __restrict__ capi,
                       int* __restrict__ iperm) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        capi[perm[v]] = capv[v];
        iperm[perm[v]] = (int)v;
    }
}

// Sort keys: the tail (internal id) of every residual arc; dead slots sort last.
__global__ void k_pos_keys(int hi, int sentinel, const unsigned char* __restrict__ alive, const int* __restrict__ src,
                           const int* __restrict__ dst, const int* __restrict__ perm, unsigned* __restrict__ keys,
                           int* __restrict__ vals) {
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK) {
        const bool a = alive[s];
        keys[2 * s] = a ? (unsigned)perm[src[s]] : (unsigned)sentinel;
        keys[2 * s + 1] = a ? (unsigned)perm[dst[s]] : (unsigned)sentinel;
        vals[2 * s] = (int)(2 * s);
        vals[2 * s + 1] = (int)(2 * s + 1);
    }
}

// rs[v] = lower bound of v in the sorted keys, v ∈ [0, nn].
__global__ void k_first(int nn, long long m2, const unsigned* __restrict__ keys, int* __restrict__ rs) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v <= nn; v += (long long)gridDim.x * BLK) {
        long long lo = 0, hi = m2;
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (keys[mid] < (unsigned)v) lo = mid + 1; else hi = mid;
        }
        rs[v] = (int)lo;
    }
}

// Every position inert, owned by the node whose segment holds it.
__global__ void k_inert_all(long long m2cap, int nn, const int* __restrict__ first, Pos* __restrict__ pos,
                            int* __restrict__ ent) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2cap; p += (long long)gridDim.x * BLK) {
        int lo = 0, hi = nn;   // owner: the last v with first[v] <= p
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (first[mid] <= p) lo = mid; else hi = mid;
        }
        pos[p] = Pos{DEAD_COST, 0, 0, lo, (int)p};
        ent[p] = -1;
    }
}

__global__ void k_fill_csr(long long m2, int nn, const unsigned* __restrict__ keys, const int* __restrict__ vals,
                           const int* __restrict__ rs, const int* __restrict__ first, const int* __restrict__ perm,
                           const int* __restrict__ src, const int* __restrict__ dst, const long long* __restrict__ low,
                           const long long* __restrict__ cap, const long long* __restrict__ cost, long long mult,
                           Pos* __restrict__ pos, int* __restrict__ ent, int* __restrict__ fwd,
                           int* __restrict__ pos_of) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < m2; i += (long long)gridDim.x * BLK) {
        const int v = (int)keys[i];
        if (v >= nn) continue;
        const int p = first[v] + (int)(i - rs[v]);
        const int val = vals[i];
        const int s = val >> 1;
        const bool r = val & 1;
        pos_of[val] = p;
        const long long u = cap[s] - low[s];
        pos[p].head = perm[r ? src[s] : dst[s]];
        pos[p].rcap = r ? 0 : u;
        pos[p].ucap = u;
        pos[p].cost = (r ? -cost[s] : cost[s]) * mult;
        ent[p] = val;
        if (!r) fwd[s] = p;
    }
}

__global__ void k_fill_rev(long long m2, int nn, const unsigned* __restrict__ keys, const int* __restrict__ vals,
                           const int* __restrict__ pos_of, Pos* __restrict__ pos) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < m2; i += (long long)gridDim.x * BLK) {
        if ((int)keys[i] >= nn) continue;
        const int val = vals[i];
        pos[pos_of[val]].rev = pos_of[val ^ 1];
    }
}

__global__ void k_used(int nn, const int* __restrict__ rs, int* __restrict__ used) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < nn; v += (long long)gridDim.x * BLK)
        used[v] = rs[v + 1] - rs[v];
}

// ------------------------------------------------------------ cold reset ---
// Zero flow: forward residual = u, reverse 0; excess = supply with the
// lower-bound transform; prices 0. Runs before every cold solve (no rebuild).
__global__ void k_reset_pos(long long m2cap, const int* __restrict__ ent, Pos* __restrict__ pos) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2cap; p += (long long)gridDim.x * BLK) {
        const int e = ent[p];
        if (e >= 0) pos[p].rcap = (e & 1) ? 0 : pos[p].ucap;
    }
}

// Segment bounds into the node records (the CSR's first[] is fixed per build).
__global__ void k_node_bounds(int nn, const int* __restrict__ first, long long* __restrict__ nd) {
    for (long long x = blockIdx.x * (long long)BLK + threadIdx.x; x < nn; x += (long long)gridDim.x * BLK)
        nd[ni(x) + ND_SEG] = (long long)(((unsigned long long)(unsigned)first[x + 1] << 32) | (unsigned)first[x]);
}

__global__ void k_reset_nodes(int nn, int ncap, const int* __restrict__ iperm, const unsigned char* __restrict__ alive,
                              const long long* __restrict__ supply, long long* __restrict__ excess,
                              long long* __restrict__ p0, long long* __restrict__ p1) {
    for (long long x = blockIdx.x * (long long)BLK + threadIdx.x; x < nn; x += (long long)gridDim.x * BLK) {
        const int v = iperm[x];
        excess[x] = (v >= 0 && v < ncap && alive[v]) ? supply[v] : 0;
        p0[ni(x)] = 0;
        p1[ni(x)] = 0;
    }
}

__global__ void k_reset_low(int hi, const unsigned char* __restrict__ alive, const int* __restrict__ src,
                            const int* __restrict__ dst, const int* __restrict__ perm,
                            const long long* __restrict__ low, long long* __restrict__ excess) {
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK) {
        const long long l = low[s];
        if (alive[s] && l) {
            atom_add(&excess[perm[src[s]]], -l);
            atom_add(&excess[perm[dst[s]]], l);
        }
    }
}

// max |cost| over live arcs → *out (the first phase's ε).
__global__ void k_max_cost(int hi, const unsigned char* __restrict__ alive, const long long* __restrict__ cost,
                           long long* __restrict__ out) {
    long long mx = 0;
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK)
        if (alive[s]) mx = max(mx, cost[s] < 0 ? -cost[s] : cost[s]);
    // one atomic per workgroup (per-wave atomics on one address serialise)
    __shared__ long long sh[WPB];
    mx = wave_max(mx);
    if (lane_id() == 0) sh[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < WPB; ++i) mx = max(mx, sh[i]);
        if (mx) __hip_atomic_fetch_max(out, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The compact solve (ks_opts.compact_pos): every position's 16-B copy
// and its reverse before the phases; a value a 32-bit field cannot hold sets *bad
// and the solve reads the 32-B records instead. The residuals go back before
// verification (k_unpack_pos).
__global__ void k_pack_pos(long long m2, const Pos* __restrict__ pos, CPos* __restrict__ cp, int* __restrict__ crev,
                           int* __restrict__ bad) {
    int b = 0;
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK) {
        const Pos q = ld_pos(pos + p);
        const bool dead = q.cost >= DEAD_COST;
        b |= (!dead && (q.cost > CPOS_MAX || q.cost < -CPOS_MAX)) || q.rcap < 0 || q.rcap > CPOS_MAX || q.ucap < 0 ||
             q.ucap > CPOS_MAX;
        int4 w;
        w.x = (int)q.rcap;
        w.y = (int)q.ucap;
        w.z = dead ? CPOS_DEAD : (int)q.cost;
        w.w = q.head;
        reinterpret_cast<int4*>(cp)[p] = w;
        crev[p] = q.rev;
    }
    if (__any(b) && lane_id() == 0) atomicOr(bad, 1);
}
__global__ void k_unpack_pos(long long m2, const CPos* __restrict__ cp, Pos* __restrict__ pos) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK)
        pos[p].rcap = cp[p].rcap;
}

struct ClassIs {
    const unsigned char* cls;
    unsigned char c;
    __host__ __device__ bool operator()(const int& v) const { return cls[v] == c; }
};

// ================================================= saturate (phase start) ===
// Push the full residual capacity of every arc with negative reduced cost
// (Goldberg's refine start) over the whole graph; reads the authoritative p0.
template <int G, bool CP>
__device__ __forceinline__ void sat_group(const DG& g, int v, long long thr, Pend& pd, int& out, Cnt& c) {
    const long long* P = g.p0;
    const int lig = lane_id() & (G - 1);
    int b0 = 0, en = 0;
    long long pv = 0;
    if (v >= 0) {
        seg_of(g.p0, v, b0, en);
        pv = P[ni(v)];
    }
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;   // G == 64: one node per wave
    long long tot = 0;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        if (a < en) {
            const Pos q = PL<CP>::ld(g, a);
            const long long r = q.rcap;
            if (r > 0) {
                const int w = q.head;
                if (q.cost + pv - P[ni(w)] < -thr) {
                    push_arc<CP>(g, nullptr, a, w, r, r, pd, out, q.rev, q.ucap);
                    tot += r;
                    c.push++;
                }
            }
        }
        flush_pending(g, nullptr, pd, out);
    }
    tot = g_sum<G>(tot);
    if (v >= 0 && lig == 0 && tot) atom_add(&g.excess[v], -tot);
}

// thr = 0: Goldberg's refine start (every negative reduced cost); thr = ε on a
// warm start: only arcs that violate ε-optimality are saturated.
template <bool CP>
__global__ __launch_bounds__(BLK) void k_saturate(DG g, long long thr) {
    const long long* P = g.p0;
    Pend pd{-1, 0};
    Cnt c;
    int out = 0;
    if ((int)blockIdx.x < g.nhitems) {
        __shared__ long long sh[WPB];
        const HItem it = g.hitems[blockIdx.x];
        const long long px = P[ni(it.node)];
        long long tot = 0;
#pragma unroll
        for (int k = 0; k < PER_T; ++k) {
            const int a = it.begin + threadIdx.x * PER_T + k;
            if (a < it.end) {
                const Pos q = PL<CP>::ld(g, a);
                const long long r = q.rcap;
                if (r > 0) {
                    const int w = q.head;
                    if (q.cost + px - P[ni(w)] < -thr) {
                        push_arc<CP>(g, nullptr, a, w, r, r, pd, out, q.rev, q.ucap);
                        tot += r;
                        c.push++;
                    }
                }
            }
        }
        flush_pending(g, nullptr, pd, out);
        tot = block_sum(tot, sh);
        if (threadIdx.x == 0 && tot) atom_add(&g.excess[it.node], -tot);
        flush_counters(g, c);
        return;
    }
    const Scan sc{nullptr, 1};
#define KS_SAT_CALL(C) sat_group<G_, CP>(g, v, thr, pd, out, c)
    KS_BY_CLASS(wave_index_in_grid(g.nhitems), sc, KS_SAT_CALL)
#undef KS_SAT_CALL
    flush_pending(g, nullptr, pd, out);
    flush_counters(g, c);
}

// =================================================== push/relabel sweep ===
// One node per G-lane group, one residual arc per lane; admissible capacity is
// distributed by an in-group prefix sum, the relabel minimum by a group min.
template <int G, bool CP>
__device__ __forceinline__ void sweep_group(const DG& g, const Front& nf, int v, long long e, long long pv, int b0,
                                            int en, long long* __restrict__ PN, const long long* __restrict__ P,
                                            long long eps, Pend& pd, int& out, Cnt& c) {
    const int lig = lane_id() & (G - 1);
    if (v < 0) e = 0;
    const bool act = e > 0;
    if (!act) en = b0;
    if (act && lig == 0) c.visit++;
    long long rem = e, minc = INF64;
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;   // G == 64: one node per wave
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        const bool valid = a < en;
        long long r = 0, cr = 0;
        int w = 0;
        int rv = 0;
        long long uc = 0;
        if (valid) {
            const Pos q = PL<CP>::ld(g, a);   // the whole record: a push needs no further load
            r = q.rcap;
            w = q.head;
            rv = q.rev;
            uc = q.ucap;
            cr = q.cost + pv - P[ni(w)];
            c.scan++;
        }
        const long long adm = (valid && cr < 0 && r > 0) ? r : 0;
        const long long incl = g_incl_scan<G>(adm);
        const long long total = __shfl(incl, G - 1, G);
        long long d = rem - (incl - adm);
        d = d < 0 ? 0 : (d > adm ? adm : d);
        if (d > 0) {
            push_arc<CP>(g, &nf, a, w, r, d, pd, out, rv, uc);
            c.push++;
        }
        if (valid) {
            if (cr < 0) {
                if (r - d > 0) minc = min(minc, cr);
            } else if (r > 0 || cr <= eps) {
                minc = min(minc, cr);
            }
        }
        rem -= total < rem ? total : rem;
        flush_pending(g, &nf, pd, out);
        if (G == 64 && rem == 0) break;
    }
    minc = g_min<G>(minc);
    if (act && lig == 0) {
        const long long pushed = e - rem;
        if (pushed) atom_add(&g.excess[v], -pushed);
        long long np = pv;
        if (rem > 0) {
            if (minc >= INF64) atomicOr(&g.ctl->infeasible, 1);
            else np = pv - (minc + eps);
            c.relabel++;
            nf.flag[v] = 1;   // still active next sweep
            out = 1;
        }
        PN[ni(v)] = np;
    }
}

// -------------------------------------------------- chunked claim protocol ---
// Hubs (one workgroup per 1024-arc chunk) discharge cooperatively. Every chunk reads the node's excess E
// once, requests its admissible capacity Ac with ONE returning atomicAdd on the
// node's request counter (no CAS loop), takes clamp(E − start, 0, Ac), pushes,
// and reports (taken, relabel minimum, unsaturated). The last-arriving chunk
// settles the node: subtracts what was taken, drains the hub inbox, relabels if
// every admissible arc was saturated and excess is left, and marks it active.
// Concurrent inflows only ever add excess, so Σ taken ≤ the excess present.
__device__ __forceinline__ long long claim(const DG& g, int slot, long long E, long long Ac) {
    if (Ac <= 0) return 0;
    const long long start = __hip_atomic_fetch_add(&g.q_req[slot], Ac, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long take = E - start;
    return take < 0 ? 0 : (take > Ac ? Ac : take);
}

// One lane per chunk. Returns nothing; settles the node when it arrives last.
__device__ __forceinline__ void settle(const DG& g, const Front& F, const Front& N, int slot, int x, int nch,
                                       bool hub, long long take, long long Ac, long long minc, long long px,
                                       long long* __restrict__ PN, long long eps, int& out, Cnt& c) {
    if (minc < INF64) atom_min(&g.q_min[slot], minc);
    if (take < Ac) atom_exch_i(&g.q_unsat[slot], 1);
    if (take) atom_add(&g.q_taken[slot], take);
    drain_vm();
    const int old = __hip_atomic_fetch_add(&g.q_arrive[slot], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old != nch - 1) return;
    // every returning atomic of the settle issued together (one round trip), then
    // one fetch-add applies the taken units and the drained inbox
    const long long mn = atom_exch(&g.q_min[slot], INF64);
    const int unsat = atom_exch_i(&g.q_unsat[slot], 0);
    const long long taken = atom_exch(&g.q_taken[slot], 0);
    atom_exch(&g.q_req[slot], 0LL);
    long long inflow = 0;
    if (hub) {
        long long* ib = &g.inbox[(x - g.hub_base) * SHARDS];
#pragma unroll
        for (int k = 0; k < SHARDS; ++k) inflow += atom_exch(&ib[k], 0LL);
    }
    const long long delta = inflow - taken;
    const long long now = (delta ? atom_add_ret(&g.excess[x], delta) : atom_load(&g.excess[x])) + delta;
    long long np = px;
    if (!unsat && now > 0) {
        if (mn >= INF64) atomicOr(&g.ctl->infeasible, hub ? 2 : 4);
        else np = px - (mn + eps);
        c.relabel++;
    }
    c.visit++;
    PN[ni(x)] = np;
    if (now > 0) mark(g, N, x, out);
    if (!hub) F.flag[x] = 0;   // every chunk has read it
    atom_exch_i(&g.q_arrive[slot], 0);
}

// Hub chunk: one workgroup, 1024 arcs (four per thread, loads issued together).
// px, E: the hub's price and excess, loaded by the caller with its flag.
template <bool CP>
__device__ void hub_chunk(const DG& g, const Front& F, const Front& N, const HItem& it, long long px, long long E,
                          const long long* __restrict__ P, long long* __restrict__ PN, long long eps, Pend& pd,
                          int& out, Cnt& c) {
    __shared__ long long sh[WPB];
    __shared__ long long s_take;
    const int x = it.node;
    long long r[PER_T], cr[PER_T], adm[PER_T], uc[PER_T];
    int w[PER_T], rv[PER_T];
    long long mine = 0;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        r[k] = 0;
        w[k] = 0;
        rv[k] = 0;
        uc[k] = 0;
        cr[k] = 0;
        if (a < it.end) {
            const Pos q = PL<CP>::ld(g, a);
            r[k] = q.rcap;
            w[k] = q.head;
            rv[k] = q.rev;
            uc[k] = q.ucap;
            cr[k] = q.cost;   // + px − P[head], below
        }
    }
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        if (a < it.end) {
            cr[k] += px - P[ni(w[k])];
            c.scan++;
        }
        adm[k] = (a < it.end && cr[k] < 0 && r[k] > 0) ? r[k] : 0;
        mine += adm[k];
    }
    long long Ac = 0;
    const long long excl = block_excl_scan(mine, sh, &Ac);
    if (threadIdx.x == 0) s_take = claim(g, it.hid, E, Ac);
    __syncthreads();
    const long long take = s_take;
    long long rt = take - excl;
    rt = rt < 0 ? 0 : (rt > mine ? mine : rt);
    long long minc = INF64;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        const long long d = adm[k] < rt ? adm[k] : rt;
        rt -= d;
        if (d > 0) {
            push_arc<CP>(g, &N, a, w[k], r[k], d, pd, out, rv[k], uc[k]);
            c.push++;
        }
        if (a < it.end) {
            if (cr[k] < 0) {
                if (r[k] - d > 0) minc = min(minc, cr[k]);
            } else if (r[k] > 0 || cr[k] <= eps) {
                minc = min(minc, cr[k]);
            }
        }
    }
    flush_pending(g, &N, pd, out);
    minc = block_min(minc, sh);
    if (threadIdx.x == 0)
        settle(g, F, N, it.hid, x, g.hnchunks[it.hid], true, take, Ac, minc, px, PN, eps, out, c);
}

// Chunked-class discharge: one wave per 64-arc chunk of node x (flagged in F).

// Whole-node discharge by one wave (chunked class, 65..4096 arcs): the wave of
// the node's lead chunk item loads its arcs NB×64 at a time (all loads of a
// batch issued together, then the price gathers), distributes the excess with
// one wave scan per 64 arcs and relabels like sweep_group. One dependent chain
// per batch instead of the claim/arrive protocol of hubs.
// e, px, b0, en: the node's excess, price and segment, loaded by the caller
// together with its frontier flag (one dependent step fewer).
// Whole-node discharge by one workgroup (chunked class): 512 arcs
// per pass (two per thread, all loads issued together), the excess distributed
// by one block-wide scan. A rack (≈ 440 arcs) is one pass — with one wave per
// node it took two dependent batches, and the chunked node was the last block
// of almost every sweep (round 3's per-launch block stamps).
template <bool CP>
__device__ void node_discharge_blk(const DG& g, const Front& F, const Front& N, int x, long long e, long long px,
                                   int b0, int en, long long* __restrict__ PN, const long long* __restrict__ P,
                                   long long eps, Pend& pd, int& out, Cnt& c) {
    __shared__ long long sh[WPB];
    if (threadIdx.x == 0) F.flag[x] = 0;   // the block consumes the node's flag
    if (e <= 0) return;                    // block-uniform
    if (threadIdx.x == 0) c.visit++;
    long long rem = e, minc = INF64;
    for (int base = b0; base < en; base += 2 * BLK) {   // block-uniform trip count
        long long r[2], cs[2], pw[2], uc[2], adm[2], cr[2];
        int w[2], rv[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int a = base + j * BLK + (int)threadIdx.x;
            r[j] = 0;
            cs[j] = 0;
            w[j] = 0;
            rv[j] = 0;
            uc[j] = 0;
            if (a < en) {
                const Pos q = PL<CP>::ld(g, a);
                r[j] = q.rcap;
                w[j] = q.head;
                cs[j] = q.cost;
                rv[j] = q.rev;
                uc[j] = q.ucap;
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) pw[j] = (base + j * BLK + (int)threadIdx.x < en) ? P[ni(w[j])] : 0;
        long long mine = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bool valid = base + j * BLK + (int)threadIdx.x < en;
            cr[j] = cs[j] + px - pw[j];
            adm[j] = (valid && cr[j] < 0 && r[j] > 0) ? r[j] : 0;
            mine += adm[j];
        }
        long long tot = 0;
        const long long excl = block_excl_scan(mine, sh, &tot);
        long long avail = rem - excl;   // units this thread's arcs may take, in arc order
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int a = base + j * BLK + (int)threadIdx.x;
            long long d = avail < adm[j] ? avail : adm[j];
            d = d < 0 ? 0 : d;
            avail -= d;
            if (d > 0) {
                push_arc<CP>(g, &N, a, w[j], r[j], d, pd, out, rv[j], uc[j]);
                c.push++;
            }
            if (a < en) {
                c.scan++;
                if (cr[j] < 0) {
                    if (r[j] - d > 0) minc = min(minc, cr[j]);
                } else if (r[j] > 0 || cr[j] <= eps) {
                    minc = min(minc, cr[j]);
                }
            }
        }
        flush_pending(g, &N, pd, out);
        rem -= tot < rem ? tot : rem;
        if (rem == 0) break;   // no relabel needed: the rest of the arcs need no scan
    }
    minc = block_min(minc, sh);
    if (threadIdx.x == 0) {
        const long long pushed = e - rem;
        if (pushed) atom_add(&g.excess[x], -pushed);
        long long np = px;
        if (rem > 0) {
            if (minc >= INF64) g.ctl->infeasible = 1;
            else np = px - (minc + eps);
            c.relabel++;
            N.flag[x] = 1;
            out = 1;
        }
        PN[ni(x)] = np;
    }
}

// ------------------------------------------------------ grid-stride windows ---
// Sparse passes use a one-generation grid: each wave owns WPW windows (class
// windows, then chunk items) strided across the grid, ballots all their flags
// first (independent loads), then processes only the active ones.
__device__ __forceinline__ int class_of_window(const DG& g, int w) {
    int c = 0;
#pragma unroll
    for (int k = 1; k < CCLS; ++k) c += (w >= g.wbeg[k]) ? 1 : 0;
    return c;
}

// Window w's frontier flags in two steps, so a launch can issue them before it
// knows whether it has work: window_load reads this lane's flag (class windows:
// one node slot per lane; chunk items: the node's flag on lane 0), window_take
// clears what was set (class windows only; a chunk item's flag is cleared by
// the node's owner) and ballots it — nothing when go is false.
struct WinFlag {
    int slot;        // flag index this lane read (-1: none)
    int raw;         // the flag byte
    long long a;     // class windows: loaded WITH the flag — sweeps: the node's
    long long p;     //   excess and price (read buffer); Bellman-Ford: its distance and p0;
    long long seg;   //   both: its packed segment bounds (one dependent step fewer per launch)
};
// MODE 0: the flag only; 1: sweep (excess, P); 2: Bellman-Ford (dist, p0).
template <int MODE>
__device__ __forceinline__ WinFlag window_load(const DG& g, const unsigned char* flags, int w,
                                               const long long* P = nullptr) {
    w = __builtin_amdgcn_readfirstlane(w);   // wave-uniform: the class selection stays scalar
    WinFlag f{-1, 0, 0, 0, 0};
    const int ln = lane_id();
    if (w < g.wbeg[CCLS]) {
        // class c = the last with wbeg[c] <= w, selected over static fields (kernel
        // arguments: no dependent load before the flag's)
        int ob = g.obeg[0], wb = g.wbeg[0], ws = win_slots(0);
#pragma unroll
        for (int k = 1; k < CCLS; ++k)
            if (w >= g.wbeg[k]) {
                ob = g.obeg[k];
                wb = g.wbeg[k];
                ws = win_slots(k);
            }
        if (ln < ws) f.slot = ob + (w - wb) * ws + ln;
        if (MODE && f.slot >= 0) {
            f.seg = g.p0[ni(f.slot) + ND_SEG];
            if (MODE == 1) {
                f.a = atom_load(&g.excess[f.slot]);
                f.p = P[ni(f.slot)];
            } else {
                f.a = atom_load(&g.dist[ni(f.slot)]);
                f.p = g.p0[ni(f.slot)];
            }
        }
    } else if (w < g.wbeg[CCLS] + g.ncitems) {
        if (ln == 0) f.slot = g.citems[w - g.wbeg[CCLS]].node;
    }
    if (f.slot >= 0) f.raw = flags[f.slot];
    return f;
}
__device__ __forceinline__ unsigned long long window_take(const DG& g, unsigned char* flags, int w, const WinFlag& f,
                                                          bool go) {
    const bool on = go && f.raw != 0;
    if (on && w < g.wbeg[CCLS]) flags[f.slot] = 0;
    return __ballot(on);
}
// The prefetched record of node v (v − base = the lane that loaded it), to every lane.
__device__ __forceinline__ void window_node(const WinFlag& f, int v, int base, long long& a, long long& p, int& b0,
                                            int& en) {
    const int src = v >= 0 ? v - base : 0;
    a = __shfl(f.a, src);
    p = __shfl(f.p, src);
    const unsigned long long sg = (unsigned long long)__shfl(f.seg, src);
    b0 = (int)(unsigned)(sg & 0xffffffffULL);
    en = (int)(unsigned)(sg >> 32);
}

// The control words of a launch pass through an empty asm that also takes the
// launch's first loads as inputs: the words are only tested after every one of
// those loads was issued (one wait for all of them; the compiler would
// otherwise test the words first, or sink the other loads under the test).
#define KS_AFTER_LOADS(c0, c1, ...) asm volatile("" : "+v"(c0), "+v"(c1) : __VA_ARGS__)

template <int C, bool CP>
__device__ __forceinline__ void sweep_win(const DG& g, const Front& N, int w, unsigned long long mask,
                                          const WinFlag& f, const long long* __restrict__ P,
                                          long long* __restrict__ PN, long long eps, Pend& pd, int& out, Cnt& c) {
    constexpr int G = class_lanes(C);
    constexpr int PER = 64 / G;
    constexpr int WS = win_slots(C);
    const int base = g.obeg[C] + (w - g.wbeg[C]) * WS;
    const int k = lane_id() / G;
    while (mask) {
        unsigned long long mm = mask;
        for (int j = 0; j < k; ++j) mm &= mm - 1;
        const int v = mm ? base + __ffsll((long long)mm) - 1 : -1;
        long long e = 0, pv = 0;
        int b0 = 0, en = 0;
        window_node(f, v, base, e, pv, b0, en);
        if (v < 0) e = 0;
        sweep_group<G, CP>(g, N, v, e, pv, b0, en, PN, P, eps, pd, out, c);
        for (int j = 0; j < PER; ++j) mask &= mask - 1;
    }
}


template <bool CP>
__global__ __launch_bounds__(BLK) void k_sweep(DG g, int pos, int seq) {
    if (pos == 0 && blockIdx.x == 0 && threadIdx.x == 0) g.ctl->t_sw0 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0)
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) g.sf[(seq + 2) % 3].hub[h] = 0;
    // The preceding global update was applied (c_done) and the frontier is
    // non-empty (c_act): tested only after each block issued its own first loads
    // (flags, excess, node records; KS_AFTER_LOADS), so the control read is not
    // a dependent step of its own.
    int c_done, c_act;   // read in each branch, after its first loads
    auto ctl_words = [&]() {
        c_done = g.ctl->bf_done;
        c_act = pos == 0 ? g.ctl->apply_act : g.ctl->sweep_act[pos - 1];
    };
    const Front F = g.sf[seq % 3], N = g.sf[(seq + 1) % 3];
    const long long eps = g.ctl->eps;
    const long long* P = (pos & 1) ? g.p1 : g.p0;
    long long* PN = (pos & 1) ? g.p0 : g.p1;
    Pend pd{-1, 0};
    Cnt c;
    int out = 0;
    if ((int)blockIdx.x < g.nhitems) {
        const HItem it = g.hitems[blockIdx.x];
        const int fl = F.hub[it.hid];
        const long long px = P[ni(it.node)];
        const long long E = atom_load(&g.excess[it.node]);
        ctl_words();
        KS_AFTER_LOADS(c_done, c_act, "v"(fl), "v"(px), "v"(E));
        if (c_done && c_act && fl) {
            hub_chunk<CP>(g, F, N, it, px, E, P, PN, eps, pd, out, c);
        }
    } else if ((int)blockIdx.x >= g.nhitems + g.sw_clsb) {
        // chunked class: one workgroup per node (a wave per node made the chunked
        // node the last block of almost every sweep)
        const int i = (int)blockIdx.x - g.nhitems - g.sw_clsb;
        if (i < g.ncls_c) {
            const int x = g.obeg[CCLS] + i;
            // flag, excess and record (price, segment) issued together
            const int fl = F.flag[x];
            const long long e = atom_load(&g.excess[x]);
            const long long px = P[ni(x)];
            const long long sw = g.p0[ni(x) + ND_SEG];
            ctl_words();
            KS_AFTER_LOADS(c_done, c_act, "v"(fl), "v"(e), "v"(px), "v"(sw));
            const int b0 = (int)(unsigned)((unsigned long long)sw & 0xffffffffULL);
            const int en = (int)(unsigned)((unsigned long long)sw >> 32);
            // the flag and the excess may change under the block's feet (pushes into
            // x, the flag cleared by thread 0): thread 0's reading decides for all
            __shared__ long long s_e;
            __shared__ int s_go;
            if (threadIdx.x == 0) {
                s_e = e;
                s_go = c_done && c_act && fl;
            }
            __syncthreads();
            if (s_go) {
                node_discharge_blk<CP>(g, F, N, x, s_e, px, b0, en, PN, P, eps, pd, out, c);
            }
        }
    } else {
        // class windows, WPW per wave strided across the class blocks
        const int tw = g.sw_clsb * WPB;
        const int w0 = wave_index_in_grid(g.nhitems);
        WinFlag wf[WPW];
        int any_raw = 0;
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            const int w = w0 + j * tw;
            wf[j] = w < g.wbeg[CCLS] ? window_load<1>(g, F.flag, w, P) : WinFlag{-1, 0, 0, 0, 0};
            any_raw |= wf[j].raw;
        }
        ctl_words();
        KS_AFTER_LOADS(c_done, c_act, "v"(any_raw));
        const bool go = c_done && c_act;
        unsigned long long mk[WPW];
#pragma unroll
        for (int j = 0; j < WPW; ++j) mk[j] = window_take(g, F.flag, w0 + j * tw, wf[j], go);
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            if (!mk[j]) continue;
            const int w = w0 + j * tw;
            switch (class_of_window(g, w)) {
                case 0: sweep_win<0, CP>(g, N, w, mk[j], wf[j], P, PN, eps, pd, out, c); break;
                case 1: sweep_win<1, CP>(g, N, w, mk[j], wf[j], P, PN, eps, pd, out, c); break;
                case 2: sweep_win<2, CP>(g, N, w, mk[j], wf[j], P, PN, eps, pd, out, c); break;
                case 3: sweep_win<3, CP>(g, N, w, mk[j], wf[j], P, PN, eps, pd, out, c); break;
                default: sweep_win<4, CP>(g, N, w, mk[j], wf[j], P, PN, eps, pd, out, c); break;
            }
        }
    }
    if (__any(out) && lane_id() == 0) g.ctl->sweep_act[pos] = 1;
    flush_counters(g, c);
}

// ================================================ Bellman-Ford (GU and PR) ===
// Global price update (GU): distances from the deficit nodes over residual arcs
// of length clamp(floor(rc/ε)+1, 0, LEN_CAP), unreached = INF.
// Price refinement (PR): all distances start at 0, lengths floor(rc/ε)+1 may be
// negative (difference constraints of ε-optimality).
// Push-style: a node whose distance dropped relaxes its IN-arcs (u→v), i.e. the
// reverses of its CSR arcs a = (v→u): residual ucap(a) − rcap(a), cost −cost(a).
// No returning atomics: a plain pre-check filters (a stale distance is only
// larger), atomicMin commits, the flag store marks u for the next round.
//
// PR = 2: price refinement that also finds negative cycles (the
// cycle-cancelling finish). A node's dist slot then packs its distance (biased;
// d ≤ 0 from d ≡ 0) above its parent arc — the position, in the parent's
// segment, of the arc that ends at the node (the parent arc itself is its
// reverse) — so one 64-bit atomicMin keeps each distance and its parent
// consistent, and the parent graph holds the negative cycles that keep the
// refinement from converging.
constexpr int PK_NB = 24;                              // positions below 2^24
constexpr long long PK_NONE = (1LL << PK_NB) - 1;      // no parent (d = 0 from the start)
constexpr long long PK_BIAS = 1LL << 37;
__device__ __forceinline__ long long pk(long long d, long long v) {
    d = d < 1 - PK_BIAS ? 1 - PK_BIAS : (d > PK_BIAS - 1 ? PK_BIAS - 1 : d);
    return ((d + PK_BIAS) << PK_NB) | v;
}
__device__ __forceinline__ long long pk_d(long long key) { return (key >> PK_NB) - PK_BIAS; }
template <int PR>
__device__ __forceinline__ long long dkey(long long raw) { return PR == 2 ? pk_d(raw) : raw; }
// a < b as distances (packed keys: an equal distance through another parent is no improvement)
template <int PR>
__device__ __forceinline__ bool dless(long long a, long long b) { return PR == 2 ? (a >> PK_NB) < (b >> PK_NB) : a < b; }

template <int PR>
__device__ __forceinline__ long long arc_len(long long pu, long long ca, long long pv, long long eps) {
    long long len = floordiv(pu - ca - pv, eps) + 1;
    if (!PR) len = len < 0 ? 0 : (len > LEN_CAP ? LEN_CAP : len);
    return len;
}

// Offer distance cand to node u. Returns true when u is a grouped node whose
// distance this call lowered (the caller then owns propagating it).
template <int PR>
__device__ __forceinline__ bool offer(const DG& g, const Front& nf, int u, long long cand, long long du,
                                      long long B, long long* hub_min, int& out) {
    if (cand >= B) return false;   // at or beyond every listed excess node's distance (bounded update)
    if (u >= g.hub_base) {
        const int h = u - g.hub_base;
        if (h < HUB_LDS) {
            __hip_atomic_fetch_min(&hub_min[h], cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (dless<PR>(cand, atom_min_ret(&g.dist[ni(u)], cand))) {
            nf.hub[h] = 1;
            out = 1;
        }
        return false;
    }
    if (!dless<PR>(cand, du)) return false;
    atom_min(&g.dist[ni(u)], cand);
    return true;
}

// Relax the in-arcs of a low-degree node u (≤ 8 arcs: tasks, PUs) right after
// its distance dropped to du: a second hop inside the same round.
template <int PR, bool CP>
__device__ __forceinline__ void expand_leaf(const DG& g, const Front& nf, int u, long long du, long long pu,
                                            int b0, int b1, long long eps, long long B, long long* hub_min, int& out,
                                            long long& lscan) {
    lscan += b1 - b0;   // the second hop's in-arc positions examined (ks_result.gu_leaf_scans)
    // the records of all (≤ 8) arcs issued together; usually one in-arc carries
    // flow (a task's assignment), so the dependent loads follow for it alone
    unsigned live = 0;
    int hd[8];
    long long cb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        hd[k] = 0;
        cb[k] = 0;
        if (b0 + k < b1) {
            const Pos q = PL<CP>::ld_nr(g, b0 + k);
            hd[k] = q.head;
            cb[k] = q.cost;
            if (q.ucap - q.rcap > 0) live |= 1u << k;
        }
    }
    for (int b = b1 - b0 > 8 ? b0 + 8 : b1; b < b1; ++b) {   // leaves have ≤ 8 arcs; kept for safety
        const Pos q = PL<CP>::ld_nr(g, b);
        if (q.ucap - q.rcap > 0) {
            const int u2 = q.head;
            long long cand = du + arc_len<PR>(g.p0[ni(u2)], q.cost, pu, eps);
            if (PR == 2) cand = pk(cand, b);
            if (offer<PR>(g, nf, u2, cand, u2 < g.hub_base ? g.dist[ni(u2)] : INF64, B, hub_min, out)) {
                nf.flag[u2] = 1;
                out = 1;
            }
        }
    }
    while (live) {
        const int k = __builtin_ctz(live);
        live &= live - 1;
        int u2 = 0;
        long long c2 = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)   // register select (no dynamic indexing into scratch)
            if (j == k) {
                u2 = hd[j];
                c2 = cb[j];
            }
        const long long pu2 = g.p0[ni(u2)];
        const long long du2 = u2 < g.hub_base ? g.dist[ni(u2)] : INF64;
        long long cand = du + arc_len<PR>(pu2, c2, pu, eps);
        if (PR == 2) cand = pk(cand, b0 + k);
        if (offer<PR>(g, nf, u2, cand, du2, B, hub_min, out)) {
            nf.flag[u2] = 1;
            out = 1;
        }
    }
}

// Relax in-arc (u→v) = reverse of CSR arc a = (v→u); residual ucap − rcap,
// cost −cost(a). Loads are issued before the residual test (short chain).
template <int PR, bool CP>
__device__ __forceinline__ void relax_in(const DG& g, const Front& nf, int v, int a, long long dv, long long pv,
                                         long long eps, long long B, long long* hub_min, int& out, long long& lscan) {
    const Pos q = PL<CP>::ld_nr(g, a);
    const long long rin = q.ucap - q.rcap;
    // an arc that cannot relax reads node 0's (hot) record instead of its head's
    // random line: the loads stay unconditional (no branch join to wait at) and
    // the line is not fetched (config 3: −1…2 ms per solve, interleaved A/B)
    const int u = rin > 0 ? q.head : 0;
    const long long ca = q.cost;
    const long long pu = g.p0[ni(u)];
    const long long du = u < g.hub_base ? g.dist[ni(u)] : INF64;
    const bool leaf = g.expand && u < g.obeg[2];
    int b0 = 0, b1 = 0;
    if (leaf) seg_of(g.p0, u, b0, b1);   // same record line as pu, du
    if (rin <= 0) return;
    const long long cand = dv + arc_len<PR>(pu, ca, pv, eps);   // (dv decoded: a distance in every mode)
    if (!offer<PR>(g, nf, u, PR == 2 ? pk(cand, a) : cand, du, B, hub_min, out)) return;
    if (leaf) {
        expand_leaf<PR, CP>(g, nf, u, cand, pu, b0, b1, eps, B, hub_min, out, lscan);   // tasks, PUs: two hops per round
    } else {
        nf.flag[u] = 1;
        out = 1;
    }
}

template <int G, int PR, bool CP>
__device__ __forceinline__ void bf_group_pre(const DG& g, const Front& nf, int v, long long dv, long long pv, int b0,
                                             int en, long long eps, long long B, long long* hub_min, int& out, long long& scans, long long& lscan) {
    const int lig = lane_id() & (G - 1);
    const bool act = v >= 0 && (PR || dv < INF64);
    if (!act) en = b0;
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        if (a < en) {
            relax_in<PR, CP>(g, nf, v, a, dkey<PR>(dv), pv, eps, B, hub_min, out, lscan);
            scans++;
        }
    }
}

// Sparse Bellman-Ford pass over window w of class C (mask from window_mask).
template <int C, int PR, bool CP>
__device__ __forceinline__ void bf_win(const DG& g, const Front& N, int w, unsigned long long mask, const WinFlag& f,
                                       long long eps, long long B, long long* hub_min, int& out, long long& scans, long long& lscan) {
    constexpr int G = class_lanes(C);
    constexpr int PER = 64 / G;
    constexpr int WS = win_slots(C);
    const int base = g.obeg[C] + (w - g.wbeg[C]) * WS;
    const int k = lane_id() / G;
    while (mask) {
        unsigned long long mm = mask;
        for (int j = 0; j < k; ++j) mm &= mm - 1;
        const int v = mm ? base + __ffsll((long long)mm) - 1 : -1;
        long long d = INF64, pv = 0;
        int b0 = 0, en = 0;
        window_node(f, v, base, d, pv, b0, en);
        if (v < 0) d = INF64;
        bf_group_pre<G, PR, CP>(g, N, v, d, pv, b0, en, eps, B, hub_min, out, scans, lscan);
        for (int j = 0; j < PER; ++j) mask &= mask - 1;
    }
}

// One 64-arc chunk of a chunked-class node (its flag already tested).
template <int PR, bool CP>
__device__ __forceinline__ void bf_chunk(const DG& g, const Front& N, const CItem& ci, long long eps,
                                         long long B, long long* hub_min, int& out, long long& scans, long long& lscan) {
    const long long dv = atom_load(&g.dist[ni(ci.node)]);
    if (!PR && dv >= INF64) return;
    const int a = ci.begin + lane_id();
    if (a < ci.end) {
        relax_in<PR, CP>(g, N, ci.node, a, dkey<PR>(dv), g.p0[ni(ci.node)], eps, B, hub_min, out, lscan);
        scans++;
    }
}

template <int G, int PR, bool CP>
__device__ __forceinline__ void bf_group(const DG& g, const Front& nf, int v, long long eps, long long B, long long* hub_min,
                                         int& out, long long& scans, long long& lscan) {
    const int lig = lane_id() & (G - 1);
    long long dv = INF64;
    if (v >= 0) dv = atom_load(&g.dist[ni(v)]);
    const bool act = v >= 0 && (PR || dv < INF64);
    long long pv = 0;
    int b0 = 0, en = 0;
    if (act) {
        pv = g.p0[ni(v)];
        seg_of(g.p0, v, b0, en);
    }
    const int iters = G < 64 ? 1 : (en - b0 + 63) / 64;
    for (int it = 0; it < iters; ++it) {
        const int a = b0 + it * G + lig;
        if (a < en) {
            relax_in<PR, CP>(g, nf, v, a, dkey<PR>(dv), pv, eps, B, hub_min, out, lscan);
            scans++;
        }
    }
}

// One Bellman-Ford round. dense = 1: every node (first round of an update).
// dense_arg < 0: the round is dense iff it is the running update's first
// (bf_seq0, set by the init kernel); ≥ 0: as given.
template <int PR, bool CP>
__global__ __launch_bounds__(BLK) void k_bf_round(DG g, int seq, int dense_arg) {
    const unsigned long long t_entry = PR == 2 ? __builtin_amdgcn_s_memrealtime() : 0;
    const int dense = dense_arg >= 0 ? dense_arg : (seq == g.ctl->bf_seq0 ? 1 : 0);
    __shared__ long long hub_min[HUB_LDS];
    if (blockIdx.x == 0) {
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) g.bf[(seq + 2) % 3].hub[h] = 0;
        if (threadIdx.x == 0) g.ctl->bfa[(seq + 2) % 3] = 0;
    }
    const Front F = g.bf[seq % 3], N = g.bf[(seq + 1) % 3];
    if (threadIdx.x < HUB_LDS) hub_min[threadIdx.x] = INF64;
    __syncthreads();   // (waits for outstanding loads: the control words are read after it)
    // The update is still running (!done) and this round's frontier is non-empty
    // (dense || any): read in each branch after its first loads and tested only
    // once they were issued (KS_AFTER_LOADS).
    int done = 0, any = 0;
    auto ctl_words = [&]() {
        done = g.ctl->bf_done;
        any = g.ctl->bfa[seq % 3];
    };
    const long long eps = g.ctl->eps;
    // bounded update (tail): offers at or above the listed excess nodes' largest
    // tentative distance are dropped (that bound only falls, so a stale copy is safe)
    const long long B = (!PR && g.bound) ? atom_load(&g.ctl->bf_bound) : INF64;
    int out = 0;
    long long scans = 0, lscan = 0;
    // Hub chunks are split over HSPLIT workgroups: a relaxation is a dependent
    // chain (arc, tail record, leaf expansion, atomic), and a thread that runs
    // several of them in a row made the hub the last block of its round.
    const int nhb = g.nhitems * HSPLIT;
    if ((int)blockIdx.x < nhb) {
        const HItem it = g.hitems[blockIdx.x / HSPLIT];
        const int sub = (int)blockIdx.x % HSPLIT;
        const int fl = F.hub[it.hid];
        const long long dv = atom_load(&g.dist[ni(it.node)]);
        const long long pv = g.p0[ni(it.node)];
        ctl_words();
        KS_AFTER_LOADS(done, any, "v"(fl), "v"(dv), "v"(pv));
        if (!done && (dense || any) && (dense || fl)) {
            if (PR || dv < INF64) {
#pragma unroll
                for (int k = 0; k < BF_PER_T; ++k) {
                    const int a = it.begin + sub * (CHUNK / HSPLIT) + threadIdx.x * BF_PER_T + k;
                    if (a < it.end) {
                        relax_in<PR, CP>(g, N, it.node, a, dkey<PR>(dv), pv, eps, B, hub_min, out, lscan);
                        scans++;
                    }
                }
            }
        }
    } else if (dense) {
        const int w = wave_index_in_grid(nhb);
        ctl_words();
        if (done) {
            // the update already converged
        } else if (w < g.wbeg[CCLS]) {
            const Scan sc{F.flag, 1};
#define KS_BF_CALL(C) bf_group<G_, PR, CP>(g, N, v, eps, B, hub_min, out, scans, lscan)
            KS_BY_CLASS(w, sc, KS_BF_CALL)
#undef KS_BF_CALL
        } else if (w - g.wbeg[CCLS] < g.ncitems) {
            bf_chunk<PR, CP>(g, N, g.citems[w - g.wbeg[CCLS]], eps, B, hub_min, out, scans, lscan);
        }
    } else {
        const int tw = ((int)gridDim.x - nhb) * WPB;
        const int w0 = wave_index_in_grid(nhb);
        WinFlag wf[WPW];
        int any_raw = 0;
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            wf[j] = window_load<2>(g, F.flag, w0 + j * tw);
            any_raw |= wf[j].raw;
        }
        ctl_words();
        KS_AFTER_LOADS(done, any, "v"(any_raw));
        const bool go = !done && any;
        unsigned long long mk[WPW];
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            const int w = w0 + j * tw;
            mk[j] = window_take(g, F.flag, w, wf[j], go);
            // chunk items: a node's flag is read by all its chunks; the lead chunk
            // clears it two rounds later (in the buffer read by the previous round)
            if (go && w >= g.wbeg[CCLS] && w - g.wbeg[CCLS] < g.ncitems && lane_id() == 0) {
                const CItem ci = g.citems[w - g.wbeg[CCLS]];
                if (ci.lead) g.bf[(seq + 2) % 3].flag[ci.node] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            if (!mk[j]) continue;
            const int w = w0 + j * tw;
            if (w >= g.wbeg[CCLS]) {
                bf_chunk<PR, CP>(g, N, g.citems[w - g.wbeg[CCLS]], eps, B, hub_min, out, scans, lscan);
                continue;
            }
            switch (class_of_window(g, w)) {
                case 0: bf_win<0, PR, CP>(g, N, w, mk[j], wf[j], eps, B, hub_min, out, scans, lscan); break;
                case 1: bf_win<1, PR, CP>(g, N, w, mk[j], wf[j], eps, B, hub_min, out, scans, lscan); break;
                case 2: bf_win<2, PR, CP>(g, N, w, mk[j], wf[j], eps, B, hub_min, out, scans, lscan); break;
                case 3: bf_win<3, PR, CP>(g, N, w, mk[j], wf[j], eps, B, hub_min, out, scans, lscan); break;
                default: bf_win<4, PR, CP>(g, N, w, mk[j], wf[j], eps, B, hub_min, out, scans, lscan); break;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < HUB_LDS && (int)threadIdx.x < g.nheavy) {
        const long long val = hub_min[threadIdx.x];
        if (val < INF64) {
            long long* dx = &g.dist[ni(g.hub_base + threadIdx.x)];
            if (dless<PR>(val, atom_load(dx)) && dless<PR>(val, atom_min_ret(dx, val))) {
                N.hub[threadIdx.x] = 1;
                out = 1;
            }
        }
    }
    if (__any(out) && lane_id() == 0) g.ctl->bfa[(seq + 1) % 3] = 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // block 0 is a hub block or a window block: done/any are final here
        if (PR == 2 && g.ctl->t_srch) {   // the finish: the search before this round ended when it started
            g.ctl->srch_ticks += t_entry - g.ctl->t_srch;
            g.ctl->t_srch = 0;
        }
        if (!done && (dense || any)) {
            atomicAdd(g.ctr + C_BFROUND, 1ULL);
            g.ctl->bf_count += 1;
        } else if (!done) {
            g.ctl->bf_done = 1;   // empty frontier: the update converged
        }
    }
    // the next rounds' bound: the largest tentative distance of the listed excess
    // nodes once all of them are reached (every value taken is ≥ the final one)
    if (!PR && g.bound && blockIdx.x == 0 && threadIdx.x < WAVE && !done && (dense || any)) {
        const int nb = g.ctl->n_bx;
        if (nb > 0 && nb <= BX_CAP) {
            long long d = 0;
            if ((int)threadIdx.x < nb) d = atom_load(&g.dist[ni(g.bx[threadIdx.x])]);
            d = wave_max(d);
            if (threadIdx.x == 0 && d < INF64)
                __hip_atomic_fetch_min(&g.ctl->bf_bound, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    scans = wave_sum(scans);
    lscan = wave_sum(lscan);
    if (lane_id() == 0 && (scans | lscan)) {
        const int sh = ((blockIdx.x * WPB) + (threadIdx.x >> 6)) & (CTR_SHARDS - 1);
        if (scans) atomicAdd(g.ctr + sh * NCTR + C_GUSCAN, (unsigned long long)scans);
        if (lscan) atomicAdd(g.ctr + sh * NCTR + C_GULEAF, (unsigned long long)lscan);
    }
}

__device__ __forceinline__ void clear_fronts(const DG& g, const Front* fs) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < g.hub_base; i += (long long)gridDim.x * BLK) {
        fs[0].flag[i] = 0;
        fs[1].flag[i] = 0;
        fs[2].flag[i] = 0;
    }
    if (blockIdx.x == 0)
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) fs[0].hub[h] = fs[1].hub[h] = fs[2].hub[h] = 0;
}

// Wave-aggregated append of the lanes with on set to the bound's excess list.
__device__ __forceinline__ void bx_append(const DG& g, bool on, int v) {
    const unsigned long long m = __ballot(on);
    if (!m) return;
    int base = 0;
    if (lane_id() == 0) base = atomicAdd(&g.ctl->n_bx, (int)__popcll(m));
    base = __shfl(base, 0);
    if (on) {
        const int idx = base + (int)__popcll(m & ((1ULL << lane_id()) - 1));
        if (idx < BX_CAP) g.bx[idx] = v;
    }
}

// GU init: drain hub inboxes, dist = 0 at deficits / INF elsewhere, clean flags.
// A cycle whose predecessor left its update unconverged (gu_pending) continues
// that update instead; seq0 = the sequence number of this cycle's first round.
// The deficits are the first round's frontier (a sparse round: the dense pass
// over every node cost 16–60 µs per update). Each flag is set by the thread that
// cleared it (same grid-stride mapping as clear_fronts; hubs: block 0).
__global__ void k_gu_init(DG g, int seq0, int list) {
    if (g.ctl->gu_pending) return;
    clear_fronts(g, g.bf);
    const Front F0 = g.bf[seq0 % 3];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        __hip_atomic_store(&g.ctl->bf_bound, INF64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g.ctl->gu_B = INF64;
        g.ctl->bf_done = 0;
        g.ctl->gu_L = 0;
        g.ctl->gu_X = -1;
        g.ctl->bf_r0 = g.ctl->bf_count;
        g.ctl->bf_seq0 = seq0;
        g.ctl->n_exc = 0;
        g.ctl->u_exc = 0;
        g.ctl->aug_reached = 0;
        g.ctl->aug_short = 0;
        for (int k = 0; k < 3; ++k) g.ctl->bfa[k] = k == seq0 % 3 ? 1 : 0;
    }
    // list: the host expects few excess nodes (the last apply found ≤ BX_CAP) —
    // list them (n_bx, reset by k_gu_max) so the rounds can bound the update
    for (long long v0 = blockIdx.x * (long long)BLK; v0 < g.hub_base; v0 += (long long)gridDim.x * BLK) {
        const long long v = v0 + threadIdx.x;
        long long e = 0;
        if (v < g.hub_base) {
            e = atom_load(&g.excess[v]);
            g.dist[ni(v)] = e < 0 ? 0 : INF64;
            if (e < 0) F0.flag[v] = 1;
        }
        if (list) bx_append(g, e > 0, (int)v);
    }
    if (blockIdx.x == 0)
        for (int h0 = 0; h0 < g.nheavy; h0 += BLK) {
            const int h = h0 + threadIdx.x;
            long long e = 0;
            if (h < g.nheavy) {
                drain_inbox(g, h);
                e = atom_load(&g.excess[g.hub_base + h]);
                g.dist[ni(g.hub_base + h)] = e < 0 ? 0 : INF64;
                if (e < 0) F0.hub[h] = 1;
            }
            if (list) bx_append(g, e > 0, g.hub_base + h);
        }
}

// PR init: dist = 0 everywhere, or dist = p (canonical prices: see k_pr_apply);
// from_p = 2: d = 0 with no parent, packed (the cycle-cancelling refinement).
__global__ void k_pr_init(DG g, int seq0, int from_p) {
    clear_fronts(g, g.bf);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g.ctl->bf_done = 0;
        g.ctl->bf_seq0 = seq0;
        for (int k = 0; k < 3; ++k) g.ctl->bfa[k] = 0;
    }
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK)
        g.dist[ni(v)] = from_p == 2 ? ((PK_BIAS << PK_NB) | PK_NONE) : from_p ? g.p0[ni(v)] : 0;
}

// End of a cycle: an update that has not converged is continued by the next
// cycle; the control block goes straight to pinned host memory (a copy engine
// transfer would drain the queue around it: ~65 µs of idle GPU per cycle).
__global__ void k_cycle_end(DG g, Ctl* host, int fwd) {
    static_assert(sizeof(Ctl) % 4 == 0, "Ctl is copied as words");
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        if (!fwd) g.ctl->gu_pending = g.ctl->bf_done ? 0 : 1;   // (forward: k_fs_end)
        g.ctl->t_end = t;
    }
    __syncthreads();
    const int* src = reinterpret_cast<const int*>(g.ctl);
    int* dst = reinterpret_cast<int*>(host);
    for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x)
        __hip_atomic_store(&dst[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    // a forward init counts excess nodes into n_exc from every block: zero it here
    // (a backward init zeroes it itself; forward updates: k_fs_end)
    if (threadIdx.x == 0) {
        if (!fwd) {
            g.ctl->n_exc = 0;
            g.ctl->u_exc = 0;
        }
        g.ctl->fs_moved_cyc = 0;
    }
    __threadfence_system();
}

// max finite distance (only once the update converged); cleans the sweep
// frontiers and flags the apply step and the sweeps write.
constexpr int SET_FWD = 1;   // k_set_eps: no forward search pending, its counters zeroed
constexpr int SET_CYC = 2;   //            the finish's cycle counters zeroed
__global__ void k_set_eps(DG g, long long eps, int flags) {
    g.ctl->eps = eps;
    if (flags & SET_FWD) {
        g.ctl->fs_pending = 0;
        g.ctl->fs_cnt[0] = g.ctl->fs_cnt[1] = g.ctl->fs_cnt[2] = 0;
        g.ctl->fs_completed = 0;
    }
    if (flags & SET_CYC) {
        g.ctl->cyc_done = 0;
        g.ctl->cyc_rej = 0;
    }
}

// The finish's batch end: closes the running search's time and copies the control
// block into pinned host memory (no copy-engine transfer: that drains the queue).
__global__ void k_prc_snap(DG g, Ctl* host) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && g.ctl->t_srch) {
        g.ctl->srch_ticks += t - g.ctl->t_srch;
        g.ctl->t_srch = 0;
    }
    __syncthreads();
    const int* src = reinterpret_cast<const int*>(g.ctl);
    int* dst = reinterpret_cast<int*>(host);
    for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x)
        __hip_atomic_store(&dst[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
}

__global__ void k_gu_max(DG g) {
    __shared__ long long sh[WPB];
    clear_fronts(g, g.sf);
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < MAXB; k += BLK) g.ctl->sweep_act[k] = 0;
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) {
            g.aug_req[h] = 0;
        }
        if (threadIdx.x == 0) {
            g.ctl->apply_act = 0;
            g.ctl->n_xl2 = 0;
        }
    }
    if (!g.ctl->bf_done) return;
    if (g.bound && blockIdx.x == 0 && threadIdx.x < WAVE) {
        // a bounded update caps the prices at the listed excess nodes' largest
        // distance (exact there; every node at or beyond it gets the cap)
        const int nb = g.ctl->n_bx;
        if (nb > 0 && nb <= BX_CAP) {
            long long d = 0;
            if ((int)threadIdx.x < nb) d = atom_load(&g.dist[ni(g.bx[threadIdx.x])]);
            d = wave_max(d);
            if (threadIdx.x == 0) g.ctl->gu_B = d;
        }
        if (threadIdx.x == 0) g.ctl->n_bx = 0;   // the next update lists afresh
    }
    long long mx = 0;
    long long mxx = -1;   // the farthest node holding excess
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = atom_load(&g.dist[ni(v)]);
        if (d < INF64) mx = max(mx, d);
        if (d < INF64 && atom_load(&g.excess[v]) > 0) mxx = max(mxx, d);
    }
    mx = wave_max(mx);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) sh[w] = mx;
    mxx = wave_max(mxx);
    __shared__ long long shx[WPB];
    if (lane_id() == 0) shx[w] = mxx;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int i = 0; i < WPB; ++i) t = max(t, sh[i]);
        if (t) __hip_atomic_fetch_max(&g.ctl->gu_L, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        long long tx = -1;
        for (int i = 0; i < WPB; ++i) tx = max(tx, shx[i]);
        if (tx >= 0) __hip_atomic_fetch_max(&g.ctl->gu_X, tx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// apply p ← p − ε·min(d, L) and seed the sweep frontier with every excess node
// (L: the largest finite distance, capped at the farthest excess node's).
__global__ void k_gu_apply(DG g, int sseq) {
    if (!g.ctl->bf_done) return;
    const long long eps = g.ctl->eps;
    const long long lim = (1LL << 60) / eps;
    long long L = g.ctl->gu_L;
    L = L < g.ctl->gu_B ? L : g.ctl->gu_B;   // bounded update: the cap
    {   // and at the farthest excess node's distance: min(d, X) keeps the triangle inequality
        // (monotone, 1-Lipschitz), every excess node still gets its full step, and the
        // nodes beyond X — far from the deficits or cut off — stop drifting by ε·L per
        // update (config 4: 34–37 → 29–31 ms per round, config 3 unchanged)
        const long long X = g.ctl->gu_X;
        if (X >= 0) L = L < X ? L : X;
    }
    L = L < lim ? L : lim;
    const Front F = g.sf[sseq % 3];
    int out = 0, xv = -1;
    long long units = 0;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = atom_load(&g.dist[ni(v)]);
        const long long e = atom_load(&g.excess[v]);
        units += e > 0 ? e : 0;
        if (d >= INF64 && e > 0) atomicOr(&g.ctl->infeasible, 8);
        const long long dd = d < L ? d : L;
        const long long np = g.p0[ni(v)] - eps * dd;
        g.p0[ni(v)] = np;
        g.p1[ni(v)] = np;
        if (e > 0) {
            mark(g, F, (int)v, out);
            xv = (int)v;
        }
    }
    // count the excess nodes (one atomic per wave) and list the first aug_k for the walkers
    const unsigned long long ex = __ballot(out);
    int base = 0;
    if (ex && lane_id() == 0) {
        g.ctl->apply_act = 1;
        base = atomicAdd(&g.ctl->n_exc, (int)__popcll(ex));
    }
    base = __shfl(base, 0);
    units = wave_sum(units);
    if (units && lane_id() == 0) atom_add(&g.ctl->u_exc, units);
    if (out) {
        const int idx = base + (int)__popcll(ex & ((1ULL << lane_id()) - 1));
        if (idx < g.aug_k) g.xl[idx] = xv;
        if (idx < 4) {
            g.ctl->dbg_x[idx] = xv;
            g.ctl->dbg_e[idx] = (int)atom_load(&g.excess[xv]);
        }
    }
}

// ------------------------------------------------------- tail augmentation ---
// When a converged update leaves at most aug_k nodes with excess (the tail of a
// phase: a few units that the sweeps would move one hop per sweep over dozens
// of update cycles), each of them sends its excess straight down the update's
// distances: one wave per excess node walks from u along the residual arc
// (u, w) of least distance d(w), until it reaches a deficit. An arc qualifies
// if d(w) < d(u) (or d(w) = d(u) and it is admissible) and its reduced cost
// under the updated prices is at most slack·ε: the reverse arc a push creates
// then has reduced cost ≥ −slack·ε (slack 1 in a phase that must end
// 1-optimal). Walkers claim residual capacity with a CAS (they may share arcs);
// units that cannot go on (no arc, capacity taken, the hop limit) stay where the
// walk stands, marked for the sweeps that follow; a unit that reaches a hub is
// left there for the hub distribution (k_aug_hub), which hands it on along the
// hub's qualifying arcs in parallel, and a second walker pass starts from the
// nodes it fed. Runs between the apply and the cycle's sweeps.
//
// Measured alternative, not kept: a blocking flow (DFS walkers with
// dead-end marks). On the device's own tail state (a -DKS_DUMP snapshot read by
// tools/proto/tail_dump.c) even a sequential blocking flow needs 21–24 updates
// for config 3's last 68 units — the last ones leave two nodes one unit per
// update through the cluster aggregator — so it saved no cycles and its searches
// cost more than these walks.
constexpr int AUG_K2 = 256;        // walkers from the nodes a hub distribution fed
constexpr int AUG_STEPS = 512;     // hops per walk before its units are left where it stands

// Hub distribution (between the two walker passes): a hub that holds excess
// hands it to its qualifying arcs, one workgroup per chunk claiming its share
// with one returning atomic (as the sweeps' hub chunks do); the fed nodes are
// listed for the second walker pass.
template <bool CP>
__global__ __launch_bounds__(BLK) void k_aug_hub(DG g, int sseq, int slack) {
    __shared__ long long sh[WPB];
    __shared__ long long s_take;
    if (!g.ctl->bf_done) return;
    const int nx = g.ctl->n_exc;
    if (nx == 0 || nx > g.aug_k) return;
    const HItem it = g.hitems[blockIdx.x];
    const int x = it.node;
    const long long E = atom_load(&g.excess[x]);
    if (E <= 0) return;
    const Front F = g.sf[sseq % 3];
    const long long eps = g.ctl->eps;
    const long long dx = atom_load(&g.dist[ni(x)]);
    const long long px = g.p0[ni(x)];
    long long r[PER_T], adm[PER_T], uc[PER_T];
    int w[PER_T], rv[PER_T];
    long long mine = 0;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        r[k] = 0;
        w[k] = 0;
        rv[k] = 0;
        uc[k] = 0;
        adm[k] = 0;
        if (a < it.end) {
            const Pos q = PL<CP>::ld(g, a);
            r[k] = PL<CP>::rc_atomic(g, a);   // the first walker pass claimed with atomics
            w[k] = q.head;
            rv[k] = q.rev;
            uc[k] = q.ucap;
            if (r[k] > 0) {
                const long long cr = q.cost + px - g.p0[ni(q.head)];
                const long long dw = atom_load(&g.dist[ni(q.head)]);
                if (cr <= slack * eps && (dw < dx || (dw == dx && cr < 0))) adm[k] = r[k];
            }
        }
        mine += adm[k];
    }
    long long Ac = 0;
    const long long excl = block_excl_scan(mine, sh, &Ac);
    if (threadIdx.x == 0) {
        long long take = 0;
        if (Ac > 0) {
            const long long start = atom_add_ret(&g.aug_req[it.hid], Ac);
            take = E - start;
            take = take < 0 ? 0 : (take > Ac ? Ac : take);
        }
        s_take = take;
        if (take) atom_add(&g.excess[x], -take);
    }
    __syncthreads();
    long long rt = s_take - excl;
    rt = rt < 0 ? 0 : (rt > mine ? mine : rt);
    int dummy = 0;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const long long d = adm[k] < rt ? adm[k] : rt;
        rt -= d;
        if (d <= 0) continue;
        const int a = it.begin + threadIdx.x * PER_T + k;
        PL<CP>::set_rc(g, a, r[k] - d);   // only this chunk touches the pair in this kernel
        PL<CP>::set_rc(g, rv[k], uc[k] - (r[k] - d));
        const long long now = atom_add_ret(&g.excess[w[k]], d) + d;
        if (now > 0) {
            mark(g, F, w[k], dummy);
            const int idx = atomicAdd(&g.ctl->n_xl2, 1);
            if (idx < AUG_K2) g.xl2[idx] = w[k];
        }
    }
}

// mode 0: from the apply's excess nodes (non-hubs); mode 1: from the nodes a hub
// distribution (k_aug_hub) fed.
template <bool CP>
__global__ __launch_bounds__(WAVE) void k_augment(DG g, int sseq, int mode, int slack) {
    if (!g.ctl->bf_done) return;
    const int nx = g.ctl->n_exc;
    if (nx == 0 || nx > g.aug_k) return;
    const int cnt = mode ? min(g.ctl->n_xl2, AUG_K2) : nx;
    if ((int)blockIdx.x >= cnt) return;
    const int lane = lane_id();
    const Front F = g.sf[sseq % 3];
    const long long eps = g.ctl->eps;
    int u = mode ? g.xl2[blockIdx.x] : g.xl[blockIdx.x];
    if (u < 0 || u >= g.hub_base) return;   // hubs: k_aug_hub
    long long carry = 0;
    if (lane == 0) carry = atom_exch(&g.excess[u], 0LL);
    carry = __shfl(carry, 0);
    if (carry <= 0) {
        if (lane == 0 && carry < 0) atom_add(&g.excess[u], carry);   // (not an excess node any more)
        return;
    }
    long long du = atom_load(&g.dist[ni(u)]);
    long long pu = g.p0[ni(u)];
    int b0, en;
    seg_of(g.p0, u, b0, en);
    // A hop is two dependent levels: [u's records] → [their heads' records: price,
    // distance, segment]; then the claim on the chosen arc, the next node's excess and
    // the next node's first 64 records are all in flight at once (the head's segment
    // came with its record), so the next hop starts from loaded records.
    Pos q0{};
    if (lane < en - b0) q0 = PL<CP>::ld(g, b0 + lane);
    int hops = 0, reached = 0, dummy = 0;
    for (int step = 0; step < AUG_STEPS; ++step) {
        // the qualifying residual arc of least d(w) (ties: lowest position)
        long long bd = INF64, bp = 0, br = 0;
        unsigned long long bseg = 0;
        int ba = -1, bw = 0, brev = 0;
        for (int base = b0; base < en; base += WAVE) {
            const int a = base + lane;
            Pos q{};
            if (base == b0) q = q0;
            else if (a < en) q = PL<CP>::ld(g, a);
            long long key = INF64, pw = 0;
            unsigned long long sg = 0;
            if (a < en) {
                // (the record's residual may be stale under other walkers' claims: the CAS below corrects it)
                pw = g.p0[ni(q.head)];
                const long long dw = atom_load(&g.dist[ni(q.head)]);
                sg = (unsigned long long)g.p0[ni(q.head) + ND_SEG];
                const long long cr = q.cost + pu - pw;
                if (q.rcap > 0 && cr <= slack * eps && (dw < du || (dw == du && cr < 0))) key = dw;
            }
            const long long mn = wave_min(key);
            if (mn < bd) {
                const unsigned long long hit = __ballot(key == mn);
                const int src = __ffsll((long long)hit) - 1;
                bd = mn;
                ba = base + src;
                bw = __shfl(q.head, src);
                brev = __shfl(q.rev, src);
                br = __shfl(q.rcap, src);
                bp = __shfl(pw, src);
                bseg = (unsigned long long)__shfl((long long)sg, src);
            }
        }
        if (ba < 0) break;
        // in flight together: the next node's first records, its excess, the claim
        const int nb0 = (int)(unsigned)(bseg & 0xffffffffULL), nen = (int)(unsigned)(bseg >> 32);
        Pos qn{};
        if (lane < nen - nb0) qn = PL<CP>::ld(g, nb0 + lane);
        long long take = 0, ew = 0;
        if (lane == 0) {
            ew = atom_load(&g.excess[bw]);
            long long r = br;
            for (;;) {   // claim min(carry, residual) on arc ba
                take = r < carry ? r : carry;
                if (take <= 0) {
                    take = 0;
                    break;
                }
                long long exp = r;
                if (PL<CP>::cas_rc(g, ba, exp, r - take)) break;
                r = exp;
            }
            if (take > 0) PL<CP>::add_rc(g, brev, take);
            if (take < carry) {   // the rest stays at u
                atom_add(&g.excess[u], carry - take);
                mark(g, F, u, dummy);
            }
        }
        take = __shfl(take, 0);
        if (take == 0) {
            carry = 0;   // deposited at u above
            break;
        }
        carry = take;
        ++hops;
        u = bw;
        du = bd;
        if (lane == 0 && (ew < 0 || u >= g.hub_base)) {   // a deficit (or a hub: the hub distribution takes over)
            const long long now = atom_add_ret(&g.excess[u], carry) + carry;
            if (now > 0) mark(g, F, u, dummy);
            reached = ew < 0 ? 1 : 0;
            carry = 0;
        }
        carry = __shfl(carry, 0);
        if (carry == 0) break;
        pu = bp;
        b0 = nb0;
        en = nen;
        q0 = qn;
    }
    if (lane == 0) {
        if (carry > 0) {   // hop limit or no qualifying arc: the units stay at u
            atom_add(&g.excess[u], carry);
            mark(g, F, u, dummy);
        }
        const int sh = (int)blockIdx.x & (CTR_SHARDS - 1);
        atomicAdd(reached ? &g.ctl->aug_reached : &g.ctl->aug_short, 1);
        if (reached) atomicAdd(g.ctr + sh * NCTR + C_AUGWALK, 1ULL);
        if (hops) atomicAdd(g.ctr + sh * NCTR + C_AUGHOP, (unsigned long long)hops);
    }
}

// ------------------------------------------------- forward tail update ---
// Once only a few nodes hold excess, a global update (Bellman-Ford from every
// deficit over the whole graph, ~40–60 rounds) moves about one unit per cycle.
// The forward update searches from the excess nodes instead: distances d_f
// over residual arcs of length floor(rc/ε)+1 (≥ 0), stopping at the nearest
// deficit's distance D, then p ← p − ε·max(0, D − d_f) — the dual step of a
// successive-shortest-path solver. Every residual arc keeps length ≥ 0
// (ε-optimality), and each arc of a shortest path from an excess node to a
// deficit at distance D ends with reduced cost in [−ε, 0) (admissible), so one
// unit per such deficit is pushed along the search's parent arcs (k_fs_trace).
// The search touches only the nodes nearer than D (thousands, not the graph).
// A node's key — its record's dist slot — packs d_f above the arc that set it.
__device__ __forceinline__ long long fs_dist(long long key) { return key >> FS_PB; }

// Append the lanes with on set to list l (wave-aggregated); overflow fails the search.
__device__ __forceinline__ void fs_append(const DG& g, int l, bool on, int v) {
    const unsigned long long m = __ballot(on);
    if (!m) return;
    int base = 0;
    if (lane_id() == 0) base = atomicAdd(&g.ctl->fs_cnt[l], (int)__popcll(m));
    base = __shfl(base, 0);
    if (on) {
        const int idx = base + (int)__popcll(m & ((1ULL << lane_id()) - 1));
        if (idx < g.fl_cap) g.fl[(size_t)l * g.fl_cap + idx] = v;
        else g.ctl->fs_fail = 1;
    }
}

// Init: every excess node is a source (d_f 0, no parent), everything else
// unreached; the sources are the first round's frontier. A search still running
// (fs_pending: set by its first round, cleared by k_fs_end once it finished —
// in this cycle's earlier update or the last cycle) is continued instead.
__global__ void k_fs_init(DG g, int seq0) {
    if (g.ctl->fs_pending) return;
    clear_fronts(g, g.bf);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        __hip_atomic_store(&g.ctl->fs_D, INF64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g.ctl->fs_done = 0;
        g.ctl->fs_fail = 0;
        g.ctl->fs_rounds = 0;
        g.ctl->n_fdef = 0;
        g.ctl->fs_moved = 0;   // (n_exc was reset by the last cycle's end: this kernel counts into it)
        g.ctl->fs_maxcnt = 0;
    }
    const int l0 = seq0 % 3;
    for (long long v0 = blockIdx.x * (long long)BLK; v0 < g.hub_base; v0 += (long long)gridDim.x * BLK) {
        const long long v = v0 + threadIdx.x;
        long long e = 0;
        if (v < g.hub_base) {
            e = atom_load(&g.excess[v]);
            g.dist[ni(v)] = e > 0 ? FS_NONE : INF64;
        }
        const unsigned long long m = __ballot(e > 0);
        if (m && lane_id() == 0) atomicAdd(&g.ctl->n_exc, (int)__popcll(m));
        const long long units = wave_sum(e > 0 ? e : 0);
        if (units && lane_id() == 0) atom_add(&g.ctl->u_exc, units);
        fs_append(g, l0, e > 0, (int)v);
    }
    if (blockIdx.x == 0)
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) {
            drain_inbox(g, h);
            const long long e = atom_load(&g.excess[g.hub_base + h]);
            g.dist[ni(g.hub_base + h)] = e > 0 ? FS_NONE : INF64;
            if (e > 0) {
                g.bf[l0].hub[h] = 1;
                atomicAdd(&g.ctl->n_exc, 1);
                atom_add(&g.ctl->u_exc, e);
            }
        }
}

// Relax residual out-arc a of u (distance du, price pu). Returns 1 when a
// non-hub, non-deficit head w was lowered and is not yet listed for the next round.
template <bool CP>
__device__ __forceinline__ int fs_relax(const DG& g, const Front& N, int a, long long du, long long pu, long long eps,
                                        long long B, int& wout) {
    const Pos q = PL<CP>::ld_nr(g, a);
    const int w = q.head;
    const long long pw = g.p0[ni(w)];
    const long long kw = atom_load(&g.dist[ni(w)]);
    const long long ew = atom_load(&g.excess[w]);
    if (q.rcap <= 0) return 0;
    long long len = floordiv(q.cost + pu - pw, eps) + 1;
    len = len < 0 ? 0 : (len > LEN_CAP ? LEN_CAP : len);
    const long long cand = du + len;
    if (cand > B || cand >= FS_DMAX || cand >= fs_dist(kw)) return 0;
    const long long key = (cand << FS_PB) | (long long)a;
    if (key >= atom_min_ret(&g.dist[ni(w)], key)) return 0;
    if (ew < 0) {   // a deficit: the search's bound; paths end here
        __hip_atomic_fetch_min(&g.ctl->fs_D, cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (w >= g.hub_base) {
        N.hub[w - g.hub_base] = 1;
        return 0;
    }
    if (N.flag[w]) return 0;
    N.flag[w] = 1;
    wout = w;
    return 1;
}

// One round: the listed nodes (one wave per node, 64 arcs per batch) and the
// flagged hubs (HSPLIT workgroups per 1024-arc chunk) relax their out-arcs.
template <bool CP>
__global__ __launch_bounds__(BLK) void k_fs_round(DG g, int seq) {
    const int lin = seq % 3, lout = (seq + 1) % 3;
    const Front F = g.bf[lin], N = g.bf[lout];
    if (blockIdx.x == 0) {   // the buffers round seq + 1 appends to were read by round seq − 1
        for (int h = threadIdx.x; h < g.nheavy; h += BLK) g.bf[(seq + 2) % 3].hub[h] = 0;
        if (threadIdx.x == 0) g.ctl->fs_cnt[(seq + 2) % 3] = 0;
    }
    const int done = g.ctl->fs_done | g.ctl->fs_fail;
    const int cnt = g.ctl->fs_cnt[lin];
    const long long B = atom_load(&g.ctl->fs_D);
    const long long eps = g.ctl->eps;
    if (blockIdx.x == 0 && threadIdx.x == 0 && !done) {
        int hub_any = 0;
        for (int h = 0; h < g.nheavy; ++h) hub_any += F.hub[h];
        if (cnt == 0 && !hub_any) g.ctl->fs_done = 1;   // empty frontier: converged
        else {
            g.ctl->fs_pending = 1;   // the next init (this cycle's or the next's) continues it
            g.ctl->fs_rounds += 1;
            atomicAdd(g.ctr + C_BFROUND, 1ULL);
            const int width = cnt + 1024 * hub_any;
            if (width > g.ctl->fs_maxcnt) g.ctl->fs_maxcnt = width;
            // a frontier this wide (a hub's arcs in reach) costs more per unit than
            // the global update it replaces: fail the search as wide
            if (width > g.fs_wide) g.ctl->fs_fail = 2;
        }
    }
    if (done) return;
    const int nhb = g.nhitems * HSPLIT;
    const int lane = lane_id();
    long long scans = 0;   // residual out-arcs examined (the round's units, ks_result.fs_arc_scans)
    auto count = [&]() {
        scans = wave_sum(scans);
        if (lane == 0 && scans) {
            const int sh = ((blockIdx.x * WPB) + (threadIdx.x >> 6)) & (CTR_SHARDS - 1);
            atomicAdd(g.ctr + sh * NCTR + C_FSSCAN, (unsigned long long)scans);
        }
    };
    if ((int)blockIdx.x < nhb) {
        const HItem it = g.hitems[blockIdx.x / HSPLIT];
        if (!F.hub[it.hid]) return;
        const long long du = fs_dist(atom_load(&g.dist[ni(it.node)]));
        const long long pu = g.p0[ni(it.node)];
        const int sub = (int)blockIdx.x % HSPLIT;
        for (int k = 0; k < BF_PER_T; ++k) {
            const int a = it.begin + sub * (CHUNK / HSPLIT) + threadIdx.x * BF_PER_T + k;
            int w = -1;
            const int add = a < it.end ? fs_relax<CP>(g, N, a, du, pu, eps, B, w) : 0;
            scans += a < it.end;
            fs_append(g, lout, add, w);
        }
        count();
        return;
    }
    // listed nodes: one wave each, 64 arcs per pass (eight nodes per wave with eight
    // lanes each was measured slower: a wave then walked its wider nodes — machines —
    // one after another, lengthening the round's chain)
    const int nw = ((int)gridDim.x - nhb) * WPB;
    for (int i = ((int)blockIdx.x - nhb) * WPB + (int)(threadIdx.x >> 6); i < cnt; i += nw) {
        const int v = g.fl[(size_t)lin * g.fl_cap + i];
        const long long key = atom_load(&g.dist[ni(v)]);
        const long long pu = g.p0[ni(v)];
        const long long ev = atom_load(&g.excess[v]);
        int b0, b1;
        seg_of(g.p0, v, b0, b1);
        if (lane == 0) F.flag[v] = 0;
        if (ev < 0) continue;   // a deficit ends its paths
        const long long du = fs_dist(key);
        for (int base = b0; base < b1; base += WAVE) {
            const int a = base + lane;
            int w = -1;
            const int add = a < b1 ? fs_relax<CP>(g, N, a, du, pu, eps, B, w) : 0;
            scans += a < b1;
            fs_append(g, lout, add, w);
        }
    }
    count();
}

// Apply the dual step of a converged search: p ← p − ε·(D − d_f) below D, and
// list the deficits found at distance D for the trace.
__global__ void k_fs_apply(DG g) {
    if (!g.ctl->fs_done || g.ctl->fs_fail) return;
    if (atom_load_i(&g.ctl->n_exc) == 0) return;   // no excess left: nothing to search from
    const long long D = atom_load(&g.ctl->fs_D);
    if (D >= FS_DMAX) {   // no deficit in range: a backward update decides (infeasible or not)
        if (blockIdx.x == 0 && threadIdx.x == 0) g.ctl->fs_fail = 1;
        return;
    }
    const long long eps = g.ctl->eps;
    if (D > (1LL << 60) / eps) {   // ε·D would overflow the prices: a backward update instead
        if (blockIdx.x == 0 && threadIdx.x == 0) g.ctl->fs_fail = 1;
        return;
    }
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = fs_dist(atom_load(&g.dist[ni(v)]));
        if (d < D) {
            const long long np = g.p0[ni(v)] - eps * (D - d);
            g.p0[ni(v)] = np;
            g.p1[ni(v)] = np;
        } else if (d == D && atom_load(&g.excess[v]) < 0) {
            const int idx = atomicAdd(&g.ctl->n_fdef, 1);
            if (idx < FDEF_CAP) g.fdef[idx] = (int)v;
        }
    }
}

// Trace: one unit (or the path's bottleneck) from each listed deficit back along
// the parent arcs to its excess node — one wave per deficit, all in parallel.
// Lane 0 walks the parents (each arc must end at the node it was reached from,
// be residual, and be admissible under the updated prices) into an LDS path;
// the wave then claims the source's excess with a CAS and every arc of the path
// at once (one lane per arc, CAS against the residual); if any arc is short
// (another wave took it) every claim is rolled back and the unit waits for the
// next update. Then the reverse residuals and the deficit are credited.
constexpr int FS_PATH = 512;       // hops a trace may take
template <bool CP>
__global__ __launch_bounds__(WAVE) void k_fs_trace(DG g) {
    __shared__ int path[FS_PATH];
    __shared__ int s_len, s_src;
    __shared__ long long s_amt;
    if (!g.ctl->fs_done || g.ctl->fs_fail) return;
    if ((int)blockIdx.x >= min(g.ctl->n_fdef, FDEF_CAP)) return;
    const int lane = threadIdx.x;
    const int t = g.fdef[blockIdx.x];
    if (lane == 0) {
        long long amt = -atom_load(&g.excess[t]);
        int v = t, src = -1, len = 0;
        while (amt > 0 && len < FS_PATH) {
            const long long key = atom_load(&g.dist[ni(v)]);
            const long long a = key & FS_NONE;
            if (a == FS_NONE) {
                src = v;
                break;
            }
            if (a >= g.npos) break;   // (a key not written by this search)
            const Pos q = PL<CP>::ld(g, (int)a);
            const long long r = PL<CP>::rc_atomic(g, (int)a);
            const int u = PL<CP>::head(g, q.rev);
            if (q.head != v || r <= 0 || q.cost + g.p0[ni(u)] - g.p0[ni(v)] >= 0) break;
            amt = r < amt ? r : amt;
            path[len++] = (int)a;
            v = u;
        }
        if (src >= 0 && src != t) {   // claim the source's excess
            long long e = atom_load(&g.excess[src]);
            for (;;) {
                const long long take = e < amt ? e : amt;
                if (take <= 0) {
                    src = -1;
                    break;
                }
                long long exp = e;
                if (__hip_atomic_compare_exchange_strong(&g.excess[src], &exp, e - take, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    amt = take;
                    break;
                }
                e = exp;
            }
        } else {
            src = -1;
        }
        s_len = len;
        s_src = src;
        s_amt = amt;
    }
    __syncthreads();
    const int len = s_len, src = s_src;
    const long long amt = s_amt;
    if (src < 0) return;
    // claim every arc of the path at once
    bool ok = true;
    unsigned long long mine = 0;   // bit i: this lane holds the claim on path[lane + 64 i]
    for (int i = lane, k = 0; i < len; i += WAVE, ++k) {
        long long r = PL<CP>::rc_atomic(g, path[i]);
        for (;;) {
            if (r < amt) {
                ok = false;
                break;
            }
            long long exp = r;
            if (PL<CP>::cas_rc(g, path[i], exp, r - amt)) {
                mine |= 1ULL << k;
                break;
            }
            r = exp;
        }
    }
    const bool all = __all(ok);
    for (int i = lane, k = 0; i < len; i += WAVE, ++k) {
        if (!(mine >> k & 1)) continue;
        if (all) PL<CP>::add_rc(g, PL<CP>::rev(g, path[i]), amt);
        else PL<CP>::add_rc(g, path[i], amt);   // roll back
    }
    if (lane == 0) {
        if (all) {
            atom_add(&g.excess[t], amt);
            atomicAdd(&g.ctl->fs_moved, 1);
            atomicAdd(&g.ctl->fs_moved_cyc, 1);
        } else {
            atom_add(&g.excess[src], amt);   // the unit stays for the next update
        }
    }
}

// End of a forward update: a finished (or failed) search releases the init and
// reports its excess counts; one still running keeps them (its init is skipped).
__global__ void k_fs_end(DG g) {
    if (threadIdx.x || blockIdx.x) return;
    if (!g.ctl->fs_done && !g.ctl->fs_fail) return;
    g.ctl->fs_pending = 0;
    g.ctl->fs_cnt[0] = g.ctl->fs_cnt[1] = g.ctl->fs_cnt[2] = 0;
    g.ctl->n_exc_rep = atom_load_i(&g.ctl->n_exc);
    g.ctl->u_exc_rep = atom_load(&g.ctl->u_exc);
    g.ctl->n_exc = 0;
    g.ctl->u_exc = 0;
    if (g.ctl->fs_done && !g.ctl->fs_fail) g.ctl->fs_completed += 1;
}

// TESTS ONLY (ks_opts.fault_inject bit 6): move one unit on the first arc that can
// take it without touching any excess word — the flow then violates conservation,
// which only the verifier's balance of the arc flows can see.
__global__ void k_break_conservation(DG g, long long m2) {
    if (threadIdx.x || blockIdx.x) return;
    for (long long p = 0; p < m2; ++p) {
        const Pos q = g.pos[p];
        if (q.rcap > 0 && q.ucap > 0 && q.cost < (1LL << 50)) {
            g.pos[p].rcap = q.rcap - 1;
            g.pos[q.rev].rcap += 1;
            return;
        }
    }
}

// TESTS ONLY (ks_opts.fault_inject bit 1): lower one node's price by delta after
// the solve, so the certificate fails on an optimal flow and must be repaired.
__global__ void k_perturb_price(DG g, int x, long long delta) {
    if (x < g.n) {
        g.p0[ni(x)] -= delta;
        g.p1[ni(x)] -= delta;
    }
}

// PR success: p ← p − ε·d. From d ≡ 0 (d ≤ 0) prices only rise, keeping their
// history. From d = p at ε = 1 the fixpoint is d(u) = p(u) + min(0, min_w dist(u, w))
// over residual paths of length cost + 1 per arc, so p − d = −min(0, min_w dist(u, w)):
// the canonical prices of the flow, the same for any prices it started from
// (warm_canon: the drift of carried prices).
__global__ void k_pr_apply(DG g, int packed) {
    if (!g.ctl->bf_done) return;
    const long long eps = g.ctl->eps;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = atom_load(&g.dist[ni(v)]);
        const long long np = g.p0[ni(v)] - eps * (packed ? pk_d(d) : d);
        g.p0[ni(v)] = np;
        g.p1[ni(v)] = np;
    }
}

// ------------------------------------------- cycle-cancelling refinement ---
// The finish that replaces the final cost-scaling phase: the flow of
// the last coarse phase is feasible and nearly optimal, and what keeps it from
// optimality is a few negative cycles (CPU prototype tools/proto/cycle_cancel.c:
// 11–13 on config 3, 24–120 arcs of cost −1…−4 each). The refinement's
// Bellman-Ford (PR = 2) records each node's parent; when it has not converged
// after a batch of rounds, the parent graph — one parent per node, so its cycles
// are node-disjoint — is searched: pointer doubling (2^k steps) lands every node
// of a cycle no longer than that, the least id of each window groups a cycle, its
// nodes sum the cost and take the bottleneck with atomics, a group that is not a
// union of cycles (nodes disagreeing on the id, a non-residual arc, a node with
// other than one member pointing at it) is dropped, and every good negative group
// pushes its bottleneck around in parallel; the cycle's nodes rejoin the frontier.
// The refinement then continues; once its frontier drains, every residual arc
// meets d(u) ≤ d(v) + len(u, v): the prices p − d certify the flow optimal.
constexpr int CYC_LOG = 10;      // cycles up to 1,024 arcs are found
[[maybe_unused]] constexpr int CYC_WALK = 1 << CYC_LOG;
constexpr int CYC_SHORT = 7;              // a short search's doubling steps
// refinement rounds between parent-graph searches: 4 where the whole
// search is one workgroup's LDS pass (small graphs: a search costs ~3 rounds),
// 8 for the multi-launch search of large graphs (twice the launches for no gain)
constexpr int CYC_EVERY_LDS = 4;
constexpr int CYC_EVERY = 8;
constexpr int CYC_PERIODS = 3;            // rounds + search periods per host check
constexpr long long kPrcUnitsDiv = 4;   // an earlier finish (run_phase prc_early)

// The parent of every node (itself for a root) from its key's position a (the
// parent v is the head of a's reverse); the jump word (node one step ahead, least
// id over the one-node window = its own id); the per-group sums reset.
template <bool CP>
__global__ void k_cyc_par(DG g, int* __restrict__ J0, int2* __restrict__ JM, int* __restrict__ onc,
                          int* __restrict__ R, long long* __restrict__ gsum, long long* __restrict__ gcap,
                          int* __restrict__ gbad, int* __restrict__ indeg) {
    if (g.ctl->bf_done) return;   // the refinement converged: no search
    if (blockIdx.x == 0 && threadIdx.x == 0) g.ctl->t_srch = __builtin_amdgcn_s_memrealtime();
    for (long long u = blockIdx.x * (long long)BLK + threadIdx.x; u < g.n; u += (long long)gridDim.x * BLK) {
        const long long a = atom_load(&g.dist[ni(u)]) & PK_NONE;
        int v = (int)u;
        if (a != PK_NONE) v = PL<CP>::head(g, PL<CP>::rev(g, (int)a));
        J0[u] = v;
        JM[u] = make_int2(v, (int)u);
        R[u] = (int)a;
        onc[u] = 0;
        gsum[u] = 0;
        gcap[u] = INF64;
        gbad[u] = 0;
        indeg[u] = 0;
    }
}
// One jump step: a window of w nodes → F·w (F jumps of the previous step chained;
// F = 4 per launch where the window allows, 2 for an odd power of two: a search
// covers 128 steps in 4 launches, 1,024 in 5, instead of 7 and 10 doublings). The
// jump word packs the node w steps ahead and the least id over the window. On the
// search's last step (mark) every node a window ahead of another is marked — it
// lies on a cycle, or (past the window) on a chain, which the union-of-cycles test
// rejects; roots (their own parent) are skipped.
template <int F>
__global__ void k_cyc_jump(int n, const int* __restrict__ done, const int2* __restrict__ JMi,
                           int2* __restrict__ JMo, int mark, const int* __restrict__ J0, int* __restrict__ onc) {
    if (*done) return;
    for (long long u = blockIdx.x * (long long)BLK + threadIdx.x; u < n; u += (long long)gridDim.x * BLK) {
        int2 c = JMi[u];
        int mn = c.y;
#pragma unroll
        for (int f = 1; f < F; ++f) {
            const int2 x = JMi[c.x];
            mn = min(mn, x.y);
            c.x = x.x;
        }
        JMo[u] = make_int2(c.x, mn);
        if (mark && J0[c.x] != c.x) onc[c.x] = 1;
    }
}
// Each cycle node adds its parent arc (u → v, the reverse of position R[u]) to its
// group — the least id of its window, the cycle's least id when the cycle has at
// most CYC_WALK nodes: cost sum, bottleneck residual. A group whose nodes disagree
// on the group (a longer cycle) or whose arc is not residual is marked bad.
template <bool CP>
__global__ void k_cyc_group(DG g, const int* __restrict__ J0, const int2* __restrict__ MK, const int* __restrict__ onc,
                            const int* __restrict__ R, long long* __restrict__ gsum, long long* __restrict__ gcap,
                            int* __restrict__ gbad, int* __restrict__ indeg) {
    if (g.ctl->bf_done) return;
    for (long long u = blockIdx.x * (long long)BLK + threadIdx.x; u < g.n; u += (long long)gridDim.x * BLK) {
        if (!onc[u] || J0[u] == (int)u) continue;
        const int m = MK[u].y, mn = MK[J0[u]].y;
        // a parent off the group (another group, or unmarked): u's arc leaves the
        // group, which is then no union of cycles. The parent's group is not blamed:
        // it counts only its own members' pointers (a chain of another group that
        // runs into a cycle leaves the cycle's group intact, and cancelling it moves
        // nothing the chain's group owns).
        if (mn != m || !onc[J0[u]]) gbad[m] = 1;
        else atomicAdd(&indeg[J0[u]], 1);
        const Pos q = PL<CP>::ld_nr(g, R[u]);
        const long long res = q.ucap - q.rcap;   // residual of the reverse: the arc u → v
        if (res <= 0) gbad[m] = 1;
        atom_add(&gsum[m], -q.cost);
        __hip_atomic_fetch_min(&gcap[m], res, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// A group is a union of cycles only if each of its nodes has exactly one member
// of the group pointing at it (and every member's parent is a member, k_cyc_group):
// each member then has one push out and one push in. A chain longer than the
// doubling window (its nodes marked too) that joins a cycle's group gives the
// junction two, its first node none, and the group is dropped (pushing along a
// chain would break conservation).
// Such nodes are counted (ctl->cyc_rej); apply = 0 (TESTS ONLY, fault_inject bit 8)
// counts them without dropping their groups.
__global__ void k_cyc_check(int n, const int* __restrict__ done, const int* __restrict__ J0,
                            const int2* __restrict__ MK, const int* __restrict__ onc, const int* __restrict__ indeg,
                            int* __restrict__ gbad, int apply, int* __restrict__ rej) {
    if (*done) return;
    int cnt = 0;
    for (long long u = blockIdx.x * (long long)BLK + threadIdx.x; u < n; u += (long long)gridDim.x * BLK)
        if (onc[u] && J0[u] != (int)u && atom_load_i(&indeg[u]) != 1) {
            if (apply) gbad[MK[u].y] = 1;
            ++cnt;
        }
    cnt = (int)wave_sum(cnt);
    if (cnt && lane_id() == 0) atomicAdd(rej, cnt);
}

// Cancel every good negative group: each of its nodes pushes the bottleneck along
// its own parent arc (the arcs of different nodes are different positions), and
// rejoins the frontier the next refinement round reads (buffer seq).
template <bool CP>
__global__ void k_cyc_push(DG g, const int* __restrict__ J0, const int2* __restrict__ MK, const int* __restrict__ onc,
                           const int* __restrict__ R, const long long* __restrict__ gsum,
                           const long long* __restrict__ gcap, const int* __restrict__ gbad, int seq) {
    if (g.ctl->bf_done) return;
    const Front F = g.bf[seq % 3];
    int out = 0, cyc = 0;
    for (long long u = blockIdx.x * (long long)BLK + threadIdx.x; u < g.n; u += (long long)gridDim.x * BLK) {
        if (!onc[u] || J0[u] == (int)u) continue;
        const int m = MK[u].y;
        const long long dl = gcap[m];
        if (gbad[m] || gsum[m] >= 0 || dl <= 0 || dl >= INF64) continue;
        const int a = R[u];
        const Pos q = PL<CP>::ld(g, a);
        PL<CP>::set_rc(g, a, q.rcap + dl);        // the arc u → v is rev(a): its residual falls by dl
        PL<CP>::add_rc(g, q.rev, -dl);
        mark(g, F, (int)u, out);
        cyc += u == m;
    }
    if (__any(out) && lane_id() == 0) g.ctl->bfa[seq % 3] = 1;
    cyc = (int)wave_sum(cyc);
    if (cyc && lane_id() == 0) atomicAdd(&g.ctl->cyc_done, cyc);
}

// The whole search in ONE workgroup with the parent graph in LDS (graphs of at most
// CYC_LDS_K · 1024 internal ids that the LDS holds: config 2's cells). Round 5
// measured a one-workgroup search over global memory slower than the 12 launches;
// here every doubling step, the marks and the in-degrees stay in LDS — three words
// per node: the parent (J0) and the doubling words (jump | least id << CYC_LDS_IDB,
// double-buffered as in the cell solver; the free buffer holds the in-degrees
// afterwards). Each thread owns CYC_LDS_K nodes and issues their loads together
// (the parents' keys, then the reverse positions, then the heads: three dependent
// levels in all, not three per node). Only the marked nodes touch global memory
// after that: their group sums (zeroed by the group's own members) and the pushes.
// Same steps and the same union-of-cycles test as k_cyc_par … k_cyc_push.
constexpr int CYC_LDS_T = 1024;
constexpr int CYC_LDS_K = 14;              // nodes per thread
constexpr int CYC_LDS_IDB = 15;
constexpr int CYC_LDS_IDM = (1 << CYC_LDS_IDB) - 1;
constexpr int CYC_LDS_ON = 1 << 30;
constexpr int CYC_LDS_MAX = CYC_LDS_K * CYC_LDS_T;   // (< 2^15: ids fit the packed word)
static_assert(CYC_LDS_MAX <= CYC_LDS_IDM, "node ids must fit the packed doubling word");
__host__ __device__ constexpr size_t cyc_lds_bytes(int n) { return (size_t)3 * sizeof(int) * (size_t)n; }

template <bool CP>
__global__ __launch_bounds__(CYC_LDS_T) void k_cyc_lds(DG g, int lg, int apply_check, int seq,
                                                      long long* __restrict__ gsum, long long* __restrict__ gcap,
                                                      int* __restrict__ gbad) {
    if (g.ctl->bf_done) return;   // the refinement converged: no search
    if (threadIdx.x == 0) g.ctl->t_srch = __builtin_amdgcn_s_memrealtime();
    extern __shared__ int cyc_sm[];
    const int n = g.n;
    int* J0 = cyc_sm;
    int* Wi = cyc_sm + n;
    int* Wo = Wi + n;
    const int t = threadIdx.x;
    {   // parents: each level's loads for all of this thread's nodes issued together
        long long key[CYC_LDS_K];
        int rv[CYC_LDS_K], hd[CYC_LDS_K];
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) {
            const int u = t + k * CYC_LDS_T;
            key[k] = u < n ? atom_load(&g.dist[ni(u)]) & PK_NONE : PK_NONE;
        }
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) rv[k] = PL<CP>::rev(g, key[k] != PK_NONE ? (int)key[k] : 0);
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) hd[k] = PL<CP>::head(g, rv[k]);
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) {
            const int u = t + k * CYC_LDS_T;
            if (u < n) {
                const int v = key[k] != PK_NONE ? hd[k] : u;
                J0[u] = v;
                Wi[u] = v | (u << CYC_LDS_IDB);
            }
        }
    }
    __syncthreads();
    for (int d = 0; d < lg; ++d) {   // 2^d steps ahead, then 2^d more; the least id over them
        int w[CYC_LDS_K], wx[CYC_LDS_K];
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) {
            const int u = t + k * CYC_LDS_T;
            w[k] = u < n ? Wi[u] : 0;
        }
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) wx[k] = Wi[w[k] & CYC_LDS_IDM];
#pragma unroll
        for (int k = 0; k < CYC_LDS_K; ++k) {
            const int u = t + k * CYC_LDS_T;
            if (u < n)
                Wo[u] = (wx[k] & CYC_LDS_IDM) | (min(w[k] >> CYC_LDS_IDB, wx[k] >> CYC_LDS_IDB) << CYC_LDS_IDB);
        }
        __syncthreads();
        int* tmp = Wi;
        Wi = Wo;
        Wo = tmp;
    }
    // every node a window ahead of another lies on a cycle (or, past the window, on
    // a chain — the test below); roots are skipped. Wo now holds the in-degrees.
    for (int u = t; u < n; u += CYC_LDS_T) {
        const int x = Wi[u] & CYC_LDS_IDM;
        if (J0[x] != x) atomicOr(&Wi[x], CYC_LDS_ON);
        Wo[u] = 0;
    }
    __syncthreads();
    // the marked nodes reset their group's sums (every member writes the same values)
    for (int u = t; u < n; u += CYC_LDS_T) {
        const int w = Wi[u];
        if (!(w & CYC_LDS_ON) || J0[u] == u) continue;
        const int m = (w & ~CYC_LDS_ON) >> CYC_LDS_IDB;
        gsum[m] = 0;
        gcap[m] = INF64;
        gbad[m] = 0;
    }
    __syncthreads();
    for (int u = t; u < n; u += CYC_LDS_T) {
        const int w = Wi[u];
        const int p = J0[u];
        if (!(w & CYC_LDS_ON) || p == u) continue;
        const int m = (w & ~CYC_LDS_ON) >> CYC_LDS_IDB;
        const int wp = Wi[p];
        const int mn = (wp & ~CYC_LDS_ON) >> CYC_LDS_IDB;
        if (mn != m || !(wp & CYC_LDS_ON)) gbad[m] = 1;   // u's arc leaves its group (k_cyc_group)
        else atomicAdd(&Wo[p], 1);
        const int a = (int)(atom_load(&g.dist[ni(u)]) & PK_NONE);
        const Pos q = PL<CP>::ld_nr(g, a);
        const long long res = q.ucap - q.rcap;   // residual of the reverse: the arc u → v
        if (res <= 0) gbad[m] = 1;
        __hip_atomic_fetch_add(&gsum[m], -q.cost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_min(&gcap[m], res, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    int rej = 0;
    for (int u = t; u < n; u += CYC_LDS_T) {   // the union-of-cycles test (k_cyc_check)
        const int w = Wi[u];
        if ((w & CYC_LDS_ON) && J0[u] != u && Wo[u] != 1) {
            if (apply_check) gbad[(w & ~CYC_LDS_ON) >> CYC_LDS_IDB] = 1;
            ++rej;
        }
    }
    __syncthreads();
    const Front F = g.bf[seq % 3];
    int out = 0, cyc = 0;
    for (int u = t; u < n; u += CYC_LDS_T) {
        const int w = Wi[u];
        if (!(w & CYC_LDS_ON) || J0[u] == u) continue;
        const int m = (w & ~CYC_LDS_ON) >> CYC_LDS_IDB;
        // (agent-scope loads: the sums were made by atomics in L2, never from a stale L1 line)
        const long long dl = atom_load(&gcap[m]);
        if (atom_load_i(&gbad[m]) || atom_load(&gsum[m]) >= 0 || dl <= 0 || dl >= INF64) continue;
        const int a = (int)(atom_load(&g.dist[ni(u)]) & PK_NONE);
        const Pos q = PL<CP>::ld(g, a);
        PL<CP>::set_rc(g, a, q.rcap + dl);        // the arc u → v is rev(a): its residual falls by dl
        PL<CP>::add_rc(g, q.rev, -dl);
        mark(g, F, u, out);
        cyc += u == m;
    }
    if (__any(out) && lane_id() == 0) g.ctl->bfa[seq % 3] = 1;
    cyc = (int)wave_sum(cyc);
    rej = (int)wave_sum(rej);
    if (lane_id() == 0) {
        if (cyc) atomicAdd(&g.ctl->cyc_done, cyc);
        if (rej) atomicAdd(&g.ctl->cyc_rej, rej);
    }
}

// ================================================================ verify ===
// Conservation, capacity and 1-optimality (scaled units); per-block cost sums.
__global__ void k_drain_all(DG g) {
    const int h = blockIdx.x * BLK + threadIdx.x;
    if (h < g.nheavy) drain_inbox(g, h);
}

// Per live arc slot: flow (lower bound included) into flows[s], capacity
// feasibility, the cost sum, and the flow value measured from the resident
// flow: net inflow into the demand nodes (supply < 0).
__global__ void k_verify_arcs(DG g, int hi, const unsigned char* __restrict__ alive, const int* __restrict__ fwd,
                              const int* __restrict__ src, const int* __restrict__ dst,
                              const long long* __restrict__ supply, const long long* __restrict__ low,
                              const long long* __restrict__ cap, const long long* __restrict__ cost,
                              long long* __restrict__ flows, long long* __restrict__ part,
                              long long* __restrict__ partf, long long* __restrict__ bal) {
    __shared__ long long sh[WPB];
    // a hub's balance (the sink, the cluster aggregator: every arc into it adds to
    // one word) is summed in LDS and added once per workgroup — one device atomic
    // per arc on the same word serialised at the memory-side atomic unit (~0.1 ms
    // per config-3 verify)
    __shared__ long long hbal[HUB_LDS];
    __shared__ int hslot[HUB_LDS];
    if (threadIdx.x < HUB_LDS) hbal[threadIdx.x] = 0;
    __syncthreads();
    auto add_bal = [&](int x, int slot, long long v) {
        const int h = x - g.hub_base;
        if (h >= 0 && h < HUB_LDS) {
            __hip_atomic_fetch_add(&hbal[h], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            hslot[h] = slot;   // (every writer stores the same slot)
        } else {
            atom_add(&bal[slot], v);
        }
    };
    long long csum = 0, fsum = 0;
    int bad = 0;
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < hi; i += (long long)gridDim.x * BLK) {
        if (!alive[i]) {
            flows[i] = 0;
            continue;
        }
        const int p = fwd[i];
        if (p < 0) {
            bad = 1;
            flows[i] = 0;
            continue;
        }
        const long long cp = cap[i] - low[i];
        const Pos qf = g.pos[p], qr = g.pos[g.pos[p].rev];
        const long long rf = qf.rcap, rr = qr.rcap;
        const long long f = cp - rf;
        if (rf < 0 || rr < 0 || f < 0 || f != rr) bad = 1;
        const long long fl = f + low[i];
        flows[i] = fl;
        if (fl) {   // conservation from the flows themselves (k_verify_balance), not from the excess words
            add_bal(qr.head, src[i], -fl);   // (the reverse position's head is the arc's tail)
            add_bal(qf.head, dst[i], fl);
        }
        csum += fl * cost[i];
        if (supply[dst[i]] < 0) fsum += fl;
        if (supply[src[i]] < 0) fsum -= fl;
    }
    csum = block_sum(csum, sh);
    fsum = block_sum(fsum, sh);
    __syncthreads();
    if (threadIdx.x < HUB_LDS && hbal[threadIdx.x]) atom_add(&bal[hslot[threadIdx.x]], hbal[threadIdx.x]);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = csum;
        partf[blockIdx.x] = fsum;
    }
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 1);
}

// Every live node's net inflow plus its supply is zero (the sink's supply is the
// demand set for this solve): conservation of the flow the caller downloads,
// independent of the solver's own excess bookkeeping.
__global__ void k_verify_balance(DG g, int ncap, const unsigned char* __restrict__ alive,
                                 const long long* __restrict__ supply, const long long* __restrict__ bal) {
    int bad = 0;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK)
        if (alive[v] && atom_load(&bal[v]) + supply[v] != 0) bad = 1;
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 4);
}

__global__ void k_verify_opt(DG g, long long m2) {
    int bad = 0;
    const long long eps = g.ctl->eps;
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK) {
        if (g.pos[p].rcap > 0) {
            const int t = g.pos[g.pos[p].rev].head;
            const long long cr = g.pos[p].cost + g.p0[ni(t)] - g.p0[ni(g.pos[p].head)];
            if (cr < -eps) bad = 1;
        }
    }
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 2);
}

__global__ void k_verify_nodes(DG g) {
    int bad = 0;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK)
        if (atom_load(&g.excess[v]) != 0) bad = 1;
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 4);
}

// ======================================================== warm start ===
// Incremental re-solve (config 4). While the CSR stays valid the previous flow
// and prices simply remain in place (the store's kernels keep the residual
// state consistent with every delta). Across a rebuild they are carried by arc
// slot and node slot: saved before, restored (clamped to the new bounds) after.
__global__ void k_save_flows(int hi, const unsigned char* __restrict__ alive, const int* __restrict__ fwd,
                             const Pos* __restrict__ pos, long long* __restrict__ saved) {
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK) {
        const int p = fwd[s];
        saved[s] = (alive[s] && p >= 0) ? pos[pos[p].rev].rcap : 0;
    }
}

__global__ void k_restore_flows(int hi, const unsigned char* __restrict__ alive, const long long* __restrict__ saved,
                                const long long* __restrict__ low, const long long* __restrict__ cap,
                                const int* __restrict__ fwd, const int* __restrict__ src,
                                const int* __restrict__ dst, const int* __restrict__ perm, Pos* __restrict__ pos,
                                long long* __restrict__ excess) {
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK) {
        if (!alive[s]) continue;
        const long long u = cap[s] - low[s];
        long long f = saved[s];
        f = f < 0 ? 0 : (f > u ? u : f);
        if (f > 0) {
            const int p = fwd[s];
            pos[p].rcap = u - f;
            pos[pos[p].rev].rcap = f;
            atom_add(&excess[perm[src[s]]], -f);
            atom_add(&excess[perm[dst[s]]], f);
        }
    }
}

// Per-cell fallback: the cells in rng (node-slot ranges [lo, hi),
// nr of them) restart cold on the multi-kernel engine — their arcs' carried flows
// and their nodes' carried prices are zeroed between the save and the restore.
// *resets counts the live arc slots and node slots it reset (ks_result.fb_resets).
__global__ void k_fb_reset(int hi, int ncap, int nr, const long long* __restrict__ rng, const int* __restrict__ a_src,
                           const unsigned char* __restrict__ alive, long long* __restrict__ saved,
                           long long* __restrict__ pslot, unsigned long long* __restrict__ resets) {
    const long long n = hi > ncap ? hi : ncap;
    unsigned long long cnt = 0;
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < n; i += (long long)gridDim.x * BLK) {
        const long long vs = i < hi ? a_src[i] : -1, vn = i < ncap ? i : -1;
        bool rs = false, rn = false;
        for (int r = 0; r < nr; ++r) {
            rs |= vs >= rng[2 * r] && vs < rng[2 * r + 1];
            rn |= vn >= rng[2 * r] && vn < rng[2 * r + 1];
        }
        if (rs) saved[i] = 0;
        if (rn) pslot[i] = 0;
        cnt += (rs && alive[i] ? 1 : 0) + (rn ? 1 : 0);
    }
    cnt = (unsigned long long)wave_sum((long long)cnt);
    if (lane_id() == 0 && cnt) atomicAdd(resets, cnt);
}

__global__ void k_save_prices(int ncap, const int* __restrict__ perm, const long long* __restrict__ p0,
                              long long* __restrict__ pslot) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK)
        pslot[v] = p0[ni(perm[v])];
}

// Saved prices by node slot, rescaled when the cost multiplier changed.
__global__ void k_restore_prices(int ncap, int n_prev, long long mult_prev, long long mult,
                                 const long long* __restrict__ pslot, const int* __restrict__ perm,
                                 long long* __restrict__ p0, long long* __restrict__ p1) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        long long p = 0;
        if (v < n_prev) {
            const long long q = pslot[v];
            p = mult == mult_prev ? q : (q / mult_prev) * mult + (q % mult_prev) * mult / mult_prev;
        }
        p0[ni(perm[v])] = p;
        p1[ni(perm[v])] = p;
    }
}

// Warm start: a node whose flow-carrying out-arc got dearer by δ (cost units)
// since the previous solve is priced down by δ·mult, so that arc keeps its
// reduced cost (ks_store.hip k_arc_upserts records δ).
__global__ void k_price_shift(int ncap, const unsigned long long* __restrict__ shift, const int* __restrict__ perm,
                              long long mult, long long* __restrict__ nd) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        const unsigned long long d = shift[v];
        if (!d) continue;
        const int x = perm[v];
        nd[ni(x)] -= (long long)d * mult;
        nd[ni(x) + 2] -= (long long)d * mult;
    }
}

// Nodes created since the previous solve (fresh[v] = 1) get the lowest price
// at which none of their residual out-arcs has a negative reduced cost.
__global__ void k_fresh_prices(int ncap, const unsigned char* __restrict__ fresh, const int* __restrict__ perm, DG g) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        if (!fresh[v]) continue;
        const int x = perm[v];
        long long best = -INF64;
        for (int a = g.first[x]; a < g.first[x + 1]; ++a)
            if (g.pos[a].rcap > 0) best = max(best, g.p0[ni(g.pos[a].head)] - g.pos[a].cost);
        if (best > -INF64) {
            g.p0[ni(x)] = best;
            g.p1[ni(x)] = best;
        }
    }
}

// Largest ε-optimality violation −(c + p(u) − p(w)) over residual arcs → ctl->gu_L.
__global__ void k_max_viol(DG g, long long m2) {
    long long mx = 0;
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK) {
        if (g.pos[p].rcap > 0) {
            const long long cr = g.pos[p].cost + g.p0[ni(g.pos[g.pos[p].rev].head)] - g.p0[ni(g.pos[p].head)];
            if (-cr > mx) mx = -cr;
        }
    }
    mx = wave_max(mx);
    if (lane_id() == 0 && mx > 0) __hip_atomic_fetch_max(&g.ctl->gu_L, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ================================================ task → PU mapping ===
// Path decomposition of the solved flow on device (replaces parseFlowToMapping,
// placement/solver.go:183-269). Flow units are numbered per node: the units
// leaving x are numbered along x's forward arcs in segment order (out prefix), the
// units entering y along y's reverse arcs (in prefix); unit k entering y leaves
// on y's k-th outgoing unit. A task's single unit is followed until it reaches a
// node without outflow (the sink); the last PU on the way is its placement.
__global__ void k_unit_vals(long long m2cap, const int* __restrict__ ent, const long long* __restrict__ flows,
                            long long* __restrict__ outv, long long* __restrict__ inv) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2cap; p += (long long)gridDim.x * BLK) {
        const int e = ent[p];
        const long long f = e >= 0 ? flows[e >> 1] : 0;
        outv[p] = (e >= 0 && !(e & 1)) ? f : 0;
        inv[p] = (e >= 0 && (e & 1)) ? f : 0;
    }
}

__global__ void k_node_meta(int ncap, const int* __restrict__ perm, const unsigned char* __restrict__ type,
                            const unsigned char* __restrict__ alive, unsigned char* __restrict__ itype,
                            int* __restrict__ is_task) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        const unsigned char t = alive[v] ? type[v] : 0;
        itype[perm[v]] = t;
        is_task[v] = t == KS_NODE_TASK ? 1 : 0;
    }
}

// smallest position p in [lo, hi) with pre[p] + val[p] > k (pre is the inclusive-
// exclusive pair of a scan: pre[p] = units before p within the segment)
__device__ __forceinline__ int find_unit(const long long* __restrict__ scan, const long long* __restrict__ val,
                                         int lo, int hi, long long base, long long k) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (scan[mid] - base + val[mid] <= k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void k_task_paths(int ncap, int nn, const int* __restrict__ perm, const int* __restrict__ first,
                             const Pos* __restrict__ pos,
                             const long long* __restrict__ outv, const long long* __restrict__ outs,
                             const long long* __restrict__ inv, const long long* __restrict__ ins,
                             const int* __restrict__ iperm, const unsigned char* __restrict__ itype,
                             const int* __restrict__ rank, const int* __restrict__ is_task, long long cap,
                             unsigned long long* __restrict__ out) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < ncap; v += (long long)gridDim.x * BLK) {
        if (!is_task[v]) continue;
        int x = perm[v];
        long long k = 0;   // unit index among x's outgoing units
        int last_pu = -1;
        for (int step = 0; step <= nn; ++step) {
            const int lo = first[x], hi = first[x + 1];
            if (lo >= hi) break;
            const long long obase = outs[lo];
            const long long otot = outs[hi - 1] + outv[hi - 1] - obase;
            if (k >= otot) break;   // absorbed here (no outflow left)
            const int p = find_unit(outs, outv, lo, hi, obase, k);
            const long long off = k - (outs[p] - obase);
            const int y = pos[p].head;
            if (itype[y] == KS_NODE_PU) last_pu = y;
            const int q = pos[p].rev;
            k = ins[q] - ins[first[y]] + off;
            x = y;
        }
        if (rank[v] < cap) out[rank[v]] = last_pu >= 0 ? (unsigned long long)iperm[last_pu] + 1 : 0ULL;
    }
}

// Per-partition cost and flow value of a disjoint union (k ≤ 1024 parts; one LDS
// accumulator per part and block, one atomic per part and block).
constexpr int MAX_CELLS = 1024;
__global__ void k_cell_sums(int hi, int k, const long long* __restrict__ off, const unsigned char* __restrict__ alive,
                            const int* __restrict__ src, const int* __restrict__ dst,
                            const long long* __restrict__ supply, const long long* __restrict__ cost,
                            const long long* __restrict__ flows, long long* __restrict__ out_cost,
                            long long* __restrict__ out_flow) {
    __shared__ long long sc[MAX_CELLS], sf[MAX_CELLS];
    for (int i = threadIdx.x; i < k; i += BLK) sc[i] = sf[i] = 0;
    __syncthreads();
    for (long long s = blockIdx.x * (long long)BLK + threadIdx.x; s < hi; s += (long long)gridDim.x * BLK) {
        if (!alive[s]) continue;
        const long long f = flows[s];
        if (!f) continue;
        const long long id = (long long)src[s] + 1;
        int lo = 0, hh = k;   // the part j with off[j] < id <= off[j+1]
        while (hh - lo > 1) {
            const int mid = (lo + hh) >> 1;
            if (off[mid] < id) lo = mid; else hh = mid;
        }
        __hip_atomic_fetch_add(&sc[lo], f * cost[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        long long fv = 0;
        if (supply[dst[s]] < 0) fv += f;
        if (supply[src[s]] < 0) fv -= f;
        if (fv) __hip_atomic_fetch_add(&sf[lo], fv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += BLK) {
        if (sc[i]) atom_add(&out_cost[i], sc[i]);
        if (sf[i]) atom_add(&out_flow[i], sf[i]);
    }
}

struct SlotAlive {
    const unsigned char* alive;
    __host__ __device__ bool operator()(const int& s) const { return alive[s] != 0; }
};

__global__ void k_arc_records(int cnt, const int* __restrict__ sel, const int* __restrict__ src,
                              const int* __restrict__ dst, const long long* __restrict__ low,
                              const long long* __restrict__ cap, const long long* __restrict__ cost,
                              const unsigned char* __restrict__ type, ks_arc* __restrict__ out) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < cnt; i += (long long)gridDim.x * BLK) {
        const int s = sel[i];
        ks_arc a;
        a.src = (uint64_t)src[s] + 1;
        a.dst = (uint64_t)dst[s] + 1;
        a.low = (uint64_t)low[s];
        a.cap = (uint64_t)cap[s];
        a.cost = cost[s];
        a.type = type[s];
        a._pad = 0;
        out[i] = a;
    }
}

// positive-flow arcs of the last solve as "f" records (ks_flow), slot order
struct FlowPositive {
    const unsigned char* alive;
    const long long* flows;
    __host__ __device__ bool operator()(const int& s) const { return alive[s] && flows[s] > 0; }
};

__global__ void k_flow_records(int cnt, const int* __restrict__ sel, const int* __restrict__ src,
                               const int* __restrict__ dst, const long long* __restrict__ flows,
                               ks_flow* __restrict__ out) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < cnt; i += (long long)gridDim.x * BLK) {
        const int s = sel[i];
        out[i] = ks_flow{(uint64_t)src[s] + 1, (uint64_t)dst[s] + 1, flows[s]};
    }
}

// ============================================================ host helpers ===
inline int grid_for(long long n, int cap = 4096) {
    long long b = (n + BLK - 1) / BLK;
    if (b < 1) b = 1;
    return (int)std::min<long long>(b, cap);
}

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t k) {
        if (k <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t want = std::max<size_t>(k, 1);
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess) n = want;
        return e;
    }
    // grow to ≥ k elements keeping the first `keep` ones; new tail bytes = fill
    hipError_t grow(size_t k, size_t keep, int fill, hipStream_t st) {
        if (k <= n && p) return hipSuccess;
        const size_t want = std::max<size_t>(k, 1);
        T* q = nullptr;
        hipError_t e = hipMalloc(&q, want * sizeof(T));
        if (e != hipSuccess) return e;
        keep = std::min(keep, n);
        if (keep && p) e = hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipMemsetAsync(q + keep, fill, (want - keep) * sizeof(T), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (p) (void)hipFree(p);
        p = q;
        n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace

struct EngineImpl {
    int device = 0;
    ks_opts opts{};
    hipStream_t stream = nullptr;
    hipEvent_t ev[8] = {};
    hipEvent_t kev[4] = {};   // kernel-batch timing (price refinement)
    hipEvent_t fin_ev[4] = {};      // the finish's pipelined batches: [3] its start, [b % 3] batch b's end
    // per-cycle timing, each kind's span bracketing exactly its kernels: [0] before the
    // first Bellman-Ford round, [1] after the last, [2] before the first sweep, [3] after
    // the last sweep; forward cycles: [0]/[1] around each update's search rounds (fev)
    hipEvent_t cev[CYC_SLOTS][4] = {};
    hipEvent_t fev[CYC_SLOTS][8] = {};
    hipEvent_t cdone[CYC_SLOTS] = {};   // a cycle's control snapshot has landed (timed: cycle end)
    hipEvent_t cstart = nullptr;        // start of a phase's first cycle
    Ctl* h_cyc[CYC_SLOTS] = {};         // pinned control snapshots of the cycles in flight
    Ctl* d_cyc[CYC_SLOTS] = {};         // their device-side addresses (written by k_cycle_end)

    // ---- node store (by slot = id − 1)
    int64_t nstore = 0;       // allocated slots
    int64_t nslots = 0;       // slots in use (max id)
    DBuf<long long> n_supply;
    DBuf<unsigned char> n_type, n_alive, n_fresh;
    DBuf<unsigned long long> n_cshift;   // per slot: cost rise on a flow-carrying out-arc (warm start)
    DBuf<int> n_lastrm;
    DBuf<int> n_hint;         // per slot: segment capacity of the last build
    DBuf<unsigned char> n_grow;
    DBuf<unsigned long long> n_bind;   // per slot: bound PU (scheduling deltas)
    // ---- arc table (by slot) and its hash index
    int64_t acap = 0;
    DBuf<int> a_src, a_dst, fwd, free_stack;
    DBuf<long long> a_low, a_cap, a_cost;
    DBuf<unsigned char> a_alive, a_type;
    int64_t hcap = 0;
    DBuf<unsigned long long> hkey;
    DBuf<int> hval, hlast;
    DBuf<StoreCtl> sctl;
    StoreCtl* h_sctl = nullptr;   // pinned mirror
    DBuf<ks_delta> d_recs;
    DBuf<NodeEdit> d_edits;
    DBuf<int> rec_ent;
    // ---- residual CSR built from the table (internal ids)
    bool csr_valid = false;   // CSR matches the table (deltas applied in place)
    bool incremental = false; // deltas seen since the load: rebuild with slack
    int64_t rebuilds = 0;     // CSR builds since the load
    int64_t ncap = 0;         // node slots covered by the build
    long long mult = 1;       // cost multiplier (ncap + 1)
    int64_t m2cap = 0;        // residual positions (Σ segment capacities)
    DBuf<int> first, ent, used, scur, perm, iperm;
    DBuf<Pos> pos;
    DBuf<CPos> cpos;               // the compact solve's 16-B positions (k_pack_pos)
    DBuf<int> crev;
    DBuf<int> cyc;                 // cycle-cancelling refinement: parents, doubling buffers, marks, arcs
    DBuf<long long> cyc64;         //   and per-group cost sums and bottlenecks
    DBuf<long long> excess;
    DBuf<long long> nd;            // node records [p0, dist, p1, pad] × nn
    DBuf<unsigned> keys_in, keys_out;
    DBuf<int> vals_in, vals_out, pos_of, deg, capv, capi, rs;
    DBuf<unsigned char> sort_tmp, cls;
    DBuf<int> nsel;
    DBuf<int> cls_list[NGC + 1];   // node slots of each degree class; [NGC] = heavy hubs
    DBuf<unsigned char> sel_tmp;
    DBuf<HItem> hitems;
    DBuf<CItem> citems;
    DBuf<int> hnchunks, q_unsat, q_arrive;
    DBuf<long long> q_req, q_taken, q_min, inbox, part, flows;
    DBuf<long long> vbal;               // verification: per-node balance of the arc flows (input slots)
    DBuf<unsigned char> flags;   // 6 frontier buffers × hub_base
    DBuf<int> hubflags;          // 6 × nheavy
    DBuf<unsigned long long> ctr;
    DBuf<int> xl, xl2;                 // walker start nodes (k_augment)
    DBuf<int> bx;                      // excess nodes of the running update (distance bound)
    DBuf<int> fl, fdef;                // forward tail update: frontier lists, traced deficits
    DBuf<long long> aug_req;           // per hub claim counter (k_aug_hub)
    DBuf<Ctl> ctl;
    Ctl* h_ctl = nullptr;        // pinned host mirror
    long long* h_scr = nullptr;  // pinned scratch: [0] eps, [1] max |cost|
    int ncls[NGC + 1] = {0};
    int nheavy = 0, nhitems = 0, ncitems = 0;
    int hub_base = 0, nn = 0;    // grouped node ids [0, hub_base), hubs after: nn ids
    int obeg[NGC + 1] = {0}, oend[NGC] = {0}, wbeg[NGC + 1] = {0};
    // ---- solution
    bool solved = false;         // flows/prices of the current graph are optimal
    bool has_prev = false;       // a solution exists in place (warm start possible)
    int64_t n_tasks = 0;
    DBuf<long long> saved_flows, p_slot;
    DBuf<long long> map_outv, map_inv, map_outs, map_ins;
    DBuf<int> map_rank, map_is_task, flow_sel, flow_cnt;
    DBuf<unsigned char> map_itype, map_tmp;
    DBuf<uint64_t> map_scratch;  // device vector behind ks_get_task_mapping
    DBuf<ks_flow> flow_recs;
    // ---- cell solver (ks_cell.h): one workgroup per small graph
    bool cell_layout = false;           // the CSR was built cell-major (the cell solver's node order)
    std::vector<int64_t> cell_off;      // node-id partition into independent cells (ks_batch); empty: one
    std::vector<CellDesc> h_cells;      // per cell: its class bounds in internal ids
    int cell_max = 0;                   // largest cell (node slots)
    DBuf<CellDesc> cells;
    DBuf<int> cl_lists, cl_rln;
    DBuf<long long> cl_rlp;
    DBuf<CellOut> cl_out;
    DBuf<CellPos> cl_pos;               // compact positions (k_cell_pack / k_cell_unpack)
    DBuf<int> cl_bad;
    bool cell_refused = false;          // the graph's values do not fit the compact record: engine until reload
    size_t lds_limit = 0;               // the device's opt-in LDS per workgroup (sizes the cells)
    bool fb_active = false;             // a per-cell fallback solve is running (engine order, failing cells cold)
    std::vector<int> fb_cells;          // the cells it re-solves
    DBuf<long long> fb_rng;             // their node-slot ranges on the device
    DBuf<unsigned long long> fb_cnt;    // arc + node slots k_fb_reset restarted cold
    std::vector<CellOut> h_cell_out;
    // ---- scheduler-side sweeps (ks_sched.hip)
    DBuf<int> sched_i;                  // int scratch
    DBuf<unsigned long long> sched_u;   // u64 scratch
    DBuf<unsigned char> sched_b;        // byte scratch
    DBuf<ks_sched_delta> sched_d;

    SchedDev schd() const {
        SchedDev d{};
        d.ncap = (int)ncap;
        d.nstore = nstore;
        d.perm = perm.p;
        d.iperm = iperm.p;
        d.n_alive = n_alive.p;
        d.n_type = n_type.p;
        d.n_bind = n_bind.p;
        d.hi = h_sctl ? h_sctl->hi : 0;
        d.a_alive = a_alive.p;
        d.a_type = a_type.p;
        d.a_src = a_src.p;
        d.a_dst = a_dst.p;
        d.a_cost = a_cost.p;
        d.fwd = fwd.p;
        d.first = first.p;
        d.pos = pos.p;
        d.ent = ent.p;
        d.mult = mult;
        d.csr_valid = csr_valid ? 1 : 0;
        return d;
    }

    ~EngineImpl() {
        if (stream) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(stream);
        }
        n_supply.release(); n_type.release(); n_alive.release(); n_fresh.release(); n_cshift.release(); n_lastrm.release();
        n_hint.release(); n_grow.release(); n_bind.release(); a_type.release(); sched_i.release(); sched_u.release();
        sched_b.release(); sched_d.release();
        a_src.release(); a_dst.release(); fwd.release(); free_stack.release(); a_low.release(); a_cap.release();
        a_cost.release(); a_alive.release(); hkey.release(); hval.release(); hlast.release(); sctl.release();
        d_recs.release(); d_edits.release(); rec_ent.release();
        first.release(); pos.release(); ent.release(); used.release(); scur.release(); perm.release(); iperm.release();
        excess.release(); nd.release(); cpos.release(); crev.release(); cyc.release(); cyc64.release();
        keys_in.release(); keys_out.release(); vals_in.release(); vals_out.release(); pos_of.release(); deg.release();
        capv.release(); capi.release(); rs.release(); sort_tmp.release(); cls.release(); nsel.release();
        for (auto& b : cls_list) b.release();
        sel_tmp.release(); hitems.release(); citems.release(); hnchunks.release(); q_unsat.release(); q_arrive.release();
        q_req.release(); q_taken.release(); q_min.release(); inbox.release(); part.release(); flows.release(); vbal.release();
        flags.release(); hubflags.release(); ctr.release(); xl.release(); xl2.release(); bx.release(); fl.release(); fdef.release(); aug_req.release(); ctl.release(); saved_flows.release(); p_slot.release();
        map_outv.release(); map_inv.release(); map_outs.release(); map_ins.release(); map_rank.release();
        map_is_task.release(); flow_sel.release(); flow_cnt.release(); map_itype.release(); map_tmp.release();
        map_scratch.release(); flow_recs.release();
        cells.release(); cl_lists.release(); cl_rln.release(); cl_rlp.release(); cl_out.release(); cl_pos.release();
        cl_bad.release(); fb_rng.release();
        if (h_ctl) (void)hipHostFree(h_ctl);
        for (auto* h : h_cyc)
            if (h) (void)hipHostFree(h);
        for (auto& c : cev)
            for (auto& e : c)
                if (e) (void)hipEventDestroy(e);
        for (auto& c : fev)
            for (auto& e : c)
                if (e) (void)hipEventDestroy(e);
        for (auto& e : cdone)
            if (e) (void)hipEventDestroy(e);
        if (cstart) (void)hipEventDestroy(cstart);
        if (h_scr) (void)hipHostFree(h_scr);
        if (h_sctl) (void)hipHostFree(h_sctl);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : kev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : fin_ev)
            if (e) (void)hipEventDestroy(e);
        fb_cnt.release();
        if (stream) (void)hipStreamDestroy(stream);
    }

    StoreDev sd() const {
        StoreDev d{};
        d.ncap = (int)ncap;
        d.n_supply = n_supply.p;
        d.n_type = n_type.p;
        d.n_alive = n_alive.p;
        d.n_fresh = n_fresh.p;
        d.n_cshift = n_cshift.p;
        d.n_lastrm = n_lastrm.p;
        d.n_grow = n_grow.p;
        d.n_bind = n_bind.p;
        d.perm = perm.p;
        d.acap = (int)acap;
        d.a_src = a_src.p;
        d.a_dst = a_dst.p;
        d.a_low = a_low.p;
        d.a_cap = a_cap.p;
        d.a_cost = a_cost.p;
        d.a_type = a_type.p;
        d.a_alive = a_alive.p;
        d.fwd = fwd.p;
        d.free_stack = free_stack.p;
        d.hmask = (int)(hcap - 1);
        d.hkey = hkey.p;
        d.hval = hval.p;
        d.hlast = hlast.p;
        d.nn = nn;
        d.first = first.p;
        d.used = used.p;
        d.scur = scur.p;
        d.pos = pos.p;
        d.ent = ent.p;
        d.excess = excess.p;
        d.mult = mult;
        d.csr_valid = csr_valid ? 1 : 0;
        d.ctl = sctl.p;
        return d;
    }

    DG dg() const {
        DG g{};
        g.n = nn;
        g.m = 0;
        g.hub_base = hub_base;
        g.first = first.p;
        g.pos = pos.p;
        g.excess = excess.p;
        g.p0 = nd.p;
        g.p1 = nd.p ? nd.p + 2 : nullptr;
        g.dist = nd.p ? nd.p + 1 : nullptr;
        g.inbox = inbox.p;
        for (int c = 0; c <= NGC; ++c) {
            g.obeg[c] = obeg[c];
            g.wbeg[c] = wbeg[c];
        }
        for (int c = 0; c < NGC; ++c) g.oend[c] = oend[c];
        g.hitems = hitems.p;
        g.nhitems = nhitems;
        g.citems = citems.p;
        g.ncitems = ncitems;
        g.ncls_c = ncls[CCLS];
        g.sw_clsb = sweep_cls_blocks();
        g.nheavy = nheavy;
        g.hnchunks = hnchunks.p;
        g.xl = xl.p;
        g.xl2 = xl2.p;
        g.bx = bx.p;
        g.fl = fl.p;
        g.fl_cap = (int)(fl.n / 3);
        g.fdef = fdef.p;
        g.npos = (int)m2cap;
        g.aug_req = aug_req.p;
        g.q_req = q_req.p;
        g.q_taken = q_taken.p;
        g.q_min = q_min.p;
        g.q_unsat = q_unsat.p;
        g.q_arrive = q_arrive.p;
        const int hs = std::max(1, nheavy);
        const size_t fs = std::max(1, hub_base);
        for (int k = 0; k < 6; ++k) {
            Front f{flags.p + k * fs, hubflags.p + (size_t)k * hs};
            if (k < 3) g.sf[k] = f;
            else g.bf[k - 3] = f;
        }
        g.ctl = ctl.p;
        g.ctr = ctr.p;
        return g;
    }
    int window_grid() const { return nhitems + std::max(1, (wbeg[NGC] + WPB - 1) / WPB); }
    // Bellman-Ford rounds: HSPLIT workgroups per hub chunk, then the windows / chunk items
    int dense_grid() const { return nhitems * HSPLIT + std::max(1, (wbeg[CCLS] + ncitems + WPB - 1) / WPB); }
    int sweep_cls_blocks() const { return std::max(1, (wbeg[CCLS] + WPW * WPB - 1) / (WPW * WPB)); }
    // sweeps: hub chunks, class-window blocks, one wave per chunked-class node
    int sweep_grid() const {
        return nhitems + sweep_cls_blocks() + ncls[CCLS];
    }
    int sparse_grid() const {
        return nhitems * HSPLIT + std::max(1, (wbeg[CCLS] + ncitems + WPW * WPB - 1) / (WPW * WPB));
    }
    int hi() const { return h_sctl->hi; }
};

#define KS_CHECK(expr)                                                   \
    do {                                                                 \
        hipError_t _e = (expr);                                          \
        if (_e != hipSuccess) {                                          \
            err = std::string(#expr) + ": " + hipGetErrorString(_e);     \
            return KS_E_DEVICE;                                          \
        }                                                                \
    } while (0)

// A hot kernel of the solve in the record layout the solve reads.
#define KS_HOT(CPV, K, GRID, BLKS, ST, ...)                                                     \
    do {                                                                                        \
        if (CPV) K<true><<<dim3(GRID), dim3(BLKS), 0, ST>>>(__VA_ARGS__);                      \
        else K<false><<<dim3(GRID), dim3(BLKS), 0, ST>>>(__VA_ARGS__);                         \
    } while (0)

Engine::Engine() : p_(new EngineImpl) {}
Engine::~Engine() { delete p_; }
int Engine::device() const { return p_->device; }

int Engine::init(int device, const ks_opts& opts, std::string& err) {
    EngineImpl& s = *p_;
    s.device = device;
    s.opts = opts;
    int ndev = 0;
    KS_CHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        err = "device index out of range";
        return KS_E_DEVICE;
    }
    KS_CHECK(hipSetDevice(device));
    KS_CHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    {   // LDS one workgroup may declare (the cell solver's size limit; 160 KiB on gfx950)
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, device) != hipSuccess || v <= 0)
            KS_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
        s.lds_limit = (size_t)std::max(v, 0);
    }
    for (auto& e : s.ev) KS_CHECK(hipEventCreate(&e));
    for (auto& e : s.kev) KS_CHECK(hipEventCreate(&e));
    for (auto& e : s.fin_ev) KS_CHECK(hipEventCreate(&e));
    for (auto& c : s.cev)
        for (auto& e : c) KS_CHECK(hipEventCreate(&e));
    for (auto& c : s.fev)
        for (auto& e : c) KS_CHECK(hipEventCreate(&e));
    for (auto& e : s.cdone) KS_CHECK(hipEventCreate(&e));
    KS_CHECK(hipEventCreate(&s.cstart));
    for (int i = 0; i < CYC_SLOTS; ++i) {
        KS_CHECK(hipHostMalloc(&s.h_cyc[i], sizeof(Ctl), hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(s.h_cyc[i], 0, sizeof(Ctl));
        KS_CHECK(hipHostGetDevicePointer((void**)&s.d_cyc[i], s.h_cyc[i], 0));
    }
    KS_CHECK(s.ctl.ensure(1));
    KS_CHECK(s.ctr.ensure(CTR_SHARDS * NCTR));
    KS_CHECK(s.xl.ensure(AUG_KMAX));
    KS_CHECK(s.xl2.ensure(AUG_K2));
    KS_CHECK(s.bx.ensure(BX_CAP));
    KS_CHECK(s.fdef.ensure(FDEF_CAP));
    KS_CHECK(s.sctl.ensure(1));
    KS_CHECK(hipMemset(s.sctl.p, 0, sizeof(StoreCtl)));
    KS_CHECK(hipHostMalloc(&s.h_ctl, sizeof(Ctl)));
    KS_CHECK(hipHostMalloc(&s.h_scr, 4 * sizeof(long long)));
    KS_CHECK(hipHostMalloc(&s.h_sctl, sizeof(StoreCtl)));
    std::memset(s.h_sctl, 0, sizeof(StoreCtl));
    return KS_OK;
}

// ------------------------------------------------------------------ store ---
static int read_sctl(EngineImpl& s, std::string& err) {
    KS_CHECK(hipMemcpyAsync(s.h_sctl, s.sctl.p, sizeof(StoreCtl), hipMemcpyDeviceToHost, s.stream));
    KS_CHECK(hipStreamSynchronize(s.stream));
    return KS_OK;
}

// Node store covers slots [0, need).
static int ensure_nodes(EngineImpl& s, int64_t need, std::string& err) {
    if (need <= s.nstore) return KS_OK;
    const int64_t cap = std::max<int64_t>(need + need / 8 + 64, 1024);
    hipStream_t st = s.stream;
    KS_CHECK(s.n_supply.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_type.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_alive.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_fresh.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_cshift.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_lastrm.grow(cap, s.nstore, 0xff, st));
    KS_CHECK(s.n_hint.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_grow.grow(cap, s.nstore, 0, st));
    KS_CHECK(s.n_bind.grow(cap, s.nstore, 0, st));
    s.nstore = cap;
    return KS_OK;
}

// Arc table holds slots [0, need).
static int ensure_arcs(EngineImpl& s, int64_t need, std::string& err) {
    if (need <= s.acap) return KS_OK;
    if (need >= (1LL << 30)) {
        err = "arc table beyond 2^30 slots";
        return KS_E_RANGE;
    }
    const int64_t cap = std::max<int64_t>(need + need / 4 + 64, 4096);
    hipStream_t st = s.stream;
    const int64_t keep = s.acap;
    KS_CHECK(s.a_src.grow(cap, keep, 0, st));
    KS_CHECK(s.a_dst.grow(cap, keep, 0, st));
    KS_CHECK(s.a_low.grow(cap, keep, 0, st));
    KS_CHECK(s.a_cap.grow(cap, keep, 0, st));
    KS_CHECK(s.a_cost.grow(cap, keep, 0, st));
    KS_CHECK(s.a_alive.grow(cap, keep, 0, st));
    KS_CHECK(s.a_type.grow(cap, keep, 0, st));
    KS_CHECK(s.fwd.grow(cap, keep, 0xff, st));
    KS_CHECK(s.free_stack.grow(cap, keep, 0, st));
    KS_CHECK(s.flows.grow(cap, keep, 0, st));
    s.acap = cap;
    return KS_OK;
}

// Hash index with room for `extra` more keys at load ≤ 1/2 (tombstones count).
static int ensure_hash(EngineImpl& s, int64_t extra, std::string& err) {
    const int64_t live = s.h_sctl->live, tombs = s.h_sctl->tombs;
    if (s.hcap && 2 * (live + tombs + extra) <= s.hcap) return KS_OK;
    int64_t cap = s.hcap ? s.hcap : 1024;
    while (cap < 4 * (live + extra) + 1024) cap <<= 1;
    if (cap > (1LL << 31)) {
        err = "hash index beyond 2^31 entries";
        return KS_E_RANGE;
    }
    KS_CHECK(s.hkey.ensure(cap));
    KS_CHECK(s.hval.ensure(cap));
    KS_CHECK(s.hlast.ensure(cap));
    s.hcap = cap;
    KS_CHECK(store_rehash(s.sd(), s.stream));
    return read_sctl(s, err);
}

static int run_apply(EngineImpl& s, const NodeEdit* edits, size_t ne, const ks_delta* recs, size_t k,
                     std::string& err) {
    hipStream_t st = s.stream;
    size_t narc = 0;
    for (size_t i = 0; i < k; ++i) narc += recs[i].kind == KS_ADD_ARC || recs[i].kind == KS_UPDATE_ARC;
    int rc = ensure_arcs(s, (int64_t)s.hi() + (int64_t)narc, err);
    if (rc == KS_OK) rc = ensure_hash(s, (int64_t)narc, err);
    if (rc) return rc;
    KS_CHECK(s.d_recs.ensure(std::max<size_t>(k, 1)));
    KS_CHECK(s.rec_ent.ensure(std::max<size_t>(k, 1)));
    KS_CHECK(s.d_edits.ensure(std::max<size_t>(ne, 1)));
    const auto t0 = std::chrono::steady_clock::now();
    if (k) KS_CHECK(hipMemcpyAsync(s.d_recs.p, recs, k * sizeof(ks_delta), hipMemcpyHostToDevice, st));
    if (ne) KS_CHECK(hipMemcpyAsync(s.d_edits.p, edits, ne * sizeof(NodeEdit), hipMemcpyHostToDevice, st));
    const auto t1 = std::chrono::steady_clock::now();
    KS_CHECK(store_apply(s.sd(), s.d_recs.p, (int)k, s.rec_ent.p, s.d_edits.p, (int)ne, st));
    rc = read_sctl(s, err);
    if (rc) return rc;
    if (s.opts.log_cycles) {
        const auto t2 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "apply: upload call %.3f ms (%.1f MB), store kernels + wait %.3f ms\n",
                     std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     1e-6 * (double)(k * sizeof(ks_delta) + ne * sizeof(NodeEdit)),
                     std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
    if (s.h_sctl->overflow & 12) {
        err = "store index or table exhausted";
        return KS_E_DEVICE;
    }
    if (s.h_sctl->overflow) {   // a full segment or a node beyond the build: rebuild from the table
        s.csr_valid = false;
        KS_CHECK(hipMemsetAsync(&s.sctl.p->overflow, 0, sizeof(int), st));
        s.h_sctl->overflow = 0;
    }
    if (k || ne) s.solved = false;
    return KS_OK;
}

int Engine::load(int64_t nslots, const int64_t* supply, const uint8_t* type, const uint8_t* alive, const ks_arc* arcs,
                 size_t m, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    if (nslots >= (1LL << 30) || m >= (1ULL << 29)) {
        err = "graph too large for 32-bit CSR indices";
        return KS_E_RANGE;
    }
    int rc = ensure_nodes(s, std::max<int64_t>(nslots, 1), err);
    if (rc) return rc;
    s.nslots = nslots;
    // empty store
    KS_CHECK(hipMemsetAsync(s.n_alive.p, 0, s.nstore, st));
    KS_CHECK(hipMemsetAsync(s.n_supply.p, 0, s.nstore * sizeof(long long), st));
    KS_CHECK(hipMemsetAsync(s.n_type.p, 0, s.nstore, st));
    KS_CHECK(hipMemsetAsync(s.n_fresh.p, 0, s.nstore, st));
    KS_CHECK(hipMemsetAsync(s.n_cshift.p, 0, s.nstore * sizeof(unsigned long long), st));
    KS_CHECK(hipMemsetAsync(s.n_hint.p, 0, s.nstore * sizeof(int), st));
    KS_CHECK(hipMemsetAsync(s.n_grow.p, 0, s.nstore, st));
    KS_CHECK(hipMemsetAsync(s.n_bind.p, 0, s.nstore * sizeof(unsigned long long), st));
    if (nslots) {
        KS_CHECK(hipMemcpyAsync(s.n_supply.p, supply, nslots * sizeof(long long), hipMemcpyHostToDevice, st));
        KS_CHECK(hipMemcpyAsync(s.n_type.p, type, nslots, hipMemcpyHostToDevice, st));
        KS_CHECK(hipMemcpyAsync(s.n_alive.p, alive, nslots, hipMemcpyHostToDevice, st));
    }
    if (s.acap) {
        KS_CHECK(hipMemsetAsync(s.a_alive.p, 0, s.acap, st));
        KS_CHECK(hipMemsetAsync(s.fwd.p, 0xff, s.acap * sizeof(int), st));
        KS_CHECK(hipMemsetAsync(s.a_low.p, 0, s.acap * sizeof(long long), st));
    }
    KS_CHECK(hipMemsetAsync(s.sctl.p, 0, sizeof(StoreCtl), st));
    std::memset(s.h_sctl, 0, sizeof(StoreCtl));
    s.csr_valid = false;
    s.incremental = false;
    s.rebuilds = 0;
    s.solved = false;
    s.has_prev = false;
    s.cell_refused = false;
    rc = ensure_arcs(s, (int64_t)m, err);
    if (rc) return rc;
    if (s.hcap) {   // clear the index (keeps its size)
        KS_CHECK(hipMemsetAsync(s.hkey.p, 0, s.hcap * sizeof(unsigned long long), st));
        KS_CHECK(hipMemsetAsync(s.hval.p, 0xff, s.hcap * sizeof(int), st));
        KS_CHECK(hipMemsetAsync(s.hlast.p, 0xff, s.hcap * sizeof(int), st));
    }
    // the arcs enter as ADD_ARC records of one stream (duplicates: the last wins)
    std::vector<ks_delta> recs(m);
    for (size_t i = 0; i < m; ++i) {
        ks_delta& d = recs[i];
        std::memset(&d, 0, sizeof(d));
        d.kind = KS_ADD_ARC;
        d.type = arcs[i].type;
        d.src = arcs[i].src;
        d.dst = arcs[i].dst;
        d.low = arcs[i].low;
        d.cap = arcs[i].cap;
        d.cost = arcs[i].cost;
    }
    return run_apply(s, nullptr, 0, recs.data(), m, err);
}

int Engine::apply(const NodeEdit* edits, size_t ne, const ks_delta* recs, size_t k, int64_t nslots,
                  std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    int rc = ensure_nodes(s, std::max<int64_t>(nslots, 1), err);
    if (rc) return rc;
    s.nslots = std::max(s.nslots, nslots);
    s.incremental = true;
    return run_apply(s, edits, ne, recs, k, err);
}

int64_t Engine::live_arcs() const { return p_->h_sctl ? p_->h_sctl->live : 0; }
bool Engine::solved() const { return p_->solved; }

void Engine::store_stats(ks_store_stats* o) const {
    const EngineImpl& s = *p_;
    std::memset(o, 0, sizeof(*o));
    if (!s.h_sctl) return;
    o->live_arcs = s.h_sctl->live;
    o->inserted = s.h_sctl->inserted;
    o->updated = s.h_sctl->updated;
    o->killed = s.h_sctl->killed;
    o->superseded = s.h_sctl->superseded;
    o->rebuilds = s.rebuilds;
    o->residual_slots = s.m2cap;
}

// Cell-major internal ids for the cell solver (ks_cell.h): every cell (a ks_batch
// graph, or the whole graph) is one contiguous id range, its nodes grouped by the
// cell solver's degree classes (cell_class of the segment capacity). Slots past the
// partition belong to the last cell. Computed on the host from the capacities.
static int cell_order(EngineImpl& s, int64_t ncap, std::string& err) {
    hipStream_t st = s.stream;
    std::vector<int> capv(ncap);
    if (ncap) KS_CHECK(hipMemcpyAsync(capv.data(), s.capv.p, ncap * sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    const size_t k = s.cell_off.size() >= 2 ? s.cell_off.size() - 1 : 1;
    std::vector<int64_t> bound(k + 1, 0);   // slot bounds of each cell
    for (size_t i = 1; i < k; ++i) bound[i] = std::min<int64_t>(ncap, std::max<int64_t>(0, s.cell_off[i]));
    bound[k] = ncap;
    std::vector<int> cnt(k * CELL_NCLS, 0);
    std::vector<unsigned char> cls(ncap);
    for (size_t c = 0; c < k; ++c)
        for (int64_t v = bound[c]; v < bound[c + 1]; ++v) {
            cls[v] = (unsigned char)cell_class(capv[v]);
            ++cnt[c * CELL_NCLS + cls[v]];
        }
    s.h_cells.assign(k, CellDesc{});
    std::vector<int> next(k * CELL_NCLS);
    int o = 0, mx = 0;
    for (size_t c = 0; c < k; ++c) {
        const int b = o;
        for (int q = 0; q < CELL_NCLS; ++q) {
            s.h_cells[c].cb[q] = o;
            next[c * CELL_NCLS + q] = o;
            o += cnt[c * CELL_NCLS + q];
        }
        s.h_cells[c].cb[CELL_NCLS] = o;
        mx = std::max(mx, o - b);
    }
    std::vector<int> perm(ncap);
    for (size_t c = 0; c < k; ++c)
        for (int64_t v = bound[c]; v < bound[c + 1]; ++v) perm[v] = next[c * CELL_NCLS + cls[v]]++;
    if (ncap) KS_CHECK(hipMemcpyAsync(s.perm.p, perm.data(), ncap * sizeof(int), hipMemcpyHostToDevice, st));
    s.cell_max = mx;
    for (int c = 0; c <= NGC; ++c) s.ncls[c] = 0;
    for (int c = 0; c <= NGC; ++c) s.obeg[c] = s.wbeg[c] = 0;
    for (int c = 0; c < NGC; ++c) s.oend[c] = 0;
    s.nheavy = 0;
    s.hub_base = (int)ncap;
    s.nn = (int)ncap;
    const int nn = (int)ncap;
    KS_CHECK(s.cells.ensure(k));
    KS_CHECK(hipMemcpyAsync(s.cells.p, s.h_cells.data(), k * sizeof(CellDesc), hipMemcpyHostToDevice, st));
    KS_CHECK(s.cl_lists.ensure(2 * (size_t)std::max(nn, 1)));
    KS_CHECK(s.cl_rln.ensure(std::max(nn, 1)));
    KS_CHECK(s.cl_rlp.ensure(std::max(nn, 1)));
    KS_CHECK(s.cl_out.ensure(k));
    KS_CHECK(s.cl_bad.ensure(1));
    s.h_cell_out.resize(k);
    return KS_OK;
}

// ------------------------------------------------------------------ build ---
static int build(EngineImpl& s, std::string& err) {
    hipStream_t st = s.stream;
    const int hi = s.hi();
    const int64_t spare = s.incremental ? std::max<int64_t>(64, s.nslots / 16) : 0;
    const int64_t ncap = s.nslots + spare;
    int rc = ensure_nodes(s, ncap, err);
    if (rc) return rc;
    s.ncap = ncap;
    s.mult = ncap + 1;
    KS_CHECK(s.deg.ensure(std::max<int64_t>(ncap, 1)));
    KS_CHECK(s.capv.ensure(std::max<int64_t>(ncap, 1)));
    KS_CHECK(s.cls.ensure(std::max<int64_t>(ncap, 1)));
    KS_CHECK(s.perm.ensure(std::max<int64_t>(ncap, 1)));
    for (auto& b : s.cls_list) KS_CHECK(b.ensure(std::max<int64_t>(ncap, 1)));
    KS_CHECK(s.nsel.ensure(NGC + 1));
    KS_CHECK(s.part.ensure(2 * 4096));
    KS_CHECK(hipMemsetAsync(s.deg.p, 0, ncap * sizeof(int), st));
    // 1. degrees → segment capacities → classes
    if (hi)
        hipLaunchKernelGGL(k_degree, dim3(grid_for(hi)), dim3(BLK), 0, st, hi, (const unsigned char*)s.a_alive.p,
                           (const int*)s.a_src.p, (const int*)s.a_dst.p, s.deg.p);
    hipLaunchKernelGGL(k_capacity, dim3(grid_for(ncap)), dim3(BLK), 0, st, (int)ncap, (int)s.nstore,
                       (const int*)s.deg.p, (const unsigned char*)s.n_alive.p, (const unsigned char*)s.n_type.p,
                       s.incremental ? 1 : 0, s.n_hint.p,
                       s.n_grow.p, s.capv.p, s.cls.p);
    if (s.cell_layout) {
        int rc = cell_order(s, ncap, err);   // perm, cell descriptors; no lane-group classes or hubs
        if (rc) return rc;
    } else {
        {
            hipcub::CountingInputIterator<int> it(0);
            size_t tmp = 0, t2 = 0;
            for (unsigned char c = 0; c <= NGC; ++c) {
                KS_CHECK(hipcub::DeviceSelect::If(nullptr, t2, it, s.cls_list[c].p, s.nsel.p + c, (int)ncap,
                                                  ClassIs{s.cls.p, c}, st));
                tmp = std::max(tmp, t2);
            }
            KS_CHECK(s.sel_tmp.ensure(tmp));
            for (unsigned char c = 0; c <= NGC; ++c) {
                t2 = tmp;
                KS_CHECK(hipcub::DeviceSelect::If(s.sel_tmp.p, t2, it, s.cls_list[c].p, s.nsel.p + c, (int)ncap,
                                                  ClassIs{s.cls.p, c}, st));
            }
        }
        KS_CHECK(hipMemcpyAsync(s.ncls, s.nsel.p, (NGC + 1) * sizeof(int), hipMemcpyDeviceToHost, st));
        KS_CHECK(hipStreamSynchronize(st));
        s.nheavy = s.ncls[NGC];
        // 2. internal ids: classes in order, each padded to whole 64-node blocks, hubs last
        {
            int o = 0, wv = 0;
            for (int c = 0; c < NGC; ++c) {
                s.obeg[c] = o;
                s.oend[c] = o + s.ncls[c];
                s.wbeg[c] = wv;
                const int pad = (s.ncls[c] + 63) / 64 * 64;
                o += pad;
                wv += pad / win_slots(c);
            }
            s.obeg[NGC] = o;
            s.wbeg[NGC] = wv;
            s.hub_base = o;
            s.nn = o + s.nheavy;
        }
        for (int c = 0; c <= NGC; ++c)
            if (s.ncls[c])
                hipLaunchKernelGGL(k_make_perm, dim3(grid_for(s.ncls[c])), dim3(BLK), 0, st, s.ncls[c],
                                   c < NGC ? s.obeg[c] : s.hub_base, (const int*)s.cls_list[c].p, s.perm.p);
    }
    const int nn = s.nn;
    KS_CHECK(s.capi.ensure(nn + 1));
    KS_CHECK(s.iperm.ensure(nn + 1));
    KS_CHECK(s.first.ensure(nn + 1));
    KS_CHECK(s.used.ensure(std::max(nn, 1)));
    KS_CHECK(s.scur.ensure(std::max(nn, 1)));
    KS_CHECK(hipMemsetAsync(s.scur.p, 0, std::max(nn, 1) * sizeof(int), st));
    KS_CHECK(s.rs.ensure(nn + 1));
    KS_CHECK(hipMemsetAsync(s.capi.p, 0, (nn + 1) * sizeof(int), st));
    KS_CHECK(hipMemsetAsync(s.iperm.p, 0xff, (nn + 1) * sizeof(int), st));
    hipLaunchKernelGGL(k_capi, dim3(grid_for(ncap)), dim3(BLK), 0, st, (int)ncap, (const int*)s.perm.p,
                       (const int*)s.capv.p, s.capi.p, s.iperm.p);
    {   // first = exclusive scan of the capacities (nn + 1 entries: first[nn] = Σ)
        size_t t = 0;
        KS_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t, s.capi.p, s.first.p, nn + 1, st));
        KS_CHECK(s.sort_tmp.ensure(std::max<size_t>(t, s.sort_tmp.n)));
        t = s.sort_tmp.n;
        KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.sort_tmp.p, t, s.capi.p, s.first.p, nn + 1, st));
    }
    int m2c = 0;
    KS_CHECK(hipMemcpyAsync(&m2c, s.first.p + nn, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    s.m2cap = m2c;
    const int64_t m2cap = std::max<int64_t>(m2c, 1);
    KS_CHECK(s.pos.ensure(m2cap));
    KS_CHECK(s.ent.ensure(m2cap));
    KS_CHECK(s.excess.ensure(std::max(nn, 1)));
    KS_CHECK(s.nd.ensure(4 * (size_t)std::max(nn, 1)));
    if (nn)
        hipLaunchKernelGGL(k_node_bounds, dim3(grid_for(nn)), dim3(BLK), 0, st, nn, (const int*)s.first.p, s.nd.p);
    if (m2c)
        hipLaunchKernelGGL(k_inert_all, dim3(grid_for(m2c)), dim3(BLK), 0, st, (long long)m2c, nn,
                           (const int*)s.first.p, s.pos.p, s.ent.p);
    // 3. live arcs into their segments, ordered by tail (radix sort of 2·hi keys)
    const int64_t m2 = 2 * (int64_t)hi;
    if (s.acap) KS_CHECK(hipMemsetAsync(s.fwd.p, 0xff, s.acap * sizeof(int), st));
    if (m2) {
        KS_CHECK(s.keys_in.ensure(m2));
        KS_CHECK(s.keys_out.ensure(m2));
        KS_CHECK(s.vals_in.ensure(m2));
        KS_CHECK(s.vals_out.ensure(m2));
        KS_CHECK(s.pos_of.ensure(m2));
        int bits = 1;
        while ((1LL << bits) <= nn + 1) ++bits;
        hipLaunchKernelGGL(k_pos_keys, dim3(grid_for(hi)), dim3(BLK), 0, st, hi, nn,
                           (const unsigned char*)s.a_alive.p, (const int*)s.a_src.p, (const int*)s.a_dst.p,
                           (const int*)s.perm.p, s.keys_in.p, s.vals_in.p);
        size_t t = 0;
        KS_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, t, s.keys_in.p, s.keys_out.p, s.vals_in.p,
                                                    s.vals_out.p, (int)m2, 0, bits, st));
        KS_CHECK(s.sort_tmp.ensure(std::max<size_t>(t, s.sort_tmp.n)));
        t = s.sort_tmp.n;
        KS_CHECK(hipcub::DeviceRadixSort::SortPairs(s.sort_tmp.p, t, s.keys_in.p, s.keys_out.p, s.vals_in.p,
                                                    s.vals_out.p, (int)m2, 0, bits, st));
        hipLaunchKernelGGL(k_first, dim3(grid_for(nn + 1)), dim3(BLK), 0, st, nn, (long long)m2,
                           (const unsigned*)s.keys_out.p, s.rs.p);
        hipLaunchKernelGGL(k_fill_csr, dim3(grid_for(m2)), dim3(BLK), 0, st, (long long)m2, nn,
                           (const unsigned*)s.keys_out.p, (const int*)s.vals_out.p, (const int*)s.rs.p,
                           (const int*)s.first.p, (const int*)s.perm.p, (const int*)s.a_src.p, (const int*)s.a_dst.p,
                           (const long long*)s.a_low.p, (const long long*)s.a_cap.p, (const long long*)s.a_cost.p,
                           s.mult, s.pos.p, s.ent.p, s.fwd.p, s.pos_of.p);
        hipLaunchKernelGGL(k_fill_rev, dim3(grid_for(m2)), dim3(BLK), 0, st, (long long)m2, nn,
                           (const unsigned*)s.keys_out.p, (const int*)s.vals_out.p, (const int*)s.pos_of.p, s.pos.p);
        hipLaunchKernelGGL(k_used, dim3(grid_for(nn)), dim3(BLK), 0, st, nn, (const int*)s.rs.p, s.used.p);
    } else {
        KS_CHECK(hipMemsetAsync(s.used.p, 0, std::max(nn, 1) * sizeof(int), st));
    }
    // 4. hub chunk table and the chunked class's 64-arc chunks (from the segments)
    {
        std::vector<int> hf(s.nheavy + 1);
        if (s.nheavy) {
            KS_CHECK(hipMemcpyAsync(hf.data(), s.first.p + s.hub_base, (s.nheavy + 1) * sizeof(int),
                                    hipMemcpyDeviceToHost, st));
            KS_CHECK(hipStreamSynchronize(st));
        }
        std::vector<HItem> items;
        std::vector<int> nch(s.nheavy);
        for (int h = 0; h < s.nheavy; ++h) {
            int c = 0;
            for (int b = hf[h]; b < hf[h + 1]; b += CHUNK, ++c)
                items.push_back(HItem{s.hub_base + h, h, b, std::min(b + CHUNK, hf[h + 1])});
            nch[h] = c;
        }
        s.nhitems = (int)items.size();
        KS_CHECK(s.hitems.ensure(items.size()));
        KS_CHECK(s.hnchunks.ensure(s.nheavy));
        KS_CHECK(s.inbox.ensure((size_t)s.nheavy * SHARDS));
        KS_CHECK(s.flags.ensure(6 * (size_t)std::max(1, s.hub_base)));
        KS_CHECK(s.fl.ensure(3 * ((size_t)std::max(1, s.nn) + 4096)));
        KS_CHECK(s.hubflags.ensure(6 * (size_t)std::max(1, s.nheavy)));
        KS_CHECK(hipMemsetAsync(s.flags.p, 0, 6 * (size_t)std::max(1, s.hub_base), st));
        KS_CHECK(hipMemsetAsync(s.hubflags.p, 0, 6 * (size_t)std::max(1, s.nheavy) * sizeof(int), st));
        if (s.nheavy) {
            KS_CHECK(hipMemcpyAsync(s.hitems.p, items.data(), items.size() * sizeof(HItem), hipMemcpyHostToDevice, st));
            KS_CHECK(hipMemcpyAsync(s.hnchunks.p, nch.data(), nch.size() * sizeof(int), hipMemcpyHostToDevice, st));
            KS_CHECK(hipMemsetAsync(s.inbox.p, 0, (size_t)s.nheavy * SHARDS * sizeof(long long), st));
        }
        const int c0 = s.obeg[CCLS], cn = s.ncls[CCLS];
        std::vector<int> cf(cn + 1);
        if (cn) KS_CHECK(hipMemcpyAsync(cf.data(), s.first.p + c0, (cn + 1) * sizeof(int), hipMemcpyDeviceToHost, st));
        KS_CHECK(hipStreamSynchronize(st));
        std::vector<CItem> ci;
        for (int k = 0; k < cn; ++k)
            for (int b = cf[k]; b < cf[k + 1]; b += 64)
                ci.push_back(CItem{c0 + k, b, std::min(b + 64, cf[k + 1]), b == cf[k] ? 1 : 0});
        s.ncitems = (int)ci.size();
        KS_CHECK(s.citems.ensure(std::max<size_t>(1, ci.size())));
        if (!ci.empty())
            KS_CHECK(hipMemcpyAsync(s.citems.p, ci.data(), ci.size() * sizeof(CItem), hipMemcpyHostToDevice, st));
        const int nq = std::max(1, s.nheavy);
        KS_CHECK(s.q_req.ensure(nq));
        KS_CHECK(s.aug_req.ensure(nq));
        KS_CHECK(hipMemsetAsync(s.aug_req.p, 0, nq * sizeof(long long), st));
        KS_CHECK(s.q_taken.ensure(nq));
        KS_CHECK(s.q_min.ensure(nq));
        KS_CHECK(s.q_unsat.ensure(nq));
        KS_CHECK(s.q_arrive.ensure(nq));
        std::vector<long long> qm(nq, INF64);
        KS_CHECK(hipMemcpyAsync(s.q_min.p, qm.data(), nq * sizeof(long long), hipMemcpyHostToDevice, st));
        KS_CHECK(hipMemsetAsync(s.q_req.p, 0, nq * sizeof(long long), st));
        KS_CHECK(hipMemsetAsync(s.q_taken.p, 0, nq * sizeof(long long), st));
        KS_CHECK(hipMemsetAsync(s.q_unsat.p, 0, nq * sizeof(int), st));
        KS_CHECK(hipMemsetAsync(s.q_arrive.p, 0, nq * sizeof(int), st));
        KS_CHECK(hipStreamSynchronize(st));
    }
    s.csr_valid = true;
    ++s.rebuilds;
    return KS_OK;
}

// zero flow, supplies with the lower-bound transform, zero prices
static int cold_reset(EngineImpl& s, std::string& err) {
    hipStream_t st = s.stream;
    const int hi = s.hi();
    if (s.m2cap)
        hipLaunchKernelGGL(k_reset_pos, dim3(grid_for(s.m2cap)), dim3(BLK), 0, st, (long long)s.m2cap,
                           (const int*)s.ent.p, s.pos.p);
    hipLaunchKernelGGL(k_reset_nodes, dim3(grid_for(s.nn)), dim3(BLK), 0, st, s.nn, (int)s.ncap,
                       (const int*)s.iperm.p, (const unsigned char*)s.n_alive.p, (const long long*)s.n_supply.p,
                       s.excess.p, s.nd.p, (s.nd.p + 2));
    if (hi)
        hipLaunchKernelGGL(k_reset_low, dim3(grid_for(hi)), dim3(BLK), 0, st, hi, (const unsigned char*)s.a_alive.p,
                           (const int*)s.a_src.p, (const int*)s.a_dst.p, (const int*)s.perm.p,
                           (const long long*)s.a_low.p, s.excess.p);
    KS_CHECK(hipGetLastError());
    return KS_OK;
}

void Engine::set_cells(const int64_t* off, size_t k) {
    EngineImpl& s = *p_;
    std::vector<int64_t> v;
    if (off && k) v.assign(off, off + k + 1);
    if (v != s.cell_off) {
        s.cell_off.swap(v);
        if (s.cell_layout) s.csr_valid = false;   // the cells are laid out anew by the next build
    }
}

// The cell solver runs when every cell (the ks_batch partition, else the whole
// graph) fits one workgroup's LDS and ks_opts.cell_nodes allows it. Sizes are node
// slots as the build lays them out (the current build's, or the next one's). By
// default a lone graph takes it only up to kCellSingleNodes: one workgroup is one
// CU's VALU, and above that size the multi-kernel engine over the whole chip solves
// a single graph sooner (config 2: ~21 ms vs ~37 ms); a partition's cells run side
// by side on separate CUs, so they take it up to the LDS limit.
constexpr int64_t kCellSingleNodes = 4096;
static bool want_cells(const EngineImpl& s) {
    if (s.opts.cell_nodes < 0 || s.cell_refused || s.fb_active) return false;
    int64_t lim = std::min<int64_t>(cell_max_nodes(s.lds_limit), s.opts.cell_nodes > 0 ? s.opts.cell_nodes : INT32_MAX);
    if (s.opts.cell_nodes == 0 && s.cell_off.size() < 2) lim = std::min(lim, kCellSingleNodes);
    const int64_t ncap =
        s.csr_valid ? s.ncap : s.nslots + (s.incremental ? std::max<int64_t>(64, s.nslots / 16) : 0);
    if (ncap <= 0) return false;
    const size_t k = s.cell_off.size() >= 2 ? s.cell_off.size() - 1 : 1;
    int64_t prev = 0;
    for (size_t i = 1; i <= k; ++i) {
        const int64_t b = i == k ? ncap : std::min<int64_t>(ncap, std::max<int64_t>(prev, s.cell_off[i]));
        if (b - prev > lim) return false;
        prev = b;
    }
    return true;
}

int Engine::set_nodes(const NodeEdit* edits, size_t ne, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    return run_apply(s, edits, ne, nullptr, 0, err);
}

int Engine::task_pu(uint64_t* dev_out, size_t cap, size_t* count, int64_t n_tasks, std::string& err) {
    EngineImpl& s = *p_;
    if (!s.solved) {
        err = "no successful solve";
        return KS_E_INVALID;
    }
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    *count = (size_t)n_tasks;
    if (!dev_out || cap < (size_t)n_tasks || n_tasks == 0) {
        if (dev_out && cap < (size_t)n_tasks) {
            err = "output buffer smaller than the task count";
            return KS_E_INVALID;
        }
        return KS_OK;
    }
    const int64_t m2 = std::max<int64_t>(s.m2cap, 1), ncap = s.ncap;
    const int nn = s.nn;
    KS_CHECK(s.map_outv.ensure(m2));
    KS_CHECK(s.map_inv.ensure(m2));
    KS_CHECK(s.map_outs.ensure(m2));
    KS_CHECK(s.map_ins.ensure(m2));
    KS_CHECK(s.map_itype.ensure(nn + 1));
    KS_CHECK(s.map_rank.ensure(ncap + 1));
    KS_CHECK(s.map_is_task.ensure(ncap + 1));
    KS_CHECK(hipMemsetAsync(s.map_itype.p, 0, nn + 1, st));
    if (s.m2cap)
        hipLaunchKernelGGL(k_unit_vals, dim3(grid_for(s.m2cap)), dim3(BLK), 0, st, (long long)s.m2cap,
                           (const int*)s.ent.p, (const long long*)s.flows.p, s.map_outv.p, s.map_inv.p);
    hipLaunchKernelGGL(k_node_meta, dim3(grid_for(ncap)), dim3(BLK), 0, st, (int)ncap, (const int*)s.perm.p,
                       (const unsigned char*)s.n_type.p, (const unsigned char*)s.n_alive.p, s.map_itype.p,
                       s.map_is_task.p);
    size_t t1 = 0, t2 = 0;
    if (s.m2cap) KS_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, s.map_outv.p, s.map_outs.p, (int)s.m2cap, st));
    KS_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, s.map_is_task.p, s.map_rank.p, (int)ncap, st));
    KS_CHECK(s.map_tmp.ensure(std::max(t1, t2)));
    size_t tt = s.map_tmp.n;
    if (s.m2cap) {
        KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.map_tmp.p, tt, s.map_outv.p, s.map_outs.p, (int)s.m2cap, st));
        tt = s.map_tmp.n;
        KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.map_tmp.p, tt, s.map_inv.p, s.map_ins.p, (int)s.m2cap, st));
    }
    tt = s.map_tmp.n;
    KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.map_tmp.p, tt, s.map_is_task.p, s.map_rank.p, (int)ncap, st));
    hipLaunchKernelGGL(k_task_paths, dim3(grid_for(ncap)), dim3(BLK), 0, st, (int)ncap, nn, (const int*)s.perm.p,
                       (const int*)s.first.p, (const Pos*)s.pos.p,
                       (const long long*)s.map_outv.p, (const long long*)s.map_outs.p,
                       (const long long*)s.map_inv.p, (const long long*)s.map_ins.p, (const int*)s.iperm.p,
                       (const unsigned char*)s.map_itype.p, (const int*)s.map_rank.p,
                       (const int*)s.map_is_task.p, (long long)cap, (unsigned long long*)dev_out);
    KS_CHECK(hipGetLastError());
    KS_CHECK(hipStreamSynchronize(st));
    return KS_OK;
}

int Engine::download(void* host_dst, const void* dev_src, size_t bytes, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    if (bytes) {
        KS_CHECK(hipMemcpyAsync(host_dst, dev_src, bytes, hipMemcpyDeviceToHost, s.stream));
        KS_CHECK(hipStreamSynchronize(s.stream));
    }
    return KS_OK;
}

int Engine::scratch(uint64_t** dev, size_t n, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    KS_CHECK(s.map_scratch.ensure(std::max<size_t>(1, n)));
    *dev = s.map_scratch.p;
    return KS_OK;
}

int Engine::flows(std::vector<ks_flow>& out, std::string& err) {
    EngineImpl& s = *p_;
    if (!s.solved) {
        err = "no successful solve";
        return KS_E_INVALID;
    }
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    const int hi = s.hi();
    out.clear();
    if (!hi) return KS_OK;
    KS_CHECK(s.flow_sel.ensure(hi));
    KS_CHECK(s.flow_cnt.ensure(1));
    hipcub::CountingInputIterator<int> it(0);
    FlowPositive pred{s.a_alive.p, s.flows.p};
    size_t t = 0;
    KS_CHECK(hipcub::DeviceSelect::If(nullptr, t, it, s.flow_sel.p, s.flow_cnt.p, hi, pred, st));
    KS_CHECK(s.map_tmp.ensure(std::max(t, s.map_tmp.n)));
    t = s.map_tmp.n;
    KS_CHECK(hipcub::DeviceSelect::If(s.map_tmp.p, t, it, s.flow_sel.p, s.flow_cnt.p, hi, pred, st));
    int cnt = 0;
    KS_CHECK(hipMemcpyAsync(&cnt, s.flow_cnt.p, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    if (!cnt) return KS_OK;
    KS_CHECK(s.flow_recs.ensure(cnt));
    hipLaunchKernelGGL(k_flow_records, dim3(grid_for(cnt)), dim3(BLK), 0, st, cnt, (const int*)s.flow_sel.p,
                       (const int*)s.a_src.p, (const int*)s.a_dst.p, (const long long*)s.flows.p, s.flow_recs.p);
    out.resize(cnt);
    KS_CHECK(hipMemcpyAsync(out.data(), s.flow_recs.p, cnt * sizeof(ks_flow), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    return KS_OK;
}

// ------------------------------------------------- scheduler-side sweeps ---
int Engine::set_bindings(const uint64_t* task, const uint64_t* pu, size_t k, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    if (!k) return KS_OK;
    std::vector<unsigned long long> ids(task, task + k), vals(pu, pu + k);
    for (size_t i = 0; i < k; ++i)
        if (ids[i] == 0 || (int64_t)ids[i] > s.nstore) {
            err = "binding for a task id beyond the graph";
            return KS_E_INVALID;
        }
    KS_CHECK(s.sched_u.ensure(2 * k));
    hipStream_t st = s.stream;
    KS_CHECK(hipMemcpyAsync(s.sched_u.p, ids.data(), k * 8, hipMemcpyHostToDevice, st));
    KS_CHECK(hipMemcpyAsync(s.sched_u.p + k, vals.data(), k * 8, hipMemcpyHostToDevice, st));
    // the same scatter as the running counts: n_bind[id − 1] = pu
    KS_CHECK(sched_running_counts(s.schd(), s.sched_u.p, s.sched_u.p + k, (int)k, s.n_bind.p, st));
    KS_CHECK(hipStreamSynchronize(st));
    return KS_OK;
}

int Engine::sched_deltas(int commit, std::vector<ks_sched_delta>* out, size_t* count, int64_t n_tasks,
                         std::string& err) {
    EngineImpl& s = *p_;
    if (!s.solved) {
        err = "no successful solve";
        return KS_E_INVALID;
    }
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    uint64_t* dense = nullptr;
    size_t nt = 0;
    int rc = scratch(&dense, std::max<int64_t>(n_tasks, 1), err);
    if (rc == KS_OK) rc = task_pu(n_tasks ? dense : nullptr, n_tasks, &nt, n_tasks, err);   // also is_task / rank
    if (rc) return rc;
    const int64_t ncap = s.ncap;
    if (!n_tasks) {   // no tasks: map arrays were not built; every binding is a preemption
        KS_CHECK(s.map_is_task.ensure(ncap + 1));
        KS_CHECK(s.map_rank.ensure(ncap + 1));
        KS_CHECK(hipMemsetAsync(s.map_is_task.p, 0, (ncap + 1) * sizeof(int), st));
        KS_CHECK(hipMemsetAsync(s.map_rank.p, 0, (ncap + 1) * sizeof(int), st));
    }
    KS_CHECK(s.sched_i.ensure(4 * (ncap + 1) + 4));
    int* pre = s.sched_i.p;
    int* other = pre + (ncap + 1);
    int* pre_pos = other + (ncap + 1);
    int* other_pos = pre_pos + (ncap + 1);
    int* bad = other_pos + (ncap + 1);
    KS_CHECK(hipMemsetAsync(bad, 0, 4 * sizeof(int), st));
    const SchedDev d = s.schd();
    KS_CHECK(sched_delta_kinds(d, s.map_is_task.p, s.map_rank.p, (const unsigned long long*)dense, pre, other, bad, st));
    size_t t = 0;
    KS_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t, pre, pre_pos, (int)ncap + 1, st));
    KS_CHECK(s.map_tmp.ensure(std::max(t, s.map_tmp.n)));
    t = s.map_tmp.n;
    KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.map_tmp.p, t, pre, pre_pos, (int)ncap + 1, st));
    t = s.map_tmp.n;
    KS_CHECK(hipcub::DeviceScan::ExclusiveSum(s.map_tmp.p, t, other, other_pos, (int)ncap + 1, st));
    int h[3] = {0, 0, 0};
    KS_CHECK(hipMemcpyAsync(&h[0], pre_pos + ncap, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipMemcpyAsync(&h[1], other_pos + ncap, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipMemcpyAsync(&h[2], bad, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    if (h[2]) {
        err = "mapping names a destination that is not a PU (graph_manager.go:259-262)";
        return KS_E_VERIFY;
    }
    const int npre = h[0], noth = h[1];
    *count = (size_t)(npre + noth);
    if (!out) return KS_OK;
    KS_CHECK(s.sched_d.ensure(std::max(1, npre + noth)));
    KS_CHECK(sched_delta_emit(d, s.map_rank.p, (const unsigned long long*)dense, pre, pre_pos, other, other_pos, npre,
                              s.sched_d.p, commit, st));
    out->resize(npre + noth);
    if (npre + noth)
        KS_CHECK(hipMemcpyAsync(out->data(), s.sched_d.p, (npre + noth) * sizeof(ks_sched_delta), hipMemcpyDeviceToHost,
                                st));
    KS_CHECK(hipStreamSynchronize(st));
    return KS_OK;
}

int Engine::unsched_costs(const uint64_t* ids, size_t k, int mode, int64_t ucost, int64_t ccost, size_t* changed,
                          std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    const int64_t nb = (s.nstore + 4) & ~3LL;   // byte flags, word-aligned for the atomics
    KS_CHECK(s.sched_b.ensure(nb));
    KS_CHECK(s.sched_i.ensure(4));
    KS_CHECK(hipMemsetAsync(s.sched_b.p, 0, nb, st));
    KS_CHECK(hipMemsetAsync(s.sched_i.p, 0, sizeof(int), st));
    const unsigned long long* dids = nullptr;
    if (ids && k) {
        for (size_t i = 0; i < k; ++i)
            if (ids[i] == 0 || (int64_t)ids[i] > s.nstore) {
                err = "unscheduled aggregator id beyond the graph";
                return KS_E_INVALID;
            }
        KS_CHECK(s.sched_u.ensure(k));
        KS_CHECK(hipMemcpyAsync(s.sched_u.p, ids, k * 8, hipMemcpyHostToDevice, st));
        dids = s.sched_u.p;
    }
    KS_CHECK(sched_unsched_costs(s.schd(), ids ? dids : nullptr, (int)k, s.sched_b.p, mode, ucost, ccost, s.sched_i.p,
                                 st));
    int h = 0;
    KS_CHECK(hipMemcpyAsync(&h, s.sched_i.p, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    if (changed) *changed = (size_t)h;
    if (h) s.solved = false;
    return KS_OK;
}

int Engine::topology_stats(uint64_t mtpp, const uint64_t* pu_ids, const uint64_t* pu_running, size_t k,
                           int64_t sink_slot, uint64_t* slots_below, uint64_t* running_below, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    if (!s.csr_valid) {   // the BFS walks the residual CSR's in-arcs
        int rc = build(s, err);
        if (rc) return rc;
        s.has_prev = false;
        s.solved = false;
    }
    const int64_t ncap = s.ncap, nn = s.nn;
    if (sink_slot < 0 || sink_slot >= ncap || ncap == 0) {
        std::memset(slots_below, 0, s.nslots * sizeof(uint64_t));
        std::memset(running_below, 0, s.nslots * sizeof(uint64_t));
        return KS_OK;
    }
    KS_CHECK(s.sched_u.ensure(3 * (ncap + 1) + 2 * k));
    unsigned long long* cnt = s.sched_u.p;
    unsigned long long* slots = cnt + (ncap + 1);
    unsigned long long* run = slots + (ncap + 1);
    unsigned long long* kid = run + (ncap + 1);
    KS_CHECK(hipMemsetAsync(cnt, 0, 3 * (ncap + 1) * 8, st));
    if (pu_ids && k) {
        for (size_t i = 0; i < k; ++i)
            if (pu_ids[i] == 0 || (int64_t)pu_ids[i] > ncap) {
                err = "PU id beyond the graph";
                return KS_E_INVALID;
            }
        KS_CHECK(hipMemcpyAsync(kid, pu_ids, k * 8, hipMemcpyHostToDevice, st));
        KS_CHECK(hipMemcpyAsync(kid + k, pu_running, k * 8, hipMemcpyHostToDevice, st));
    }
    const SchedDev d = s.schd();
    KS_CHECK(sched_running_counts(d, pu_ids ? kid : nullptr, kid + k, (int)k, cnt, st));
    KS_CHECK(s.sched_i.ensure(3 * (nn + 1) + 2));
    int* lvl = s.sched_i.p;
    int* fa = lvl + (nn + 1);
    int* fb = fa + (nn + 1);
    int* nnext = fb + (nn + 1);
    KS_CHECK(hipMemsetAsync(lvl, 0xff, (nn + 1) * sizeof(int), st));
    int sink_x = 0;
    KS_CHECK(hipMemcpyAsync(&sink_x, s.perm.p + sink_slot, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    const int zero = 0;
    KS_CHECK(hipMemcpyAsync(lvl + sink_x, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    KS_CHECK(hipMemcpyAsync(fa, &sink_x, sizeof(int), hipMemcpyHostToDevice, st));
    int nfront = 1;
    for (int level = 0; nfront > 0 && level <= nn; ++level) {
        KS_CHECK(hipMemsetAsync(nnext, 0, sizeof(int), st));
        KS_CHECK(sched_topo_level(d, fa, nfront, level, lvl, fb, nnext, mtpp, cnt, slots, run, st));
        KS_CHECK(hipMemcpyAsync(&nfront, nnext, sizeof(int), hipMemcpyDeviceToHost, st));
        KS_CHECK(hipStreamSynchronize(st));
        std::swap(fa, fb);
    }
    const int64_t n = std::min<int64_t>(s.nslots, ncap);
    if (n) {
        KS_CHECK(hipMemcpyAsync(slots_below, slots, n * 8, hipMemcpyDeviceToHost, st));
        KS_CHECK(hipMemcpyAsync(running_below, run, n * 8, hipMemcpyDeviceToHost, st));
        KS_CHECK(hipStreamSynchronize(st));
    }
    return KS_OK;
}

int Engine::arcs(std::vector<ks_arc>& out, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    const int hi = s.hi();
    out.clear();
    if (!hi) return KS_OK;
    KS_CHECK(s.flow_sel.ensure(hi));
    KS_CHECK(s.flow_cnt.ensure(1));
    hipcub::CountingInputIterator<int> it(0);
    SlotAlive pred{s.a_alive.p};
    size_t t = 0;
    KS_CHECK(hipcub::DeviceSelect::If(nullptr, t, it, s.flow_sel.p, s.flow_cnt.p, hi, pred, st));
    KS_CHECK(s.map_tmp.ensure(std::max(t, s.map_tmp.n)));
    t = s.map_tmp.n;
    KS_CHECK(hipcub::DeviceSelect::If(s.map_tmp.p, t, it, s.flow_sel.p, s.flow_cnt.p, hi, pred, st));
    int cnt = 0;
    KS_CHECK(hipMemcpyAsync(&cnt, s.flow_cnt.p, sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    if (!cnt) return KS_OK;
    ks_arc* d = nullptr;
    KS_CHECK(hipMalloc(&d, cnt * sizeof(ks_arc)));
    hipLaunchKernelGGL(k_arc_records, dim3(grid_for(cnt)), dim3(BLK), 0, st, cnt, (const int*)s.flow_sel.p,
                       (const int*)s.a_src.p, (const int*)s.a_dst.p, (const long long*)s.a_low.p,
                       (const long long*)s.a_cap.p, (const long long*)s.a_cost.p, (const unsigned char*)s.a_type.p, d);
    out.resize(cnt);
    hipError_t e = hipMemcpyAsync(out.data(), d, cnt * sizeof(ks_arc), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(d);
    KS_CHECK(e);
    return KS_OK;
}

hipStream_t Engine::stream() const { return p_->stream; }

int Engine::cell_sums(const int64_t* off, size_t k, int64_t* dev_cost, int64_t* dev_flow, std::string& err) {
    EngineImpl& s = *p_;
    if (!s.solved) {
        err = "no successful solve";
        return KS_E_INVALID;
    }
    if (k > (size_t)MAX_CELLS) {
        err = "more than 1024 graphs in one union";
        return KS_E_INVALID;
    }
    KS_CHECK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    const int hi = s.hi();
    KS_CHECK(s.sched_u.ensure(k + 1));
    KS_CHECK(hipMemcpyAsync(s.sched_u.p, off, (k + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
    KS_CHECK(hipMemsetAsync(dev_cost, 0, k * sizeof(int64_t), st));
    KS_CHECK(hipMemsetAsync(dev_flow, 0, k * sizeof(int64_t), st));
    if (hi && k)
        hipLaunchKernelGGL(k_cell_sums, dim3(grid_for(hi, 1024)), dim3(BLK), 0, st, hi, (int)k,
                           (const long long*)s.sched_u.p, (const unsigned char*)s.a_alive.p, (const int*)s.a_src.p,
                           (const int*)s.a_dst.p, (const long long*)s.n_supply.p, (const long long*)s.a_cost.p,
                           (const long long*)s.flows.p, (long long*)dev_cost, (long long*)dev_flow);
    KS_CHECK(hipGetLastError());
    KS_CHECK(hipStreamSynchronize(st));
    return KS_OK;
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
    return ms;
}

int Engine::solve(ks_result& res, bool warm, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    const auto t_host0 = std::chrono::steady_clock::now();
    auto wall_s = [&]() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_host0).count();
    };
    hipStream_t st = s.stream;
    // a per-cell fallback carries the cell solver's state (the cells that converged
    // keep their optima; the failing ones restart cold, k_fb_reset)
    const bool fb = s.fb_active;
    const bool use_warm = (warm && s.has_prev) || fb;
    s.solved = false;
    {   // the cell solver's node order, or the multi-kernel engine's (a change rebuilds the CSR)
        const bool cells_now = want_cells(s);
        if (cells_now != s.cell_layout) {
            s.cell_layout = cells_now;
            s.csr_valid = false;
        }
    }
    res.warm_started = use_warm ? 1 : 0;
    res.rebuilt = s.csr_valid ? 0 : 1;
    res.recoveries = 0;
    res.cell_fallbacks = 0;
    res.cycles_cancelled = 0;
    res.fb_resets = 0;
    res.cycles_rejected = 0;
    KS_CHECK(hipEventRecord(s.ev[0], st));
    KS_CHECK(hipMemsetAsync(s.ctr.p, 0, CTR_SHARDS * NCTR * sizeof(unsigned long long), st));
    KS_CHECK(hipMemsetAsync(s.ctl.p, 0, sizeof(Ctl), st));
    std::memset(s.h_ctl, 0, sizeof(Ctl));

    // ------------------------------------------------- build / reset ---
    // The CSR persists between solves; it is rebuilt from the arc table only when
    // an in-place delta did not fit (or after a load). A cold solve resets the
    // residual state; a warm one keeps it (carried across a rebuild by slot).
    if (!s.csr_valid) {
        const int64_t ncap_prev = s.ncap;
        const long long mult_prev = s.mult;
        const bool carry = use_warm && s.nn > 0;
        const int hi0 = s.hi();
        if (carry) {
            KS_CHECK(s.saved_flows.ensure(std::max(hi0, 1)));
            KS_CHECK(s.p_slot.ensure(std::max<int64_t>(ncap_prev, 1)));
            if (hi0)
                hipLaunchKernelGGL(k_save_flows, dim3(grid_for(hi0)), dim3(BLK), 0, st, hi0,
                                   (const unsigned char*)s.a_alive.p, (const int*)s.fwd.p, (const Pos*)s.pos.p,
                                   s.saved_flows.p);
            hipLaunchKernelGGL(k_save_prices, dim3(grid_for(ncap_prev)), dim3(BLK), 0, st, (int)ncap_prev,
                               (const int*)s.perm.p, (const long long*)s.nd.p, s.p_slot.p);
            if (fb && !s.fb_cells.empty()) {
                std::vector<long long> rng;
                const size_t kc = s.cell_off.size() >= 2 ? s.cell_off.size() - 1 : 1;
                for (int c : s.fb_cells) {
                    rng.push_back(kc > 1 ? s.cell_off[c] : 0);
                    rng.push_back(kc > 1 ? s.cell_off[c + 1] : ncap_prev);
                }
                KS_CHECK(s.fb_rng.ensure(rng.size()));
                KS_CHECK(hipMemcpyAsync(s.fb_rng.p, rng.data(), rng.size() * sizeof(long long), hipMemcpyHostToDevice,
                                        st));
                const int n = (int)std::max<int64_t>(hi0, ncap_prev);
                KS_CHECK(s.fb_cnt.ensure(1));
                KS_CHECK(hipMemsetAsync(s.fb_cnt.p, 0, sizeof(unsigned long long), st));
                hipLaunchKernelGGL(k_fb_reset, dim3(grid_for(std::max(n, 1))), dim3(BLK), 0, st, hi0, (int)ncap_prev,
                                   (int)(rng.size() / 2), (const long long*)s.fb_rng.p, (const int*)s.a_src.p,
                                   (const unsigned char*)s.a_alive.p, s.saved_flows.p, s.p_slot.p, s.fb_cnt.p);
                unsigned long long nres = 0;
                KS_CHECK(hipMemcpyAsync(&nres, s.fb_cnt.p, sizeof(nres), hipMemcpyDeviceToHost, st));
                KS_CHECK(hipStreamSynchronize(st));   // (rng is a host vector)
                res.fb_resets = nres;
            }
        }
        int rc = build(s, err);
        if (rc) return rc;
        rc = cold_reset(s, err);
        if (rc) return rc;
        if (carry) {
            if (hi0)
                hipLaunchKernelGGL(k_restore_flows, dim3(grid_for(hi0)), dim3(BLK), 0, st, hi0,
                                   (const unsigned char*)s.a_alive.p, (const long long*)s.saved_flows.p,
                                   (const long long*)s.a_low.p, (const long long*)s.a_cap.p, (const int*)s.fwd.p,
                                   (const int*)s.a_src.p, (const int*)s.a_dst.p, (const int*)s.perm.p, s.pos.p,
                                   s.excess.p);
            hipLaunchKernelGGL(k_restore_prices, dim3(grid_for(s.ncap)), dim3(BLK), 0, st, (int)s.ncap,
                               (int)ncap_prev, mult_prev, s.mult, (const long long*)s.p_slot.p, (const int*)s.perm.p,
                               s.nd.p, (s.nd.p + 2));
        }
    } else if (!use_warm) {
        int rc = cold_reset(s, err);
        if (rc) return rc;
    }
    const int hi = s.hi();
    const int nn = s.nn;
    const int64_t m2 = s.m2cap;
    res.n_nodes = s.nslots;
    res.n_arcs = s.h_sctl->live;
    if (nn == 0) {
        res.total_cost = 0;
        res.flow_value = 0;   // no nodes: nothing flows
        s.solved = true;
        s.has_prev = true;
        return KS_OK;
    }
    // max |cost| → the first phase's ε
    if (hi)
        hipLaunchKernelGGL(k_max_cost, dim3(grid_for(hi, 512)), dim3(BLK), 0, st, hi,
                           (const unsigned char*)s.a_alive.p, (const long long*)s.a_cost.p, &s.ctl.p->gu_L);
    // the engine's hot kernels read 16-B copies of the positions when every value
    // fits; the range flag comes back with the control block below
    const bool want_cp = !s.cell_layout && s.opts.compact_pos >= 0 && m2 > 0;
    if (want_cp) {
        KS_CHECK(s.cpos.ensure(m2));
        KS_CHECK(s.crev.ensure(m2));
        hipLaunchKernelGGL(k_pack_pos, dim3(grid_for(m2, 4096)), dim3(BLK), 0, st, (long long)m2,
                           (const Pos*)s.pos.p, s.cpos.p, s.crev.p, &s.ctl.p->cp_bad);
    }
    KS_CHECK(hipMemcpyAsync(s.h_ctl, s.ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    const long long maxc = s.h_ctl->gu_L;
    const bool cpv = want_cp && !s.h_ctl->cp_bad;
    bool cp_dirty = false;   // the compact residuals hold changes Pos does not have yet
    res.compact = cpv ? 1 : 0;
    KS_CHECK(hipMemsetAsync(&s.ctl.p->gu_L, 0, sizeof(long long), st));
    const long long mult = s.mult;
    if (maxc > 0 && (double)maxc * (double)mult * 8.0 * (double)mult > 4.0e18) {
        err = "cost range too large for int64 scaled prices";
        return KS_E_RANGE;
    }
    KS_CHECK(hipEventRecord(s.ev[1], st));

    // ------------------------------------------------------------ phases ---
    // Tuning comes from ks_opts only (0 = default; include/ksmcmf.h): nothing in
    // the environment changes the algorithm.
    const ks_opts& o = s.opts;
    DG g = s.dg();
    g.cp = cpv ? s.cpos.p : nullptr;
    g.crev = cpv ? s.crev.p : nullptr;
    g.expand = o.two_hop < 0 ? 0 : 1;      // two hops per round through tasks and PUs
    g.bound = o.bf_bound < 0 ? 0 : 1;      // tail updates bounded at the excess nodes' distances
    g.fs_wide = std::max(2048, nn / 4);   // (measured: config 4's searches ≤ nn/6 wide, config 3's hub-bound ones ~nn/4 to 3nn/4)
    g.aug_k = o.tail_nodes > 0 ? std::min(AUG_KMAX, (int)o.tail_nodes) : 64;
    const int fgrid = s.window_grid();     // dense passes over every window (saturate)
    const int dgrid = s.dense_grid();      // dense Bellman-Ford round
    const int sgrid = s.sparse_grid();     // sparse Bellman-Ford rounds
    const int wgrid = s.sweep_grid();      // sweeps
    const int ngrid = grid_for(nn, 2048);
    const int fsgrid = s.nhitems * HSPLIT + FS_LIST_BLOCKS;   // forward tail rounds
    // forward tail updates once ≤ fwd_k nodes hold excess (ks_opts.fwd_nodes; the
    // search key packs an arc position into FS_PB bits)
    const bool use_fwd = o.fwd_nodes >= 0 && s.m2cap < FS_NONE;
    // (default by size: config 2's 12k-node searches widen sooner; interleaved A/B,
    // config 2 28.0 / 26.4 → 25.5 / 25.0 ms at 32, config 4 slower at 32 than at 64)
    const int fwd_k = o.fwd_nodes > 0 ? (int)o.fwd_nodes : (nn < 32768 ? 32 : 64);
    int kf = 16;                        // forward rounds enqueued per cycle (adaptive)
    uint64_t fwd_updates = 0, fs_launches = 0;
    // α by size: with the cycle-cancelling finish a small engine graph is best with
    // one coarse phase and the finish (12 config-2 graphs, median / max ms: α 8 14.6 /
    // 17.9, 16 14.9 / 16.5, 32 11.6 / 15.4, 48 12.6 / 15.9, 1024 — a single phase at
    // the final ε — 13.4 / 24.4); config 3 and the config-4 rounds are slower at 16
    // and 32, and the cell solver's ladder stays at 8 (config 5 36 ms at 32) — DESIGN §3
    // (the small-graph α and the D below were tuned for the finish: they follow use_prc,
    // so a graph whose positions do not fit the packed keys keeps the plain schedule)
    const bool use_pr = o.price_refine != 0;
    const bool use_prc = use_pr && o.price_refine == 1 && !s.cell_layout && s.m2cap < PK_NONE;
    const int alpha = o.alpha >= 2 ? o.alpha : (!s.cell_layout && nn < 32768 && use_prc) ? 32 : 8;
    int gi_base = o.gu_interval > 0 ? o.gu_interval : 24;
    gi_base = std::max(2, std::min(MAXB, gi_base)) & ~1;     // even: sweeps end on p0
    const int pr_cap = o.pr_rounds > 0 ? o.pr_rounds : 160;  // price-refinement rounds before giving up
    long long pr_div = 32;   // certify at ε = 1 once ε·pr_div < one (scaled) cost unit
    const bool cycle_log = o.log_cycles != 0;
    const int nhit = s.nhitems;
    const bool use_aug = o.walk_slack >= 0;               // tail augmentation (walks)
    const int aug_slack = o.walk_slack > 0 ? o.walk_slack : 4;   // walks take arcs of rc <= slack·ε
    const int walk_passes = o.walk_passes > 0 ? std::min(8, (int)o.walk_passes) : 1;
    // Bellman-Ford rounds enqueued per cycle: the last update's count + kb_margin,
    // at least kb_min (a launch that finds the update converged still costs ≈ 5 µs
    // with the gap before the next kernel; an update that needs more than was
    // enqueued costs a whole extra cycle)
    const int kb_margin = o.bf_margin > 0 ? o.bf_margin : 6, kb_min = 8;
    bool pr_failed = false;   // the last phase's refinement did not certify the flow
    // the cycle-cancelling finish replaces the final cost-scaling phase (ks_opts.price_refine
    // 1, the default; 2: the final phase and plain refinement, as before round 5)
    // refinement rounds before the final phase takes over (TESTS ONLY, fault_inject bit 5: one batch)
    const int prc_cap = (o.fault_inject & 32) ? 32 : 4096;
    bool prc_tried = false;
    const int gi_tail = o.tail_sweeps > 0 ? std::max(2, std::min(MAXB, (int)o.tail_sweeps)) & ~1 : 4;
    // A phase that another phase follows may end with a few excess nodes left:
    // refine's start (saturate every negative reduced cost) accepts any
    // pseudoflow, so the next, finer phase absorbs them with its own excess.
    // Only the last phase (the one price refinement may certify, or ε = 1) must
    // end with a feasible flow. A coarse phase ends once at most phase_exit
    // nodes AND at most 1/phase_frac of its peak hold excess (the relative bound
    // keeps phases that start small — incremental rounds — doing their share).
    const int phase_exit = o.phase_exit < 0 ? 0 : (o.phase_exit > 0 ? o.phase_exit : 256);
    const int phase_frac = o.phase_frac > 0 ? o.phase_frac : 128;
    // ε schedule: the phase that price refinement certifies runs at 1/D of a cost
    // unit (ks_opts.final_div), the others at α-multiples of it, the first in
    // [max|cost|/α², max|cost|/α) scaled. D = 48 on large graphs. Measured on config 3
    // (40 solves each): ending at 1/32 of a unit (the plain max|cost|/α^k sequence)
    // left the flow short of optimal in 15 of 40 solves — a sixth phase, ≈ 28 ms —
    // at 1/48 in none; 1/64 and 1/96 cost more per phase. D = 20 on small graphs and
    // cells (under 32,768 nodes; every cell is): their flow is usually optimal a
    // phase earlier (config 2 26–27 → 20–21 ms, config 5 53–54 → 41–43 ms).
    // Round 5: with the cycle-cancelling finish the final phase no longer runs, and
    // D only places the ladder; large graphs take D = 24 — one coarse phase fewer
    // (config 3: 35.4–36.9 vs 36.6–38.6 ms in interleaved pairs).
    long long eps = std::max<long long>(1, maxc * mult);
    {
        const long long D = o.final_div < 0 ? 0
                            : o.final_div > 0 ? o.final_div
                            : (s.cell_layout || nn < 32768) ? 20 : (use_prc ? 24 : 48);
        if (D > 0 && use_pr && maxc > 0) {
            long long e = std::max<long long>(1, (mult - 1) / D);
            // the cell solver's ladder is powers of two (α = 8): its arc lengths
            // floor(rc/ε) are then shifts (the final phase lands in (1/2D, 1/D] of a unit)
            if (s.cell_layout && (alpha & (alpha - 1)) == 0)
                while (e & (e - 1)) e &= e - 1;
            const long long lo = std::max<long long>(1, eps / ((long long)alpha * alpha));
            while (e < lo && e <= (1LL << 58) / alpha) e *= alpha;
            eps = e * alpha;   // the loop divides before each phase
            pr_div = D;
        }
    }
    uint64_t sweeps = 0, gus = 0, sweep_launches = 0, bf_launches = 0, sweep_kernels = 0, early_exits = 0;
    double ms_bf_k = 0, ms_sw_k = 0, ms_fs_k = 0;   // event-timed spans: BF rounds / sweeps / forward rounds
    int phases = 0;
    int kb = 24;                        // Bellman-Ford rounds enqueued per cycle (adaptive)
    int sseq = 0, bseq = 0;             // frontier buffer sequences
    double ms_sat = 0, ms_cycles = 0, ms_pr = 0;
    int status = KS_OK;

    auto read_ctl = [&]() -> hipError_t {
        hipError_t e = hipMemcpyAsync(s.h_ctl, s.ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) return e;
        return hipStreamSynchronize(st);
    };
    // ε (and, by flags, the control words a phase or the finish starts from) set by a
    // one-thread kernel: a host-to-device copy is a copy kernel behind a staging gap,
    // and each memset another launch
    auto set_eps = [&](long long e, int flags = 0) -> hipError_t {
        hipLaunchKernelGGL(k_set_eps, dim3(1), dim3(1), 0, st, g, e, flags);
        return hipGetLastError();
    };
    // mode 0: global update; 1: price refinement; 2: refinement with parents (cycle cancelling)
    auto bf_rounds = [&](int mode, int k, bool first_dense) {
        for (int r = 0; r < k; ++r) {
            const int dense = (first_dense && r == 0) ? 1 : 0;
            const int grid = dense ? dgrid : sgrid;
            if (mode == 2) {
                if (cpv) k_bf_round<2, true><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
                else k_bf_round<2, false><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
            } else if (mode) {
                if (cpv) k_bf_round<1, true><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
                else k_bf_round<1, false><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
            } else {
                if (cpv) k_bf_round<0, true><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
                else k_bf_round<0, false><<<dim3(grid), dim3(BLK), 0, st>>>(g, bseq, dense);
            }
            ++bseq;
            ++bf_launches;
        }
    };
    // Price refinement at eps_try: 1 = success (prices updated), 0 = failed, <0 error.
    auto price_refine = [&](long long eps_try, int* rounds_used, int cap, int from_p = 0) -> int {
        KS_CHECK(hipEventRecord(s.ev[6], st));
        KS_CHECK(set_eps(eps_try));
        hipLaunchKernelGGL(k_pr_init, dim3(ngrid), dim3(BLK), 0, st, g, bseq, from_p);
        int used = 0, ok = 0;
        for (int batch = 0; used < cap; ++batch) {
            const int k = std::min(64, cap - used);
            KS_CHECK(hipEventRecord(s.kev[0], st));
            bf_rounds(1, k, batch == 0);
            KS_CHECK(hipEventRecord(s.kev[1], st));
            used += k;
            KS_CHECK(read_ctl());
            ms_bf_k += ev_ms(s.kev[0], s.kev[1]);
            if (s.h_ctl->bf_done) {
                ok = 1;
                break;
            }
        }
        if (ok) hipLaunchKernelGGL(k_pr_apply, dim3(ngrid), dim3(BLK), 0, st, g, 0);
        KS_CHECK(hipEventRecord(s.ev[7], st));
        KS_CHECK(hipEventSynchronize(s.ev[7]));
        ms_pr += ev_ms(s.ev[6], s.ev[7]);
        *rounds_used = used;
        return ok;
    };

    // The cycle-cancelling finish: refinement rounds that record parents
    // (PR = 2), and after every batch that has not converged a search of the parent
    // graph that cancels the negative cycles it holds. 1 = certified (prices set),
    // 0 = gave up within cap rounds (the final cost-scaling phase follows), < 0 error.
    int prc_cycles = 0, prc_searches = 0;
    long long prc_rejected = 0;   // nodes / leader walks the searches' union-of-cycles test rejected
    long long solve_units = -1;   // excess units at the solve's first update (cold: the supply)
    unsigned long long gu_prev = 0;   // cycle log: Bellman-Ford relaxations counted so far
    auto prc_refine = [&](int* rounds_used, int cap) -> int {
        KS_CHECK(hipEventRecord(s.ev[6], st));
        KS_CHECK(s.cyc.ensure((size_t)9 * nn));
        KS_CHECK(s.cyc64.ensure((size_t)2 * nn));
        int2* JMa = reinterpret_cast<int2*>(s.cyc.p);   // jump words, double-buffered (8-B aligned)
        int2* JMb = JMa + nn;
        int* J0 = reinterpret_cast<int*>(JMb + nn);
        int* onc = J0 + nn;
        int* R = onc + nn;
        int* gbad = R + nn;
        int* indeg = gbad + nn;   // members of its group pointing at a node
        long long* gsum = s.cyc64.p;
        long long* gcap = gsum + nn;
        KS_CHECK(set_eps(1, SET_CYC));   // and cyc_done, cyc_rej zeroed
        hipLaunchKernelGGL(k_pr_init, dim3(ngrid), dim3(BLK), 0, st, g, bseq, 2);
        const int* done = &s.ctl.p->bf_done;
        // the parent graph: pointer doubling over CYC_WALK steps, cycles grouped by
        // their least id, every good negative one cancelled in parallel (each kernel
        // returns at once when the refinement has converged)
        int nsearch = 0;
        // graphs whose parent graph fits one workgroup's LDS search in one launch
        // (k_cyc_lds) instead of 12–15
        const bool lds_search = nn <= CYC_LDS_MAX && cyc_lds_bytes(nn) <= s.lds_limit;
        if (lds_search) {
            KS_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cyc_lds<true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)cyc_lds_bytes(nn)));
            KS_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cyc_lds<false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)cyc_lds_bytes(nn)));
        }
        auto search = [&]() {
            // three of four searches double only CYC_SHORT times (cycles of up to 128
            // arcs: the ones the finish meets); every fourth covers 2^CYC_LOG
            // (TESTS ONLY, fault_inject bit 7: every search 5 steps, a window shorter than
            // the parent chains — their nodes get marked and run into cycles' groups)
            const int lg = (o.fault_inject & 128) ? 5 : (nsearch++ % 4 == 3) ? CYC_LOG : CYC_SHORT;
            const int apply_check = (o.fault_inject & 256) ? 0 : 1;
            if (lds_search) {   // small graphs: the whole search in one workgroup, in LDS
                const size_t sh = cyc_lds_bytes(nn);
                if (cpv) k_cyc_lds<true><<<dim3(1), dim3(CYC_LDS_T), sh, st>>>(g, lg, apply_check, bseq, gsum, gcap, gbad);
                else k_cyc_lds<false><<<dim3(1), dim3(CYC_LDS_T), sh, st>>>(g, lg, apply_check, bseq, gsum, gcap, gbad);
                return;
            }
            KS_HOT(cpv, k_cyc_par, ngrid, BLK, st, g, J0, JMa, onc, R, gsum, gcap, gbad, indeg);
            const int2* JMK = JMa;
            for (int left = lg, k = 0; left > 0; ++k) {   // ×4 per launch, ×2 for an odd remainder
                const int2* in = (k & 1) ? JMb : JMa;
                int2* out = (k & 1) ? JMa : JMb;
                const int f2 = left >= 2 ? 2 : 1;
                left -= f2;
                const int mark = left == 0 ? 1 : 0;
                if (f2 == 2)
                    hipLaunchKernelGGL(k_cyc_jump<4>, dim3(ngrid), dim3(BLK), 0, st, nn, done, in, out, mark,
                                       (const int*)J0, onc);
                else
                    hipLaunchKernelGGL(k_cyc_jump<2>, dim3(ngrid), dim3(BLK), 0, st, nn, done, in, out, mark,
                                       (const int*)J0, onc);
                JMK = out;
            }
            KS_HOT(cpv, k_cyc_group, ngrid, BLK, st, g, (const int*)J0, JMK, (const int*)onc, (const int*)R, gsum, gcap,
                   gbad, indeg);
            hipLaunchKernelGGL(k_cyc_check, dim3(ngrid), dim3(BLK), 0, st, nn, done, (const int*)J0, JMK,
                               (const int*)onc, (const int*)indeg, gbad, apply_check, &s.ctl.p->cyc_rej);
            KS_HOT(cpv, k_cyc_push, ngrid, BLK, st, g, (const int*)J0, JMK, (const int*)onc, (const int*)R,
                   (const long long*)gsum, (const long long*)gcap, (const int*)gbad, bseq);
        };
        // Batches of CYC_PERIODS × (CYC_EVERY[_LDS] rounds + a search), pipelined two deep:
        // batch b+1 is enqueued before the host waits for batch b's control snapshot
        // (k_prc_snap, into pinned memory), so the GPU does not idle through the
        // host's round trip (~27 µs per batch with a copy-engine read, r06 traces).
        // Once the refinement has converged, every kernel of the batch in flight
        // exits at once. A batch's Bellman-Ford time is its event span less its
        // searches (device clock: k_cyc_par / k_cyc_lds to the next round's start).
        // One event per batch, after its snapshot: batch b's span runs from batch
        // b−1's event (the first: fin_ev[3]) — two events back to back cost a gap each.
        int used = 0, ok = 0, nb = 0;   // nb: batches enqueued
        unsigned long long srch_seen = 0;
        KS_CHECK(hipEventRecord(s.fin_ev[3], st));
        auto end_ev = [&](int b) { return s.fin_ev[b % 3]; };
        auto start_ev = [&](int b) { return b == 0 ? s.fin_ev[3] : s.fin_ev[(b - 1) % 3]; };
        auto enqueue_batch = [&](int slot) -> hipError_t {
            const int b = nb++;
            for (int per = 0; per < (b == 0 ? 1 : CYC_PERIODS) && used < cap; ++per) {
                const int every = lds_search ? CYC_EVERY_LDS : CYC_EVERY;
                const int k = std::min(b == 0 ? 2 * every : every, cap - used);
                bf_rounds(2, k, b == 0);
                used += k;
                search();
                ++prc_searches;
            }
            hipLaunchKernelGGL(k_prc_snap, dim3(1), dim3(128), 0, st, g, s.d_cyc[slot]);
            return hipEventRecord(end_ev(b), st);
        };
        auto batch_time = [&](int b) {   // → ms_bf_k
            const Ctl* hc = s.h_cyc[b & 1];
            const double span = ev_ms(start_ev(b), end_ev(b));
            const double srch = hc->srch_ticks > srch_seen ? (double)(hc->srch_ticks - srch_seen) / 1e5 : 0.0;
            srch_seen = std::max(srch_seen, hc->srch_ticks);
            ms_bf_k += std::max(0.0, span - srch);
            return span;
        };
        KS_CHECK(enqueue_batch(0));
        int done_b = 0;   // batches whose snapshot the host has read
        for (int batch = 0;; ++batch) {
            const int slot = batch & 1;
            const bool more = used < cap;
            if (more) KS_CHECK(enqueue_batch(slot ^ 1));
            KS_CHECK(hipEventSynchronize(end_ev(batch)));
            ++done_b;
            const Ctl* hc = s.h_cyc[slot];
            const double span = batch_time(batch);
            cp_dirty = cpv;
            if (cycle_log) {   // one line per batch: rounds so far, cycles so far, relaxations, time
                std::vector<unsigned long long> hctr((size_t)CTR_SHARDS * NCTR);
                KS_CHECK(hipMemcpy(hctr.data(), s.ctr.p, hctr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                unsigned long long gsc = 0;
                for (int i = 0; i < CTR_SHARDS; ++i) gsc += hctr[(size_t)i * NCTR + C_GUSCAN];
                std::fprintf(stderr, "finish batch %d rounds %d worked %d cycles %d rejected %d relax %llu ms %.3f (searches %.3f)\n",
                             batch, used, hc->bf_count, hc->cyc_done, hc->cyc_rej, gsc - gu_prev, span,
                             (double)hc->srch_ticks / 1e5);
                gu_prev = gsc;
            }
            if (hc->bf_done) {
                ok = 1;
                break;
            }
            if (!more) break;   // the round cap: this was the last batch
        }
        if (nb > done_b) {   // the batch enqueued behind the converged one (its kernels exited at once)
            KS_CHECK(hipEventSynchronize(end_ev(nb - 1)));
            batch_time(nb - 1);
        }
        if (ok) hipLaunchKernelGGL(k_pr_apply, dim3(ngrid), dim3(BLK), 0, st, g, 1);
        KS_CHECK(hipEventRecord(s.ev[7], st));
        KS_CHECK(hipEventSynchronize(s.ev[7]));
        ms_pr += ev_ms(s.ev[6], s.ev[7]);
        KS_CHECK(read_ctl());
        prc_cycles += s.h_ctl->cyc_done;
        prc_rejected += s.h_ctl->cyc_rej;
        *rounds_used = used;
        if (cycle_log)
            std::fprintf(stderr, "cycle-cancelling refinement: %s after %d rounds, %d searches, %d cycles cancelled\n",
                         ok ? "certified" : "gave up", used, prc_searches, s.h_ctl->cyc_done);
        return ok;
    };

    // One ε-phase from the pseudoflow in place: saturate every residual arc whose
    // reduced cost is below −sat_thr (thr 0: Goldberg's refine start; thr ε: only
    // the arcs that violate ε-optimality), then update/sweep cycles until no node
    // holds excess — a coarse phase (may_end_early) may stop with a few excess
    // nodes left for the next, finer one. walk_sl: the tail walks' slack (1 when the
    // phase must end ε-optimal at ε = 1). Returns KS_OK, KS_E_INFEASIBLE (status),
    // or a device / convergence error.
    // prc_early: when non-null, the phase may turn itself into the one the cycle-
    // cancelling finish follows (*prc_early = 1, the phase then drains): at its first
    // update, if at most 1/KS_PRC_UNITS_DIV of the solve's first-update units hold
    // excess — the flow is already close to optimal (config 4's churn
    // rounds, 0.07–0.11 of the supply, vs ≥ 1.9 for cold configs 2 and 3)
    auto run_phase = [&](long long eps_ph, long long sat_thr, bool may_end_early, int walk_sl,
                         int* prc_early = nullptr) -> int {
        KS_CHECK(hipEventRecord(s.ev[2], st));
        KS_CHECK(set_eps(eps_ph, use_fwd ? SET_FWD : 0));   // a phase never continues another phase's forward search
        KS_HOT(cpv, k_saturate, fgrid, BLK, st, g, sat_thr);
        cp_dirty = cpv;
        KS_CHECK(hipEventRecord(s.ev[3], st));
        uint64_t phase_sweeps = 0;
        int gi = gi_base;     // sweeps in the next cycle (fewer in a phase's tail, where walks augment)
        int phase_peak = 0;   // most excess nodes seen by an update of this phase
        int list = 0;         // the next update lists its excess nodes for the bound (the last apply found ≤ BX_CAP)
        int fwd = 0;          // the next cycle is a forward tail update (≤ fwd_k excess nodes left)
        int fwd_block = 0;    // a forward cycle failed or moved nothing: the next one is a backward update
        int fwd_budget = 64;  // rounds a forward search may take: twice the last global update's
        const int wsl = walk_sl;
        bool early = may_end_early;
        bool first_upd = true;
        int rc = KS_OK;
        // Forward cycle: nupd × [init (or continue the pending search)][kf rounds][apply]
        // [trace][end], then the cycle end; no sweeps (the trace routes the units). An
        // update whose search has not converged when the next one starts is continued
        // by it. fev brackets each update's search rounds (the forward kind's time).
        auto enqueue_fwd = [&](int par, int nupd) -> hipError_t {
            hipError_t e = hipSuccess;
            for (int u = 0; u < nupd; ++u) {
                hipLaunchKernelGGL(k_fs_init, dim3(ngrid), dim3(BLK), 0, st, g, bseq);
                if ((e = hipEventRecord(s.fev[par][2 * u], st)) != hipSuccess) return e;
                for (int r = 0; r < kf; ++r) {
                    KS_HOT(cpv, k_fs_round, fsgrid, BLK, st, g, bseq);
                    ++bseq;
                    ++fs_launches;
                }
                if ((e = hipEventRecord(s.fev[par][2 * u + 1], st)) != hipSuccess) return e;
                hipLaunchKernelGGL(k_fs_apply, dim3(ngrid), dim3(BLK), 0, st, g);
                KS_HOT(cpv, k_fs_trace, FDEF_CAP, WAVE, st, g);
                hipLaunchKernelGGL(k_fs_end, dim3(1), dim3(WAVE), 0, st, g);
            }
            hipLaunchKernelGGL(k_cycle_end, dim3(1), dim3(128), 0, st, g, s.d_cyc[par], 1);
            return hipEventRecord(s.cdone[par], st);
        };
        int nupd = 1;         // forward updates per cycle (FWD_UPD once a search finished within its rounds)
        int completed0 = 0;   // fs_completed at the phase's start of forward cycles
        // One cycle: [GU init (or continue the pending update)][kb BF rounds][max]
        // [apply][tail walks][gi sweeps][end: control block → pinned host memory].
        // cev[0..1] bracket the Bellman-Ford rounds (the sweeps: device clock).
        auto enqueue = [&](int par) -> hipError_t {   // one cycle into slot par
            hipLaunchKernelGGL(k_gu_init, dim3(ngrid), dim3(BLK), 0, st, g, bseq, list);
            hipError_t e = hipEventRecord(s.cev[par][0], st);
            if (e != hipSuccess) return e;
            for (int r = 0; r < kb; ++r) {   // sparse from the first round: k_gu_init flags the deficits
                if (cpv) k_bf_round<0, true><<<dim3(sgrid), dim3(BLK), 0, st>>>(g, bseq, 0);
                else k_bf_round<0, false><<<dim3(sgrid), dim3(BLK), 0, st>>>(g, bseq, 0);
                ++bseq;
                ++bf_launches;
            }
            if ((e = hipEventRecord(s.cev[par][1], st)) != hipSuccess) return e;
            hipLaunchKernelGGL(k_gu_max, dim3(ngrid), dim3(BLK), 0, st, g);
            hipLaunchKernelGGL(k_gu_apply, dim3(ngrid), dim3(BLK), 0, st, g, sseq);
            if (use_aug) {   // tail: walkers, hub distribution, walkers from what it fed
                KS_HOT(cpv, k_augment, g.aug_k, WAVE, st, g, sseq, 0, wsl);
                if (nhit) KS_HOT(cpv, k_aug_hub, nhit, BLK, st, g, sseq, wsl);
                KS_HOT(cpv, k_augment, AUG_K2, WAVE, st, g, sseq, 1, wsl);
                // further passes retry the units left short at the listed nodes
                for (int wp = 1; wp < walk_passes; ++wp)
                    KS_HOT(cpv, k_augment, g.aug_k, WAVE, st, g, sseq, 0, wsl);
            }
            // (the sweeps are timed by the device clock — the first sweep's start to
            // k_cycle_end's — not by HIP events: an event between two kernels costs a
            // ~5.7 µs gap of its own, two per cycle; profiles/r06_*)
            for (int k = 0; k < gi; ++k) KS_HOT(cpv, k_sweep, wgrid, BLK, st, g, k, sseq + k);
            hipLaunchKernelGGL(k_cycle_end, dim3(1), dim3(128), 0, st, g, s.d_cyc[par], 0);
            sseq += gi;
            return hipEventRecord(s.cdone[par], st);
        };
        // Cycles run one at a time (enqueueing the next one before reading this
        // one's control block was measured slower: the speculative launches cost
        // more GPU time than the host's decision gap).
        int cur = 0;
        int bf_pend = -1;   // a cycle whose Bellman-Ford event span is not read yet
        auto flush_bf = [&]() {
            if (bf_pend >= 0) ms_bf_k += ev_ms(s.cev[bf_pend][0], s.cev[bf_pend][1]);
            bf_pend = -1;
        };
        for (;;) {
            if (fwd) {
                KS_CHECK(enqueue_fwd(cur, nupd));
                KS_CHECK(hipEventSynchronize(s.cdone[cur]));
                const Ctl* hc = s.h_cyc[cur];
                double t_fs = 0;
                for (int u = 0; u < nupd; ++u) t_fs += ev_ms(s.fev[cur][2 * u], s.fev[cur][2 * u + 1]);
                ms_fs_k += t_fs;
                cur ^= 1;
                const bool completed = hc->fs_done || hc->fs_fail;
                if (cycle_log)
                    std::fprintf(stderr, "fwd cycle phase %d eps %lld updates %d rounds %d fs_ms %.3f units %lld n_exc %d done %d fail %d D %lld deficits %d moved %d width %d\n",
                                 phases, eps_ph, nupd, hc->fs_rounds, t_fs, hc->u_exc_rep, hc->n_exc_rep,
                                 hc->fs_done, hc->fs_fail, hc->fs_D < FS_DMAX ? hc->fs_D : -1LL, hc->n_fdef,
                                 hc->fs_moved_cyc, hc->fs_maxcnt);
                if (completed && hc->n_exc_rep == 0) break;   // no excess left: the phase is done
                const int done_now = hc->fs_completed - completed0;
                completed0 = hc->fs_completed;
                gus += done_now;
                fwd_updates += done_now;
                bool wide = hc->fs_fail == 2;
                if (!completed && hc->fs_rounds >= fwd_budget) {
                    // longer than two global updates: drop it like a wide one
                    KS_CHECK(hipMemsetAsync(&s.ctl.p->fs_pending, 0, sizeof(int), st));
                    KS_CHECK(hipMemsetAsync(s.ctl.p->fs_cnt, 0, sizeof(s.ctl.p->fs_cnt), st));
                    wide = true;
                }
                if (hc->fs_fail || wide) {
                    // list overflow, no deficit in range, or a search too wide or too long
                    // (a hub's arcs in reach): ONE global update, then forward again
                    fwd = 0;
                    fwd_block = 1;
                    nupd = 1;
                    continue;
                }
                if (!completed) {            // the search continues next cycle
                    kf = std::min(256, 2 * kf);
                    nupd = 1;
                    continue;
                }
                kf = std::max(8, std::min(256, hc->fs_rounds + 4));
                nupd = FWD_UPD;
                if (hc->fs_moved_cyc == 0) {
                    fwd = 0;
                    fwd_block = 1;
                }
                if (wall_s() > kSolveWallLimitS) {
                    (void)hipStreamSynchronize(st);
                    err = "forward tail did not converge (" + std::to_string(wall_s()) + " s)";
                    return KS_E_DEVICE;
                }
                continue;
            }
            if (bf_pend == cur) flush_bf();   // (the slot's events are about to be recorded again)
            KS_CHECK(enqueue(cur));
            flush_bf();   // the previous cycle's event time, read while this one runs
            KS_CHECK(hipEventSynchronize(s.cdone[cur]));
            const Ctl* hc = s.h_cyc[cur];
            sweep_kernels += gi;
            double t_bf = 0;
            if (cycle_log) {
                t_bf = ev_ms(s.cev[cur][0], s.cev[cur][1]);
                ms_bf_k += t_bf;   // BF rounds only
            } else {
                bf_pend = cur;     // read after the next cycle is enqueued (off the host's critical path)
            }
            const double t_sw = hc->t_end > hc->t_sw0 ? (double)(hc->t_end - hc->t_sw0) / 1e5 : 0.0;   // 100 MHz ticks
            ms_sw_k += t_sw;   // sweeps only
            if (hc->infeasible) {
                rc = KS_E_INFEASIBLE;
                std::memcpy(s.h_ctl, hc, sizeof(Ctl));
                break;
            }
            if (!hc->bf_done) {
                // update still running: its sweeps were skipped and the next cycle continues it
                kb = std::min(256, kb * 2);
                cur ^= 1;
                continue;
            }
            if (cycle_log) {
                // (diagnostics: the update's relaxations, from the sharded counters)
                std::vector<unsigned long long> hctr((size_t)CTR_SHARDS * NCTR);
                KS_CHECK(hipMemcpy(hctr.data(), s.ctr.p, hctr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                unsigned long long gsc = 0;
                for (int i = 0; i < CTR_SHARDS; ++i) gsc += hctr[(size_t)i * NCTR + C_GUSCAN];
                std::fprintf(stderr, "cycle phase %d eps %lld bf %d relax %llu bf_ms %.3f sw_ms %.3f active %d units %lld n_exc %d walks %d/%d",
                             phases, eps_ph, hc->bf_count - hc->bf_r0, gsc - gu_prev, t_bf, t_sw, hc->sweep_act[gi - 1], hc->u_exc, hc->n_exc,
                             hc->aug_reached, hc->aug_short);
                gu_prev = gsc;
                for (int k = 0; k < std::min(4, hc->n_exc); ++k) {
                    const int x = hc->dbg_x[k];
                    int c = 0;
                    while (c < NGC && x >= s.obeg[c + 1]) ++c;
                    std::fprintf(stderr, " [x%d c%d e%d]", x, x >= s.hub_base ? 9 : c, hc->dbg_e[k]);
                }
                std::fprintf(stderr, "\n");
            }
            if (first_upd) {
                first_upd = false;
                if (solve_units < 0) solve_units = hc->u_exc;
                if (prc_early && early && hc->u_exc * kPrcUnitsDiv <= solve_units) {
                    early = false;
                    *prc_early = 1;
                }
            }
            kb = std::max(kb_min, std::min(256, hc->bf_count - hc->bf_r0 + kb_margin));
            fwd_budget = std::max(16, 2 * (hc->bf_count - hc->bf_r0));
            ++gus;
            sweeps += gi;
            sweep_launches += gi;
            phase_sweeps += gi;
            int last = 0;
            for (int k = 0; k < gi; ++k)
                if (hc->sweep_act[k]) last = k + 1;
            if (!hc->sweep_act[gi - 1]) {
                sweeps -= gi - last;
                break;   // no excess left: refine done
            }
            phase_peak = std::max(phase_peak, hc->n_exc);
            if (early && hc->n_exc <= phase_exit && (long long)hc->n_exc * phase_frac <= phase_peak) {
                ++early_exits;
                break;   // a coarse phase: the next one absorbs the few units left
            }

            gi = (use_aug && hc->n_exc <= g.aug_k) ? gi_tail : gi_base;
            list = g.bound && hc->n_exc > 0 && hc->n_exc <= BX_CAP;
            // forward tail updates only in coarse phases: in the last phase config 3's
            // searches reach the cluster aggregator and widen
            fwd = use_fwd && early && !fwd_block && hc->n_exc > 0 && hc->n_exc <= fwd_k;
            fwd_block = 0;
            if (phase_sweeps > (uint64_t)(64 * ((uint64_t)nn + 64)) || wall_s() > kSolveWallLimitS) {
                (void)hipStreamSynchronize(st);
                err = "push/relabel did not converge (sweeps " + std::to_string(phase_sweeps) + ", " +
                      std::to_string(wall_s()) + " s)";
                return KS_E_DEVICE;
            }
            cur ^= 1;
        }
        flush_bf();
        KS_CHECK(hipEventRecord(s.ev[5], st));
        KS_CHECK(hipEventSynchronize(s.ev[5]));
        ms_sat += ev_ms(s.ev[2], s.ev[3]);
        ms_cycles += ev_ms(s.ev[3], s.ev[5]);
        return rc;
    };

    // warm start: the previous flow and prices (in place), fresh nodes priced off
    // their out-arcs, then a start at a small ε (≤ 8 cost units) saturating only
    // the arcs that violate it
    long long warm_thr = 0;
    if (use_warm && !fb) {
        if (o.warm_shift >= 0)
            hipLaunchKernelGGL(k_price_shift, dim3(grid_for(s.ncap, 2048)), dim3(BLK), 0, st, (int)s.ncap,
                               (const unsigned long long*)s.n_cshift.p, (const int*)s.perm.p, mult, s.nd.p);
        hipLaunchKernelGGL(k_fresh_prices, dim3(grid_for(s.ncap, 2048)), dim3(BLK), 0, st, (int)s.ncap,
                           (const unsigned char*)s.n_fresh.p, (const int*)s.perm.p, g);
        if (m2) hipLaunchKernelGGL(k_max_viol, dim3(grid_for(m2, 2048)), dim3(BLK), 0, st, g, (long long)m2);
        KS_CHECK(read_ctl());
        const long long viol = s.h_ctl->gu_L;
        constexpr long long kWarmUnits = 8;   // the first warm phase at ≤ 8 cost units
        long long e0 = std::max<long long>(1, std::min<long long>({viol, kWarmUnits * mult, eps}));
        if (s.cell_layout && (alpha & (alpha - 1)) == 0)   // a power of two ≥ the violation (cell ladder)
            while (e0 & (e0 - 1)) e0 += e0 & -e0;
        warm_thr = e0;
        eps = e0 * alpha;   // the first phase runs at e0
        KS_CHECK(hipMemsetAsync(&s.ctl.p->gu_L, 0, sizeof(long long), st));
        if (cycle_log) {   // diagnostics: the carried prices' span (in cost units) and the start
            std::vector<long long> h((size_t)4 * nn);
            KS_CHECK(hipMemcpyAsync(h.data(), s.nd.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost, st));
            KS_CHECK(hipStreamSynchronize(st));
            long long lo = INF64, hi2 = -INF64;
            for (int v = 0; v < nn; ++v) {
                lo = std::min(lo, h[(size_t)4 * v]);
                hi2 = std::max(hi2, h[(size_t)4 * v]);
            }
            std::fprintf(stderr, "warm start: largest violation %.3f units, first phase at %.3f units, price span %.1f units\n",
                         (double)viol / mult, (double)e0 / mult, (double)(hi2 - lo) / mult);
        }
    }

    // ---- the cell solver (ks_cell.h): every cell's whole solve in one workgroup,
    // one launch for all cells; per-cell status and counters come back in CellOut
    const int ncells = (int)s.h_cells.size();
    const long long eps_cells = eps;   // ε before the first phase's division (as the loop below)
    double ms_cell = 0;
    unsigned long long cell_ctr[5] = {0, 0, 0, 0, 0};   // scans, visits, pushes, relabels, gu scans
    unsigned long long cell_rounds = 0, cticks_max = 0, cticks_sum = 0;
    auto run_cells = [&](int mode) -> int {
        CellArgs a{};
        a.pos = s.pos.p;
        a.cp = s.cl_pos.p;
        a.first = s.first.p;
        a.m2 = (int)s.m2cap;
        a.nd = s.nd.p;
        a.excess = s.excess.p;
        a.cells = s.cells.p;
        a.ncells = ncells;
        a.nn = nn;
        a.lists = s.cl_lists.p;
        a.rl_node = s.cl_rln.p;
        a.rl_p = s.cl_rlp.p;
        a.out = s.cl_out.p;
        a.mult = mult;
        a.eps_start = eps_cells;
        a.sat_thr0 = warm_thr;
        a.warm = use_warm ? (o.warm_start >= 2 ? 2 : 1) : 0;
        a.alpha = alpha;
        a.pr_div = (int)pr_div;
        a.use_pr = use_pr ? 1 : 0;
        a.pr_cap = pr_cap;
        a.use_prc = (use_pr && o.price_refine == 1 && !use_warm && mode == 0) ? 1 : 0;
        a.prc_cap = (o.fault_inject & 32) ? 32 : 4096;
        a.gi = gi_base;
        a.bound = o.bf_bound < 0 ? 0 : 1;
        a.phase_exit = phase_exit;
        a.phase_frac = phase_frac;
        a.mode = mode;
        a.max_nodes = s.cell_max;
        a.timeout_ticks = (unsigned long long)(kCellLimitS * 1e8);
        a.diag = cycle_log ? 1 : 0;
        // TESTS ONLY (fault_inject bit 4): the middle cell gives up after 40 operations
        a.fault_cell = (o.fault_inject & 16) && mode == 0 ? ncells / 2 : -1;
        a.fault_ops = 40;
        a.cyc_lg = (o.fault_inject & 128) ? 5 : 10;   // (ks_cell.hip CYC_LOG)
        KS_CHECK(hipEventRecord(s.kev[2], st));
        {   // a launch the device refuses (its LDS) → the multi-kernel engine instead; any
            // other launch error is reported (it used to disable the cell solver)
            bool refused = false;
            const hipError_t le = cell_launch(a, s.cl_bad.p, s.lds_limit, st, &refused);
            if (le != hipSuccess) {
                (void)hipGetLastError();
                if (refused) return (int)CS_RANGE;
                err = std::string("cell solver launch: ") + hipGetErrorString(le);
                return KS_E_DEVICE;
            }
        }
        KS_CHECK(hipEventRecord(s.kev[3], st));
        KS_CHECK(hipMemcpyAsync(s.h_cell_out.data(), s.cl_out.p, ncells * sizeof(CellOut), hipMemcpyDeviceToHost, st));
        KS_CHECK(hipStreamSynchronize(st));
        ms_cell += ev_ms(s.kev[2], s.kev[3]);
        int worst = CS_OK, pmax = 0;
        for (const CellOut& o : s.h_cell_out)
            if (o.status == CS_RANGE) return (int)CS_RANGE;
        for (const CellOut& o : s.h_cell_out) {
            if (o.status != CS_OK && (worst == CS_OK || worst == CS_INFEASIBLE)) worst = o.status;
            pmax = std::max(pmax, o.phases);
            sweeps += o.sweeps;
            gus += o.updates;
            cell_rounds += o.bf_rounds;
            cell_ctr[0] += o.scans;
            cell_ctr[1] += o.visits;
            cell_ctr[2] += o.pushes;
            cell_ctr[3] += o.relabels;
            cell_ctr[4] += o.gu_scans;
            prc_cycles += o.cycles;
            prc_rejected += o.rejected;
            cticks_max = std::max<unsigned long long>(cticks_max, o.ticks);
            cticks_sum += o.ticks;
        }
        phases += pmax;
        if (cycle_log) {   // per-operation device time of the slowest cell (ks_opts.log_cycles)
            size_t w = 0;
            for (size_t i = 1; i < s.h_cell_out.size(); ++i)
                if (s.h_cell_out[i].ticks > s.h_cell_out[w].ticks) w = i;
            const CellOut& o = s.h_cell_out[w];
            static const char* names[CELL_NOPS] = {"sat", "gu_init", "bf", "gu_fin", "sweep", "pr_init", "pr", "pr_fin",
                                                   "cyc"};
            std::fprintf(stderr, "cell %zu of %d: %.3f ms, phases %d updates %d sweeps %llu rounds %llu:", w, ncells,
                         o.ticks / 1e5, o.phases, o.updates, o.sweeps, o.bf_rounds);
            for (int i = 0; i < CELL_NOPS; ++i)
                if (o.op_n[i])
                    std::fprintf(stderr, " %s %u x %.2f us (items %.2f..%.2f)", names[i], o.op_n[i],
                                 o.op_ticks[i] / 100.0 / o.op_n[i], o.first_ticks[i] / 100.0 / o.op_n[i],
                                 o.item_ticks[i] / 100.0 / o.op_n[i]);
            static const char* const steps[4] = {"sweep", "bf", "pr", "sat"};
            for (int s = 0; s < 4; ++s) {
                std::fprintf(stderr, "\n  %s items:", steps[s]);
                for (int c = 0; c < 7; ++c)
                    if (o.cls_n[8 * s + c])
                        std::fprintf(stderr, " c%d %u x %.2f us", c, o.cls_n[8 * s + c],
                                     o.cls_ticks[8 * s + c] / 100.0 / o.cls_n[8 * s + c]);
            }
            std::fprintf(stderr, "\n  finish: cycles %d searches %d parents %u marked %u leaders %u closed %u", o.cycles,
                         o.searches, o.cyc_dbg[0], o.cyc_dbg[1], o.cyc_dbg[2], o.cyc_dbg[3]);
            std::fprintf(stderr, "\n  ms by phase:");
            for (int i = 0; i < 8; ++i)
                if (o.phase_ticks[i]) std::fprintf(stderr, " %s%d %.2f", i == 7 ? "pr/" : "p", i + 1, o.phase_ticks[i] / 1e5);
            static const char* const sz[6] = {"<=16", "<=64", "<=256", "<=1k", "<=4k", ">4k"};
            for (int h = 0; h < 12; ++h) {
                if (h % 6 == 0) std::fprintf(stderr, "\n  %s by frontier:", h ? "bf" : "sweep");
                if (o.hist_n[h])
                    std::fprintf(stderr, " %s %u x %.2f us", sz[h % 6], o.hist_n[h], o.hist_t[h] / 100.0 / o.hist_n[h]);
            }
            std::fprintf(stderr, "\n");
        }
        return worst;
    };
    auto cell_status = [&](int cs, const char* what) -> int {
        if (cs == CS_OK) return KS_OK;
        if (cs == CS_INFEASIBLE) {
            status = KS_E_INFEASIBLE;
            err = std::string("infeasible: some supply cannot reach a demand node (cell solver, ") + what + ")";
            return KS_OK;
        }
        err = std::string("cell solver did not converge (") + (cs == CS_TIMEOUT ? "wall-clock limit" : "step cap") +
              ", " + what + ")";
        return KS_E_DEVICE;
    };
    if (s.cell_layout) {
        KS_CHECK(s.cl_pos.ensure(std::max<int64_t>(m2, 1)));
        KS_CHECK(hipEventRecord(s.ev[3], st));
        const int cs = run_cells(0);
        if (cs < 0) return cs;
        if (cs == CS_RANGE) {   // a value the compact record cannot hold: the multi-kernel engine instead
            s.cell_refused = true;
            s.cell_layout = false;
            s.csr_valid = false;
            // the warm start's price shift is already in the carried prices: the retry
            // must not apply it a second time
            if (use_warm) KS_CHECK(hipMemsetAsync(s.n_cshift.p, 0, s.nstore * sizeof(unsigned long long), st));
            return solve(res, warm, err);
        }
        KS_CHECK(hipEventRecord(s.ev[5], st));
        KS_CHECK(hipEventSynchronize(s.ev[5]));
        ms_cycles += ev_ms(s.ev[3], s.ev[5]);
        if (cs == CS_TIMEOUT || cs == CS_NOCONV) {
            // Per-cell fallback: only the cells that gave up are solved again, on the
            // multi-kernel engine (engine order, the state carried across the rebuild:
            // the converged cells keep their optimal flows and prices, the failing ones
            // restart cold). One hard cell no longer discards the batch.
            std::vector<int> bad;
            for (size_t i = 0; i < s.h_cell_out.size(); ++i)
                if (s.h_cell_out[i].status == CS_TIMEOUT || s.h_cell_out[i].status == CS_NOCONV) bad.push_back((int)i);
            s.fb_cells = bad;
            s.fb_active = true;
            s.cell_layout = false;
            s.csr_valid = false;
            const int rc = solve(res, warm, err);
            s.fb_active = false;
            s.fb_cells.clear();
            res.cell_fallbacks = bad.size();
            res.solver = 1;
            res.cells = ncells;
            return rc;
        }
        if (int rc = cell_status(cs, "solve")) return rc;
        eps = 1;
    } else do {
        eps = std::max<long long>(1, eps / alpha);
        ++phases;
        // After a failed refinement the flow is feasible and ε-optimal at the old ε:
        // saturating only the arcs that violate the new ε (rc < −ε) is a valid start
        // (push-relabel at ε needs an ε-optimal pseudoflow, not a 0-optimal one) and
        // disturbs far less than saturating every negative arc.
        // warm_start 2: every phase of a warm solve saturates only the arcs that
        // violate its ε (the previous optimum's arcs in [−1, 0) stay as they are)
        // per-cell fallback: the cold ε ladder, every phase saturating only the arcs
        // that violate its ε (the converged cells' optimal flows stay untouched)
        long long sat_thr = phases == 1 && use_warm && !fb
                                ? warm_thr
                                : ((pr_failed || fb || (use_warm && o.warm_start >= 2)) ? eps : 0LL);
        pr_failed = false;
        const bool last_phase = eps / alpha < 1 || eps <= 1 || (use_pr && eps * pr_div < mult);
        // the phase before the final one drains completely when the cycle-cancelling
        // finish replaces the final phase
        const long long eps_next = std::max<long long>(1, eps / alpha);
        const bool before_last = !last_phase && !prc_tried &&
                                 (eps_next / alpha < 1 || eps_next <= 1 || (use_pr && eps_next * pr_div < mult));
        const bool prc_now = use_prc && before_last;
        // two phases before the last: the finish may follow this phase instead
        // (run_phase prc_early) when the flow is already close to optimal
        const long long eps_next2 = std::max<long long>(1, eps_next / alpha);
        const bool before_last2 = !last_phase && !before_last &&
                                  (eps_next2 / alpha < 1 || eps_next2 <= 1 || (use_pr && eps_next2 * pr_div < mult));
        // walk slack > 1 only while a finer phase or price refinement still follows
        // (ε > 1): a phase at ε = 1 must end 1-optimal (fault_inject bit 0 breaks
        // exactly this, for the certificate-recovery test)
        const int walk_sl = (eps > 1 || (o.fault_inject & 1)) ? aug_slack : 1;
        int prc_early = 0;
        // (only from a phase at most two cost units coarse: earlier, the finish has
        // too many cycles to cancel — config 4 with D = 24 at 2.6 units: 26 vs 20 ms)
        const bool may_early = use_prc && !prc_tried && before_last2 && !use_warm && !fb && eps <= 2 * mult;
        const int rc = run_phase(eps, sat_thr, !last_phase && !prc_now, walk_sl, may_early ? &prc_early : nullptr);
        if (rc == KS_E_INFEASIBLE) {
            status = rc;
            break;
        }
        if (rc) return rc;
        if (prc_now || prc_early) {   // the feasible flow of the last coarse phase: cancel its negative cycles
            prc_tried = true;
            int used = 0;
            const int pr = prc_refine(&used, prc_early ? std::min(prc_cap, 1024) : prc_cap);
            if (pr < 0) return pr;
            if (pr == 1) {
                eps = 1;
                break;
            }
            pr_failed = true;   // the final phase follows, saturating only its violations
            continue;
        }
        // certify optimality early: a flow that is 1-optimal (scaled) is optimal.
        // Tried once ε is below 1/32 of a cost unit, where it usually succeeds.
        if (use_pr && eps > 1 && eps * pr_div < mult) {
            int used = 0;
            const int pr = price_refine(1, &used, pr_cap);
            if (pr < 0) return pr;
            if (pr == 1) eps = 1;
            else pr_failed = true;
        }
    } while (eps > 1);

    if (cycle_log)
        std::fprintf(stderr, "solve phases %d updates %llu (forward %llu) early phase ends %llu\n", phases,
                     (unsigned long long)gus, (unsigned long long)fwd_updates, (unsigned long long)early_exits);
    if (status == KS_E_INFEASIBLE && !s.cell_layout)
        err = "infeasible: some supply cannot reach a demand node (code " + std::to_string(s.h_ctl->infeasible) +
              ", phase " + std::to_string(phases) + ", eps " + std::to_string(eps) + ", updates " +
              std::to_string(gus) + ", sweeps " + std::to_string(sweep_launches) + ")";

    // ------------------------------------------------------------ verify ---
    // Conservation, capacity, 1-optimality of the final prices (scaled units), the
    // int64 cost and the flow value measured from the resident flow. → verify_bad bits
    const int vgrid = grid_for(hi, 2048);
    long long tot_cost = 0, tot_flow = 0;
    auto verify = [&](int* bad) -> int {
        if (cp_dirty) {   // the compact solve's residuals back into the 32-B records first
            hipLaunchKernelGGL(k_unpack_pos, dim3(grid_for(m2, 4096)), dim3(BLK), 0, st, (long long)m2,
                               (const CPos*)s.cpos.p, s.pos.p);
            cp_dirty = false;
        }
        if ((o.fault_inject & 64) && m2)   // TESTS ONLY: break conservation, not the excess words
            hipLaunchKernelGGL(k_break_conservation, dim3(1), dim3(64), 0, st, g, (long long)m2);
        KS_CHECK(hipMemsetAsync(&s.ctl.p->verify_bad, 0, sizeof(int), st));
        KS_CHECK(set_eps(1));
        hipLaunchKernelGGL(k_drain_all, dim3((std::max(1, s.nheavy) + BLK - 1) / BLK), dim3(BLK), 0, st, g);
        KS_CHECK(s.vbal.ensure(std::max<int64_t>(s.ncap, 1)));
        KS_CHECK(hipMemsetAsync(s.vbal.p, 0, std::max<int64_t>(s.ncap, 1) * sizeof(long long), st));
        if (hi)
            hipLaunchKernelGGL(k_verify_arcs, dim3(vgrid), dim3(BLK), 0, st, g, hi, (const unsigned char*)s.a_alive.p,
                               (const int*)s.fwd.p, (const int*)s.a_src.p, (const int*)s.a_dst.p,
                               (const long long*)s.n_supply.p, (const long long*)s.a_low.p,
                               (const long long*)s.a_cap.p, (const long long*)s.a_cost.p, s.flows.p, s.part.p,
                               s.part.p + 4096, s.vbal.p);
        if (s.ncap)
            hipLaunchKernelGGL(k_verify_balance, dim3(grid_for(s.ncap, 2048)), dim3(BLK), 0, st, g, (int)s.ncap,
                               (const unsigned char*)s.n_alive.p, (const long long*)s.n_supply.p,
                               (const long long*)s.vbal.p);
        if (m2) hipLaunchKernelGGL(k_verify_opt, dim3(grid_for(m2, 2048)), dim3(BLK), 0, st, g, (long long)m2);
        hipLaunchKernelGGL(k_verify_nodes, dim3(ngrid), dim3(BLK), 0, st, g);
        std::vector<long long> parts(hi ? vgrid : 0), partf(hi ? vgrid : 0);
        if (hi) {
            KS_CHECK(hipMemcpyAsync(parts.data(), s.part.p, vgrid * sizeof(long long), hipMemcpyDeviceToHost, st));
            KS_CHECK(hipMemcpyAsync(partf.data(), s.part.p + 4096, vgrid * sizeof(long long), hipMemcpyDeviceToHost,
                                    st));
        }
        KS_CHECK(read_ctl());
        tot_cost = tot_flow = 0;
        for (long long x : parts) tot_cost += x;
        for (long long x : partf) tot_flow += x;
        *bad = s.h_ctl->verify_bad;
        return KS_OK;
    };
    KS_CHECK(hipEventRecord(s.ev[6], st));
    if (status == KS_OK) {
        if (o.fault_inject & 2)   // TESTS ONLY: break the certificate, not the flow
            hipLaunchKernelGGL(k_perturb_price, dim3(1), dim3(1), 0, st, g, 0, 1000 * mult);
        int bad = 0;
        int rc = verify(&bad);
        if (rc) return rc;
        // A failed optimality certificate on a feasible flow is repaired, not fatal:
        // price refinement at ε = 1 (the flow may be optimal, only its prices off),
        // else one more ε = 1 phase from the current flow (saturating only the arcs
        // that violate 1-optimality), then verification again. Capacity and
        // conservation violations stay fatal (KS_E_VERIFY).
        for (int attempt = 0; attempt < 2 && bad == 2; ++attempt) {
            ++res.recoveries;
            if (s.cell_layout) {   // the same repair inside each cell's workgroup
                const int cs = run_cells(1);
                if (cs < 0) return cs;
                if (int rc2 = cell_status(cs, "certificate recovery")) return rc2;
                if (status != KS_OK) break;
                rc = verify(&bad);
                if (rc) return rc;
                continue;
            }
            int used = 0;
            const int pr = price_refine(1, &used, 4 * pr_cap);
            if (pr < 0) return pr;
            if (pr == 0) {
                ++phases;
                rc = run_phase(1, 1, false, 1);
                if (rc == KS_E_INFEASIBLE) {
                    status = rc;
                    err = "infeasible during certificate recovery";
                    break;
                }
                if (rc) return rc;
            }
            rc = verify(&bad);
            if (rc) return rc;
        }
        if (status == KS_OK && bad && o.verify) {
            status = KS_E_VERIFY;
            err = std::string("on-device verification failed (") + ((bad & 1) ? "capacity " : "") +
                  ((bad & 2) ? "optimality " : "") + ((bad & 4) ? "conservation" : "") + ")";
        }
        // warm starts: replace the carried prices by the flow's canonical ones (the
        // next round starts from prices without history). Kept only if the
        // Bellman-Ford converges; the certificate holds either way.
        if (status == KS_OK && !bad && o.warm_start > 0 && o.warm_canon >= 0 && !s.cell_layout) {
            int used = 0;
            const int pr = price_refine(1, &used, 4 * pr_cap, 1);
            if (pr < 0) return pr;
            if (cycle_log) std::fprintf(stderr, "canonical prices: %s after %d rounds\n", pr ? "set" : "not converged", used);
        }
    }
    if (cp_dirty) {   // (a solve that ended without verification: Pos stays the authoritative copy)
        hipLaunchKernelGGL(k_unpack_pos, dim3(grid_for(m2, 4096)), dim3(BLK), 0, st, (long long)m2,
                           (const CPos*)s.cpos.p, s.pos.p);
        cp_dirty = false;
    }
    KS_CHECK(hipEventRecord(s.ev[7], st));
    unsigned long long hc[CTR_SHARDS * NCTR];
    KS_CHECK(hipMemcpyAsync(hc, s.ctr.p, sizeof(hc), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    unsigned long long tc[NCTR] = {0};
    for (int i = 0; i < CTR_SHARDS; ++i)
        for (int k = 0; k < NCTR; ++k) tc[k] += hc[i * NCTR + k];
    if (s.cell_layout) {
        tc[C_SCAN] += cell_ctr[0];
        tc[C_VISIT] += cell_ctr[1];
        tc[C_PUSH] += cell_ctr[2];
        tc[C_RELABEL] += cell_ctr[3];
        tc[C_GUSCAN] += cell_ctr[4];
        tc[C_BFROUND] += cell_rounds;
    }
    if (cycle_log)
        std::fprintf(stderr, "solve tail walks to a deficit %llu, hops %llu, recoveries %d\n", tc[C_AUGWALK],
                     tc[C_AUGHOP], res.recoveries);

    res.total_cost = tot_cost;
    res.flow_value = tot_flow;
    res.phases = phases;
    res.sweeps = sweeps;
    res.arc_scans = tc[C_SCAN];
    res.node_visits = tc[C_VISIT];
    res.pushes = tc[C_PUSH];
    res.relabels = tc[C_RELABEL];
    res.global_updates = gus;
    res.gu_iterations = tc[C_BFROUND];
    res.ms_phase[0] = ev_ms(s.ev[0], s.ev[1]);
    res.ms_phase[1] = ms_sat;
    res.ms_phase[2] = ms_cycles;
    res.ms_phase[3] = ms_pr;
    res.ms_phase[4] = ev_ms(s.ev[6], s.ev[7]);
    res.ms_phase[5] = 1e3 * wall_s();
    res.gu_arc_scans = tc[C_GUSCAN];
    res.gu_leaf_scans = tc[C_GULEAF];
    res.fs_arc_scans = tc[C_FSSCAN];
    res.sweep_launches = sweep_kernels;
    res.ms_sweep_kernels = ms_sw_k;
    res.gu_launches = bf_launches;
    res.ms_gu_kernels = ms_bf_k;
    res.fs_launches = fs_launches;
    res.ms_fs_kernels = ms_fs_k;
    res.fwd_updates = fwd_updates;
    res.solver = s.cell_layout ? 1 : 0;
    res.cells = s.cell_layout ? ncells : 0;
    res.ms_cell_kernel = ms_cell;
    res.cell_ticks_max = cticks_max;
    res.cell_ticks_sum = cticks_sum;
    res.status = status;
    res.cycles_cancelled = (uint64_t)prc_cycles;
    res.cycles_rejected = (uint64_t)prc_rejected;
    KS_CHECK(hipMemsetAsync(s.n_cshift.p, 0, s.nstore * sizeof(unsigned long long), st));
    if (status == KS_OK) {
        KS_CHECK(hipMemsetAsync(s.n_fresh.p, 0, s.nstore, st));
        KS_CHECK(hipStreamSynchronize(st));
        s.solved = true;
        s.has_prev = true;
    } else {
        s.has_prev = false;   // a failed solve leaves no usable warm state
    }
    return status;
}

}  // namespace ks
