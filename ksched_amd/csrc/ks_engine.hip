// ks_engine.hip — gfx950 ε-scaling push-relabel min-cost flow engine.
//
// Replaces the Flowlessly solve behind ksched's placement.Solver
// (scheduling/flow/placement/solver.go:30-34, 60-90). Algorithm and data
// layout: DESIGN.md §3-§4. Summary:
//
//   build      residual CSR from the device-resident input arcs: a stable radix
//              sort of the 2m (tail, slot) keys (hipcub over rocPRIM), lower
//              bounds transformed into node excess, nodes split by degree into
//              light (thread per node), medium (wave per node) and heavy
//              (1024-arc chunks, one workgroup per chunk) lists.
//   phases     ε ← ε/α; saturate every residual arc with negative reduced cost;
//              global price update; then synchronous push/relabel sweeps until
//              no node holds positive excess, with periodic global updates.
//   sweep      every node with positive excess discharges once per sweep
//              against a price SNAPSHOT (prices are double-buffered: the sweep
//              reads P[q] and writes P[q^1]); a node relabels only if it
//              saturated all of its own admissible arcs, and its relabel amount
//              also covers arcs that may gain residual capacity from concurrent
//              pushes in the same sweep (reduced cost in (0, ε]) — this keeps
//              ε-optimality without locks.
//   heavy hubs pushes into a hub (cluster aggregator, sink: in-degree ~10^5)
//              are wave-aggregated into a 16-way sharded inbox that the hub's
//              first chunk drains; hub chunks claim excess with a CAS and the
//              last-arriving chunk (RMW-atomic arrival counter) finalises the
//              relabel.
//   verify     on-device: conservation (all excess zero), capacity, and
//              1-optimality of the final prices in scaled units (costs scaled by
//              n+1, so 1-optimal ⇒ optimal); the total cost is reduced in int64.
//
// All in-kernel cross-workgroup communication uses device-scope RMW atomics;
// everything else is handed over at kernel boundaries.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ks_engine.h"

namespace ks {
namespace {

constexpr int BLK = 256;
constexpr int WAVE = 64;
constexpr int WPB = BLK / WAVE;
constexpr int LIGHT_MAX = 32;      // degree ≤ 32: one thread per node
constexpr int MEDIUM_MAX = 4096;   // degree ≤ 4096: one wave per node
constexpr int CHUNK = 1024;        // heavy hubs: 1024 residual arcs per workgroup
constexpr int PER_T = CHUNK / BLK;
constexpr int SHARDS = 16;         // inbox shards per heavy hub
constexpr int MAXB = 64;           // max kernels per host batch
constexpr int NCTR = 8;
constexpr int CTR_SHARDS = 64;
constexpr long long INF64 = 0x3fffffffffffffffLL;
constexpr long long LEN_CAP = 1LL << 40;   // global-update arc length clamp (safe: DESIGN.md §3.3)
constexpr double kSolveWallLimitS = 120.0; // host-side guard against a non-converging solve
constexpr long long kTraceMax = 1 << 16;  // sweeps recorded when KS_TRACE is set

enum { C_SCAN = 0, C_VISIT = 1, C_PUSH = 2, C_RELABEL = 3, C_GUSCAN = 4 };

struct Ctl {
    long long eps;
    int active_prev;
    int infeasible;
    int active[MAXB];
    int gu_prev;
    int pad0;
    int gu_changed[MAXB];
    int verify_bad;
    int pad1;
};

struct HItem {
    int node, hid, begin, end;
};

struct DG {
    int n, m;
    const int* first;
    const int* head;
    const int* rev;
    long long* rcap;
    const long long* cost;
    long long* excess;
    long long* p0;
    long long* p1;
    const int* hidx;
    long long* inbox;
    const int* light;
    int nlight;
    const int* medium;
    int nmedium;
    const HItem* hitems;
    int nhitems;
    int nheavy;
    const int* hnode;
    const int* hnchunks;
    int* harrive;
    long long* hmin;
    int* hunsat;
    long long* dist;
    Ctl* ctl;
    unsigned long long* ctr;
    unsigned* trace;   // optional per-sweep [visits, relabels] (KS_TRACE diagnostics)
    int nmblocks;   // medium blocks = ceil(nmedium / WPB)
};

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
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

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
__device__ __forceinline__ long long floordiv(long long a, long long b) {  // b > 0
    long long q = a / b;
    if ((a % b) != 0 && a < 0) --q;
    return q;
}

// Per-lane pending hub push: wave-aggregated into the hub's sharded inbox.
struct Pend {
    int key;
    long long val;
};

__device__ __forceinline__ void push_excess(const DG& g, int w, long long d, Pend& pd) {
    const int h = g.hidx[w];
    if (h < 0) {
        atom_add(&g.excess[w], d);
    } else if (pd.key == h) {
        pd.val += d;
    } else if (pd.key < 0) {
        pd.key = h;
        pd.val = d;
    } else {
        atom_add(&g.inbox[h * SHARDS + (blockIdx.x & (SHARDS - 1))], d);
    }
}

// Must be called by all 64 lanes of a wave at a converged point.
__device__ __forceinline__ void flush_pending(const DG& g, Pend& pd) {
    const int lane = lane_id();
    for (;;) {
        const unsigned long long msk = __ballot(pd.key >= 0);
        if (!msk) break;
        const int leader = __ffsll((long long)msk) - 1;
        const int k = __shfl(pd.key, leader);
        const long long s = wave_sum(pd.key == k ? pd.val : 0);
        if (lane == leader) atom_add(&g.inbox[k * SHARDS + (blockIdx.x & (SHARDS - 1))], s);
        if (pd.key == k) pd.key = -1;
    }
}

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

// Drain a hub's inbox shards into its excess. Returns the drained amount.
__device__ __forceinline__ long long drain_inbox(const DG& g, int h, int x) {
    long long s = 0;
#pragma unroll
    for (int k = 0; k < SHARDS; ++k) s += atom_exch(&g.inbox[h * SHARDS + k], 0LL);
    if (s) atom_add(&g.excess[x], s);
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

// ===================================================================== build ===
__global__ void k_make_keys(int m, const int* __restrict__ src, const int* __restrict__ dst,
                            unsigned* __restrict__ keys, int* __restrict__ vals) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < m; i += (long long)gridDim.x * BLK) {
        keys[2 * i] = (unsigned)src[i];
        keys[2 * i + 1] = (unsigned)dst[i];
        vals[2 * i] = (int)(2 * i);
        vals[2 * i + 1] = (int)(2 * i + 1);
    }
}

__global__ void k_scatter_pos(long long m2, const int* __restrict__ vals, int* __restrict__ pos_of) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK)
        pos_of[vals[p]] = (int)p;
}

__global__ void k_fill(long long m2, long long mult, const int* __restrict__ vals, const int* __restrict__ pos_of,
                       const int* __restrict__ src, const int* __restrict__ dst, const long long* __restrict__ low,
                       const long long* __restrict__ cap, const long long* __restrict__ cost, int* __restrict__ head,
                       int* __restrict__ rev, long long* __restrict__ rcap, long long* __restrict__ scost,
                       int* __restrict__ fwd) {
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK) {
        const int v = vals[p];
        const int i = v >> 1;
        const bool r = v & 1;
        head[p] = r ? src[i] : dst[i];
        rev[p] = pos_of[v ^ 1];
        rcap[p] = r ? 0 : cap[i] - low[i];
        scost[p] = (r ? -cost[i] : cost[i]) * mult;
        if (!r) fwd[i] = (int)p;
    }
}

__global__ void k_first(int n, long long m2, const unsigned* __restrict__ keys, int* __restrict__ first) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v <= n; v += (long long)gridDim.x * BLK) {
        long long lo = 0, hi = m2;
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (keys[mid] < (unsigned)v) lo = mid + 1; else hi = mid;
        }
        first[v] = (int)lo;
    }
}

__global__ void k_node_init(int n, const long long* __restrict__ supply, const int* __restrict__ first,
                            long long* __restrict__ excess, long long* __restrict__ p0, long long* __restrict__ p1,
                            unsigned char* __restrict__ cls, int* __restrict__ hidx) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < n; v += (long long)gridDim.x * BLK) {
        excess[v] = supply[v];
        p0[v] = 0;
        p1[v] = 0;
        const int d = first[v + 1] - first[v];
        cls[v] = d <= LIGHT_MAX ? 0 : (d <= MEDIUM_MAX ? 1 : 2);
        hidx[v] = -1;
    }
}

__global__ void k_lower_bounds(int m, const int* __restrict__ src, const int* __restrict__ dst,
                               const long long* __restrict__ low, long long* __restrict__ excess) {
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < m; i += (long long)gridDim.x * BLK) {
        const long long l = low[i];
        if (l) {
            atom_add(&excess[src[i]], -l);
            atom_add(&excess[dst[i]], l);
        }
    }
}

__global__ void k_set_hidx(int nheavy, const int* __restrict__ hnode, int* __restrict__ hidx) {
    const int h = blockIdx.x * BLK + threadIdx.x;
    if (h < nheavy) hidx[hnode[h]] = h;
}

struct ClassIs {
    const unsigned char* cls;
    unsigned char c;
    __host__ __device__ bool operator()(const int& v) const { return cls[v] == c; }
};

// ================================================= saturate (phase start) ===
// Push the full residual capacity of every arc with negative reduced cost
// (Goldberg's refine start); reads the authoritative price buffer p0.
__global__ __launch_bounds__(BLK) void k_saturate(DG g) {
    const long long* P = g.p0;
    Pend pd{-1, 0};
    Cnt c;
    int b = blockIdx.x;
    if (b < g.nhitems) {
        __shared__ long long sh[WPB];
        const HItem it = g.hitems[b];
        const long long px = P[it.node];
        long long tot = 0;
        for (int k = 0; k < PER_T; ++k) {
            const int a = it.begin + threadIdx.x + k * BLK;
            if (a < it.end) {
                const long long r = g.rcap[a];
                if (r > 0) {
                    const int w = g.head[a];
                    if (g.cost[a] + px - P[w] < 0) {
                        g.rcap[a] = 0;
                        g.rcap[g.rev[a]] += r;
                        push_excess(g, w, r, pd);
                        tot += r;
                        c.push++;
                    }
                }
            }
        }
        flush_pending(g, pd);
        tot = block_sum(tot, sh);
        if (threadIdx.x == 0 && tot) atom_add(&g.excess[it.node], -tot);
        flush_counters(g, c);
        return;
    }
    b -= g.nhitems;
    if (b < g.nmblocks) {
        const int wi = b * WPB + (threadIdx.x >> 6);
        const int lane = lane_id();
        if (wi < g.nmedium) {
            const int v = g.medium[wi];
            const long long pv = P[v];
            const int e = g.first[v + 1];
            long long tot = 0;
            for (int a = g.first[v] + lane; a < e; a += WAVE) {
                const long long r = g.rcap[a];
                if (r > 0) {
                    const int w = g.head[a];
                    if (g.cost[a] + pv - P[w] < 0) {
                        g.rcap[a] = 0;
                        g.rcap[g.rev[a]] += r;
                        push_excess(g, w, r, pd);
                        tot += r;
                        c.push++;
                    }
                }
            }
            tot = wave_sum(tot);
            if (lane == 0 && tot) atom_add(&g.excess[v], -tot);
        }
        flush_pending(g, pd);
        flush_counters(g, c);
        return;
    }
    b -= g.nmblocks;
    const int i = b * BLK + threadIdx.x;
    if (i < g.nlight) {
        const int v = g.light[i];
        const long long pv = P[v];
        const int e = g.first[v + 1];
        long long tot = 0;
        for (int a = g.first[v]; a < e; ++a) {
            const long long r = g.rcap[a];
            if (r > 0) {
                const int w = g.head[a];
                if (g.cost[a] + pv - P[w] < 0) {
                    g.rcap[a] = 0;
                    g.rcap[g.rev[a]] += r;
                    push_excess(g, w, r, pd);
                    tot += r;
                    c.push++;
                }
            }
        }
        if (tot) atom_add(&g.excess[v], -tot);
    }
    flush_pending(g, pd);
    flush_counters(g, c);
}

__global__ void k_drain_all(DG g) {
    const int h = blockIdx.x * BLK + threadIdx.x;
    if (h < g.nheavy) drain_inbox(g, h, g.hnode[h]);
}

// =================================================== push/relabel sweep ===
__device__ __forceinline__ void light_discharge(const DG& g, int v, const long long* __restrict__ P,
                                                long long* __restrict__ PN, long long eps, Pend& pd, int& act,
                                                Cnt& c) {
    const long long e = g.excess[v];
    if (e <= 0) return;
    c.visit++;
    const long long pv = P[v];
    long long rem = e, minc = INF64;
    const int b = g.first[v], en = g.first[v + 1];
    int a = b;
    for (; a < en; ++a) {
        const long long r = g.rcap[a];
        const int w = g.head[a];
        const long long cr = g.cost[a] + pv - P[w];
        if (cr < 0) {
            if (r > 0) {
                const long long d = r < rem ? r : rem;
                g.rcap[a] = r - d;
                g.rcap[g.rev[a]] += d;
                push_excess(g, w, d, pd);
                c.push++;
                rem -= d;
                if (rem == 0) { ++a; break; }
            }
        } else if (r > 0 || cr <= eps) {
            minc = min(minc, cr);
        }
    }
    c.scan += a - b;
    const long long pushed = e - rem;
    if (pushed) atom_add(&g.excess[v], -pushed);
    long long np = pv;
    if (rem > 0) {
        if (minc >= INF64) g.ctl->infeasible = 1;
        else np = pv - (minc + eps);
        c.relabel++;
    }
    PN[v] = np;
    act |= (pushed > 0) | (rem > 0);
}

__device__ __forceinline__ void medium_discharge(const DG& g, int v, const long long* __restrict__ P,
                                                 long long* __restrict__ PN, long long eps, Pend& pd, int& act,
                                                 Cnt& c) {
    const int lane = lane_id();
    const long long e = g.excess[v];
    if (e <= 0) return;
    if (lane == 0) c.visit++;
    const long long pv = P[v];
    long long rem = e, minc = INF64;
    const int b = g.first[v], en = g.first[v + 1];
    for (int base = b; base < en; base += WAVE) {
        const int a = base + lane;
        const bool valid = a < en;
        long long r = 0, cr = 0;
        int w = 0;
        if (valid) {
            r = g.rcap[a];
            w = g.head[a];
            cr = g.cost[a] + pv - P[w];
            c.scan++;
        }
        const long long adm = (valid && cr < 0 && r > 0) ? r : 0;
        const long long incl = wave_incl_scan(adm, lane);
        const long long total = __shfl(incl, WAVE - 1);
        long long d = rem - (incl - adm);
        d = d < 0 ? 0 : (d > adm ? adm : d);
        if (d > 0) {
            g.rcap[a] = r - d;
            g.rcap[g.rev[a]] += d;
            push_excess(g, w, d, pd);
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
        flush_pending(g, pd);
        if (rem == 0) break;
    }
    if (lane == 0) {
        const long long pushed = e - rem;
        if (pushed) atom_add(&g.excess[v], -pushed);
    }
    long long np = pv;
    if (rem > 0) {
        minc = wave_min(minc);
        if (minc >= INF64) {
            if (lane == 0) g.ctl->infeasible = 1;
        } else {
            np = pv - (minc + eps);
        }
        if (lane == 0) c.relabel++;
    }
    if (lane == 0) PN[v] = np;
    act |= (e - rem > 0) | (rem > 0);
}

__device__ long long heavy_claim(long long* ex, long long want) {
    if (want <= 0) return 0;
    long long old = atom_add_ret(ex, 0);
    for (;;) {
        if (old <= 0) return 0;
        const long long take = old < want ? old : want;
        if (__hip_atomic_compare_exchange_strong(ex, &old, old - take, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return take;
    }
}

__device__ void heavy_chunk(const DG& g, const HItem& it, const long long* __restrict__ P,
                            long long* __restrict__ PN, long long eps, Pend& pd, int& act, Cnt& c) {
    __shared__ long long sh[WPB];
    __shared__ long long s_take;
    const int x = it.node, h = it.hid;
    const bool chunk0 = it.begin == g.first[x];
    if (chunk0 && threadIdx.x == 0) {
        if (drain_inbox(g, h, x)) act = 1;
    }
    const long long px = P[x];
    long long r[PER_T], cr[PER_T], adm[PER_T];
    int w[PER_T];
    long long mine = 0;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        r[k] = 0;
        cr[k] = 0;
        w[k] = 0;
        if (a < it.end) {
            r[k] = g.rcap[a];
            w[k] = g.head[a];
            cr[k] = g.cost[a] + px - P[w[k]];
            c.scan++;
        }
        adm[k] = (a < it.end && cr[k] < 0 && r[k] > 0) ? r[k] : 0;
        mine += adm[k];
    }
    long long Ac = 0;
    const long long excl = block_excl_scan(mine, sh, &Ac);
    if (threadIdx.x == 0) s_take = heavy_claim(&g.excess[x], Ac);
    __syncthreads();
    const long long take = s_take;
    long long rt = take - excl;
    rt = rt < 0 ? 0 : (rt > mine ? mine : rt);
    long long minc = INF64;
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
        const int a = it.begin + threadIdx.x * PER_T + k;
        long long d = adm[k] < rt ? adm[k] : rt;
        rt -= d;
        if (d > 0) {
            g.rcap[a] = r[k] - d;
            g.rcap[g.rev[a]] += d;
            push_excess(g, w[k], d, pd);
            c.push++;
            act = 1;
        }
        if (a < it.end) {
            if (cr[k] < 0) {
                if (r[k] - d > 0) minc = min(minc, cr[k]);
            } else if (r[k] > 0 || cr[k] <= eps) {
                minc = min(minc, cr[k]);
            }
        }
    }
    flush_pending(g, pd);
    minc = block_min(minc, sh);
    if (threadIdx.x == 0) {
        if (minc < INF64) atom_min_ret(&g.hmin[h], minc);
        if (take < Ac) atom_exch_i(&g.hunsat[h], 1);
        drain_vm();
        const int old = __hip_atomic_fetch_add(&g.harrive[h], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == g.hnchunks[h] - 1) {
            // last chunk of hub x in this sweep: finalise
            const long long mn = atom_exch(&g.hmin[h], INF64);
            const int unsat = atom_exch_i(&g.hunsat[h], 0);
            const long long ex = atom_add_ret(&g.excess[x], 0);
            long long np = px;
            if (!unsat && ex > 0) {
                if (mn >= INF64) g.ctl->infeasible = 1;
                else np = px - (mn + eps);
                c.relabel++;
            }
            if (ex > 0) {
                act = 1;
                c.visit++;
            }
            PN[x] = np;
            atom_exch_i(&g.harrive[h], 0);
        }
    }
}

__global__ __launch_bounds__(BLK) void k_sweep(DG g, int pos, int tidx) {
    const int prev = pos ? g.ctl->active[pos - 1] : g.ctl->active_prev;
    if (!prev) return;
    const long long eps = g.ctl->eps;
    const long long* P = (pos & 1) ? g.p1 : g.p0;
    long long* PN = (pos & 1) ? g.p0 : g.p1;
    Pend pd{-1, 0};
    Cnt c;
    int act = 0;
    int b = blockIdx.x;
    if (b < g.nhitems) {
        heavy_chunk(g, g.hitems[b], P, PN, eps, pd, act, c);
    } else {
        b -= g.nhitems;
        if (b < g.nmblocks) {
            const int wi = b * WPB + (threadIdx.x >> 6);
            if (wi < g.nmedium) medium_discharge(g, g.medium[wi], P, PN, eps, pd, act, c);
            flush_pending(g, pd);
        } else {
            b -= g.nmblocks;
            const int i = b * BLK + threadIdx.x;
            if (i < g.nlight) light_discharge(g, g.light[i], P, PN, eps, pd, act, c);
            flush_pending(g, pd);
        }
    }
    if (__any(act) && lane_id() == 0) g.ctl->active[pos] = 1;
    if (g.trace && tidx >= 0) {
        const long long v = wave_sum(c.visit), r = wave_sum(c.relabel);
        if (lane_id() == 0 && (v | r)) {
            const int cls = blockIdx.x < g.nhitems ? 3 : (blockIdx.x < g.nhitems + g.nmblocks ? 2 : -1);
            atomicAdd(&g.trace[4 * tidx], (unsigned)v);
            atomicAdd(&g.trace[4 * tidx + 1], (unsigned)r);
            if (cls > 0) atomicAdd(&g.trace[4 * tidx + cls], (unsigned)v);
        }
    }
    flush_counters(g, c);
}

// ===================================================== global price update ===
// Distances (in ε units) from the deficit nodes over residual arcs with length
// floor(rc/ε)+1 (clamped), by label-correcting Bellman-Ford sweeps.
__global__ void k_gu_init(DG g) {
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK)
        g.dist[v] = g.excess[v] < 0 ? 0 : INF64;
}

__device__ __forceinline__ long long relax_arc(const DG& g, int a, long long pu, const long long* __restrict__ P,
                                               long long eps) {
    if (g.rcap[a] <= 0) return INF64;
    const int v = g.head[a];
    const long long dv = g.dist[v];
    if (dv >= INF64) return INF64;
    long long len = floordiv(g.cost[a] + pu - P[v], eps) + 1;
    len = len < 0 ? 0 : (len > LEN_CAP ? LEN_CAP : len);
    const long long cand = dv + len;
    return cand < INF64 ? cand : INF64;
}

__global__ __launch_bounds__(BLK) void k_gu_relax(DG g, int pos) {
    const int prev = pos ? g.ctl->gu_changed[pos - 1] : g.ctl->gu_prev;
    if (!prev) return;
    const long long eps = g.ctl->eps;
    const long long* P = g.p0;
    int changed = 0;
    long long scans = 0;
    int b = blockIdx.x;
    if (b < g.nhitems) {
        __shared__ long long sh[WPB];
        const HItem it = g.hitems[b];
        const long long pu = P[it.node];
        long long best = INF64;
        for (int k = 0; k < PER_T; ++k) {
            const int a = it.begin + threadIdx.x * PER_T + k;
            if (a < it.end) {
                best = min(best, relax_arc(g, a, pu, P, eps));
                scans++;
            }
        }
        best = block_min(best, sh);
        if (threadIdx.x == 0 && best < INF64) {
            const long long old = atom_min_ret(&g.dist[it.node], best);
            if (best < old) changed = 1;
        }
    } else {
        b -= g.nhitems;
        if (b < g.nmblocks) {
            const int wi = b * WPB + (threadIdx.x >> 6);
            if (wi < g.nmedium) {
                const int u = g.medium[wi];
                const long long du = g.dist[u];
                if (du > 0) {
                    const long long pu = P[u];
                    long long best = INF64;
                    const int e = g.first[u + 1];
                    for (int a = g.first[u] + lane_id(); a < e; a += WAVE) {
                        best = min(best, relax_arc(g, a, pu, P, eps));
                        scans++;
                    }
                    best = wave_min(best);
                    if (best < du) {
                        if (lane_id() == 0) g.dist[u] = best;
                        changed = 1;
                    }
                }
            }
        } else {
            b -= g.nmblocks;
            const int i = b * BLK + threadIdx.x;
            if (i < g.nlight) {
                const int u = g.light[i];
                const long long du = g.dist[u];
                if (du > 0) {
                    const long long pu = P[u];
                    long long best = INF64;
                    const int e = g.first[u + 1];
                    for (int a = g.first[u]; a < e; ++a) best = min(best, relax_arc(g, a, pu, P, eps));
                    scans += e - g.first[u];
                    if (best < du) {
                        g.dist[u] = best;
                        changed = 1;
                    }
                }
            }
        }
    }
    if (__any(changed) && lane_id() == 0) g.ctl->gu_changed[pos] = 1;
    scans = wave_sum(scans);
    if (lane_id() == 0 && scans) {
        const int sh = ((blockIdx.x * WPB) + (threadIdx.x >> 6)) & (CTR_SHARDS - 1);
        atomicAdd(g.ctr + sh * NCTR + C_GUSCAN, (unsigned long long)scans);
    }
}

// per-block max of finite distances
__global__ void k_gu_maxd(DG g, long long* __restrict__ part) {
    __shared__ long long sh[WPB];
    long long mx = 0;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = g.dist[v];
        if (d < INF64) mx = max(mx, d);
    }
    mx = wave_max(mx);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) sh[w] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int i = 0; i < WPB; ++i) t = max(t, sh[i]);
        part[blockIdx.x] = t;
    }
}

__global__ void k_gu_apply(DG g, const long long* __restrict__ part, int nparts) {
    __shared__ long long s_dt;
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int i = 0; i < nparts; ++i) t = max(t, part[i]);
        const long long eps = g.ctl->eps;
        const long long lim = (1LL << 60) / eps;
        s_dt = t < lim ? t : lim;
    }
    __syncthreads();
    const long long dt = s_dt;
    const long long eps = g.ctl->eps;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK) {
        const long long d = g.dist[v];
        if (d >= INF64 && g.excess[v] > 0) g.ctl->infeasible = 1;
        const long long dd = d < dt ? d : dt;
        const long long np = g.p0[v] - eps * dd;
        g.p0[v] = np;
        g.p1[v] = np;
    }
}

// ================================================================ verify ===
// Conservation, capacity and 1-optimality (scaled units); per-block cost sums.
__global__ void k_verify_arcs(DG g, const int* __restrict__ fwd, const long long* __restrict__ low,
                              const long long* __restrict__ cap, const long long* __restrict__ cost,
                              long long* __restrict__ flows, long long* __restrict__ part) {
    __shared__ long long sh[WPB];
    long long csum = 0;
    int bad = 0;
    for (long long i = blockIdx.x * (long long)BLK + threadIdx.x; i < g.m; i += (long long)gridDim.x * BLK) {
        const int p = fwd[i];
        const long long cp = cap[i] - low[i];
        const long long rf = g.rcap[p], rr = g.rcap[g.rev[p]];
        const long long f = cp - rf;
        if (rf < 0 || rr < 0 || f < 0 || f != rr) bad = 1;
        const long long fl = f + low[i];
        flows[i] = fl;
        csum += fl * cost[i];
    }
    csum = wave_sum(csum);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) sh[w] = csum;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int i = 0; i < WPB; ++i) t += sh[i];
        part[blockIdx.x] = t;
    }
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 1);
}

__global__ void k_verify_opt(DG g, long long m2) {
    int bad = 0;
    const long long eps = g.ctl->eps;
    for (long long p = blockIdx.x * (long long)BLK + threadIdx.x; p < m2; p += (long long)gridDim.x * BLK) {
        if (g.rcap[p] > 0) {
            const int t = g.head[g.rev[p]];
            const long long cr = g.cost[p] + g.p0[t] - g.p0[g.head[p]];
            if (cr < -eps) bad = 1;
        }
    }
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 2);
}

__global__ void k_verify_nodes(DG g) {
    int bad = 0;
    for (long long v = blockIdx.x * (long long)BLK + threadIdx.x; v < g.n; v += (long long)gridDim.x * BLK)
        if (g.excess[v] != 0) bad = 1;
    if (__any(bad) && lane_id() == 0) atomicOr(&g.ctl->verify_bad, 4);
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
    hipEvent_t kev[4] = {};   // kernel-batch timing (sweeps, relaxations)

    // input (compacted) graph
    int64_t n = 0, m = 0;
    int64_t maxc = 0;
    DBuf<int> a_src, a_dst;
    DBuf<long long> a_low, a_cap, a_cost, supply;

    // residual CSR and node state
    DBuf<unsigned> keys_in, keys_out;
    DBuf<int> vals_in, vals_out, pos_of;
    DBuf<unsigned char> sort_tmp;
    DBuf<int> first, head, rev, fwd;
    DBuf<long long> rcap, scost, excess, p0, p1, dist;
    DBuf<unsigned char> cls;
    DBuf<int> hidx, light, medium, heavy, nsel;
    DBuf<unsigned char> sel_tmp;
    DBuf<HItem> hitems;
    DBuf<int> hnchunks, harrive, hunsat;
    DBuf<long long> hmin, inbox, part, flows;
    DBuf<unsigned long long> ctr;
    DBuf<unsigned> trace;
    DBuf<Ctl> ctl;
    Ctl* h_ctl = nullptr;       // pinned host mirror
    long long* h_scr = nullptr; // pinned scratch: [0] eps, [1] constant 1
    int nlight = 0, nmedium = 0, nheavy = 0, nhitems = 0;
    bool solved = false;

    ~EngineImpl() {
        if (stream) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(stream);
        }
        a_src.release(); a_dst.release(); a_low.release(); a_cap.release(); a_cost.release(); supply.release();
        keys_in.release(); keys_out.release(); vals_in.release(); vals_out.release(); pos_of.release();
        sort_tmp.release(); first.release(); head.release(); rev.release(); fwd.release();
        rcap.release(); scost.release(); excess.release(); p0.release(); p1.release(); dist.release();
        cls.release(); hidx.release(); light.release(); medium.release(); heavy.release(); nsel.release();
        sel_tmp.release(); hitems.release(); hnchunks.release(); harrive.release(); hunsat.release();
        hmin.release(); inbox.release(); part.release(); flows.release(); ctr.release(); trace.release(); ctl.release();
        if (h_ctl) (void)hipHostFree(h_ctl);
        if (h_scr) (void)hipHostFree(h_scr);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : kev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }

    DG dg() const {
        DG g{};
        g.n = (int)n;
        g.m = (int)m;
        g.first = first.p;
        g.head = head.p;
        g.rev = rev.p;
        g.rcap = rcap.p;
        g.cost = scost.p;
        g.excess = excess.p;
        g.p0 = p0.p;
        g.p1 = p1.p;
        g.hidx = hidx.p;
        g.inbox = inbox.p;
        g.light = light.p;
        g.nlight = nlight;
        g.medium = medium.p;
        g.nmedium = nmedium;
        g.hitems = hitems.p;
        g.nhitems = nhitems;
        g.nheavy = nheavy;
        g.hnode = heavy.p;
        g.hnchunks = hnchunks.p;
        g.harrive = harrive.p;
        g.hmin = hmin.p;
        g.hunsat = hunsat.p;
        g.dist = dist.p;
        g.ctl = ctl.p;
        g.ctr = ctr.p;
        g.trace = trace.n ? trace.p : nullptr;
        g.nmblocks = (nmedium + WPB - 1) / WPB;
        return g;
    }
    int sweep_grid() const {
        return std::max(1, nhitems + (nmedium + WPB - 1) / WPB + (nlight + BLK - 1) / BLK);
    }
};

#define KS_CHECK(expr)                                                   \
    do {                                                                 \
        hipError_t _e = (expr);                                          \
        if (_e != hipSuccess) {                                          \
            err = std::string(#expr) + ": " + hipGetErrorString(_e);     \
            return KS_E_DEVICE;                                          \
        }                                                                \
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
    for (auto& e : s.ev) KS_CHECK(hipEventCreate(&e));
    for (auto& e : s.kev) KS_CHECK(hipEventCreate(&e));
    KS_CHECK(s.ctl.ensure(1));
    KS_CHECK(s.ctr.ensure(CTR_SHARDS * NCTR));
    KS_CHECK(hipHostMalloc(&s.h_ctl, sizeof(Ctl)));
    KS_CHECK(hipHostMalloc(&s.h_scr, 4 * sizeof(long long)));
    s.h_scr[1] = 1;
    return KS_OK;
}

int Engine::upload(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int64_t* low,
                   const int64_t* cap, const int64_t* cost, const int64_t* supply, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    if (n < 0 || m < 0 || n > (1LL << 30) || m > (1LL << 29)) {
        err = "graph too large for 32-bit CSR indices";
        return KS_E_RANGE;
    }
    s.n = n;
    s.m = m;
    s.solved = false;
    s.maxc = 0;
    for (int64_t i = 0; i < m; ++i) s.maxc = std::max<int64_t>(s.maxc, cost[i] < 0 ? -cost[i] : cost[i]);
    KS_CHECK(s.a_src.ensure(m));
    KS_CHECK(s.a_dst.ensure(m));
    KS_CHECK(s.a_low.ensure(m));
    KS_CHECK(s.a_cap.ensure(m));
    KS_CHECK(s.a_cost.ensure(m));
    KS_CHECK(s.supply.ensure(n));
    if (m) {
        KS_CHECK(hipMemcpyAsync(s.a_src.p, src, m * sizeof(int), hipMemcpyHostToDevice, s.stream));
        KS_CHECK(hipMemcpyAsync(s.a_dst.p, dst, m * sizeof(int), hipMemcpyHostToDevice, s.stream));
        KS_CHECK(hipMemcpyAsync(s.a_low.p, low, m * sizeof(long long), hipMemcpyHostToDevice, s.stream));
        KS_CHECK(hipMemcpyAsync(s.a_cap.p, cap, m * sizeof(long long), hipMemcpyHostToDevice, s.stream));
        KS_CHECK(hipMemcpyAsync(s.a_cost.p, cost, m * sizeof(long long), hipMemcpyHostToDevice, s.stream));
    }
    if (n) KS_CHECK(hipMemcpyAsync(s.supply.p, supply, n * sizeof(long long), hipMemcpyHostToDevice, s.stream));
    KS_CHECK(hipStreamSynchronize(s.stream));
    return KS_OK;
}

int Engine::copy_to_device(void* dev_dst, const void* host_src, size_t bytes, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    if (bytes) {
        KS_CHECK(hipMemcpyAsync(dev_dst, host_src, bytes, hipMemcpyHostToDevice, s.stream));
        KS_CHECK(hipStreamSynchronize(s.stream));
    }
    return KS_OK;
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
    return ms;
}

int Engine::solve(ks_result& res, std::string& err) {
    EngineImpl& s = *p_;
    KS_CHECK(hipSetDevice(s.device));
    const auto t_host0 = std::chrono::steady_clock::now();
    hipStream_t st = s.stream;
    const int64_t n = s.n, m = s.m, m2 = 2 * m;
    s.solved = false;
    res.n_nodes = n;
    res.n_arcs = m;
    if (n == 0) {
        res.total_cost = 0;
        res.flow_value = 0;
        s.solved = true;
        return KS_OK;
    }
    const long long mult = n + 1;
    if (s.maxc > 0 && (double)s.maxc * (double)mult * 8.0 * (double)(n + 1) > 4.0e18) {
        err = "cost range too large for int64 scaled prices";
        return KS_E_RANGE;
    }

    // ------------------------------------------------------------ build ---
    KS_CHECK(hipEventRecord(s.ev[0], st));
    KS_CHECK(s.keys_in.ensure(m2));
    KS_CHECK(s.keys_out.ensure(m2));
    KS_CHECK(s.vals_in.ensure(m2));
    KS_CHECK(s.vals_out.ensure(m2));
    KS_CHECK(s.pos_of.ensure(m2));
    KS_CHECK(s.first.ensure(n + 1));
    KS_CHECK(s.head.ensure(m2));
    KS_CHECK(s.rev.ensure(m2));
    KS_CHECK(s.fwd.ensure(m));
    KS_CHECK(s.rcap.ensure(m2));
    KS_CHECK(s.scost.ensure(m2));
    KS_CHECK(s.excess.ensure(n));
    KS_CHECK(s.p0.ensure(n));
    KS_CHECK(s.p1.ensure(n));
    KS_CHECK(s.dist.ensure(n));
    KS_CHECK(s.cls.ensure(n));
    KS_CHECK(s.hidx.ensure(n));
    KS_CHECK(s.light.ensure(n));
    KS_CHECK(s.medium.ensure(n));
    KS_CHECK(s.heavy.ensure(n));
    KS_CHECK(s.nsel.ensure(4));
    KS_CHECK(s.flows.ensure(m));
    KS_CHECK(s.part.ensure(4096));
    KS_CHECK(hipMemsetAsync(s.ctr.p, 0, CTR_SHARDS * NCTR * sizeof(unsigned long long), st));
    KS_CHECK(hipMemsetAsync(s.ctl.p, 0, sizeof(Ctl), st));
    const char* trace_path = std::getenv("KS_TRACE");
    if (trace_path && *trace_path) {
        KS_CHECK(s.trace.ensure(4 * kTraceMax));
        KS_CHECK(hipMemsetAsync(s.trace.p, 0, 4 * kTraceMax * sizeof(unsigned), st));
    }
    struct PhaseRec {
        long long eps;
        uint64_t begin, end;
        std::vector<uint64_t> gu_at;
    };
    std::vector<PhaseRec> ptrace;

    if (m) {
        hipLaunchKernelGGL(k_make_keys, dim3(grid_for(m)), dim3(BLK), 0, st, (int)m, s.a_src.p, s.a_dst.p,
                           s.keys_in.p, s.vals_in.p);
        int bits = 1;
        while ((1LL << bits) <= n) ++bits;
        size_t tmp = 0;
        KS_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, s.keys_in.p, s.keys_out.p, s.vals_in.p,
                                                    s.vals_out.p, (int)m2, 0, bits, st));
        KS_CHECK(s.sort_tmp.ensure(tmp));
        KS_CHECK(hipcub::DeviceRadixSort::SortPairs(s.sort_tmp.p, tmp, s.keys_in.p, s.keys_out.p, s.vals_in.p,
                                                    s.vals_out.p, (int)m2, 0, bits, st));
        hipLaunchKernelGGL(k_scatter_pos, dim3(grid_for(m2)), dim3(BLK), 0, st, (long long)m2, s.vals_out.p,
                           s.pos_of.p);
        hipLaunchKernelGGL(k_fill, dim3(grid_for(m2)), dim3(BLK), 0, st, (long long)m2, mult, s.vals_out.p,
                           s.pos_of.p, s.a_src.p, s.a_dst.p, s.a_low.p, s.a_cap.p, s.a_cost.p, s.head.p, s.rev.p,
                           s.rcap.p, s.scost.p, s.fwd.p);
    }
    hipLaunchKernelGGL(k_first, dim3(grid_for(n + 1)), dim3(BLK), 0, st, (int)n, (long long)m2, s.keys_out.p,
                       s.first.p);
    hipLaunchKernelGGL(k_node_init, dim3(grid_for(n)), dim3(BLK), 0, st, (int)n, s.supply.p, s.first.p,
                       s.excess.p, s.p0.p, s.p1.p, s.cls.p, s.hidx.p);
    if (m)
        hipLaunchKernelGGL(k_lower_bounds, dim3(grid_for(m)), dim3(BLK), 0, st, (int)m, s.a_src.p, s.a_dst.p,
                           s.a_low.p, s.excess.p);
    {
        hipcub::CountingInputIterator<int> it(0);
        size_t tmp = 0, t2 = 0;
        for (unsigned char c = 0; c < 3; ++c) {
            KS_CHECK(hipcub::DeviceSelect::If(nullptr, t2, it, s.light.p, s.nsel.p + c, (int)n,
                                              ClassIs{s.cls.p, c}, st));
            tmp = std::max(tmp, t2);
        }
        KS_CHECK(s.sel_tmp.ensure(tmp));
        int* outs[3] = {s.light.p, s.medium.p, s.heavy.p};
        for (unsigned char c = 0; c < 3; ++c) {
            t2 = tmp;
            KS_CHECK(hipcub::DeviceSelect::If(s.sel_tmp.p, t2, it, outs[c], s.nsel.p + c, (int)n,
                                              ClassIs{s.cls.p, c}, st));
        }
    }
    int counts[4] = {0, 0, 0, 0};
    KS_CHECK(hipMemcpyAsync(counts, s.nsel.p, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    s.nlight = counts[0];
    s.nmedium = counts[1];
    s.nheavy = counts[2];
    {
        // heavy hubs: chunk table (few hubs; built on host from their CSR ranges)
        std::vector<int> hn(s.nheavy), hf(2 * s.nheavy);
        if (s.nheavy) {
            KS_CHECK(hipMemcpyAsync(hn.data(), s.heavy.p, s.nheavy * sizeof(int), hipMemcpyDeviceToHost, st));
            KS_CHECK(hipStreamSynchronize(st));
            for (int h = 0; h < s.nheavy; ++h) {
                KS_CHECK(hipMemcpyAsync(&hf[2 * h], s.first.p + hn[h], 2 * sizeof(int), hipMemcpyDeviceToHost, st));
            }
            KS_CHECK(hipStreamSynchronize(st));
        }
        std::vector<HItem> items;
        std::vector<int> nch(s.nheavy);
        for (int h = 0; h < s.nheavy; ++h) {
            int c = 0;
            for (int b = hf[2 * h]; b < hf[2 * h + 1]; b += CHUNK, ++c)
                items.push_back(HItem{hn[h], h, b, std::min(b + CHUNK, hf[2 * h + 1])});
            nch[h] = c;
        }
        s.nhitems = (int)items.size();
        KS_CHECK(s.hitems.ensure(items.size()));
        KS_CHECK(s.hnchunks.ensure(s.nheavy));
        KS_CHECK(s.harrive.ensure(s.nheavy));
        KS_CHECK(s.hunsat.ensure(s.nheavy));
        KS_CHECK(s.hmin.ensure(s.nheavy));
        KS_CHECK(s.inbox.ensure((size_t)s.nheavy * SHARDS));
        if (s.nheavy) {
            std::vector<long long> hm(s.nheavy, INF64);
            KS_CHECK(hipMemcpyAsync(s.hitems.p, items.data(), items.size() * sizeof(HItem), hipMemcpyHostToDevice, st));
            KS_CHECK(hipMemcpyAsync(s.hnchunks.p, nch.data(), nch.size() * sizeof(int), hipMemcpyHostToDevice, st));
            KS_CHECK(hipMemcpyAsync(s.hmin.p, hm.data(), hm.size() * sizeof(long long), hipMemcpyHostToDevice, st));
            KS_CHECK(hipMemsetAsync(s.harrive.p, 0, s.nheavy * sizeof(int), st));
            KS_CHECK(hipMemsetAsync(s.hunsat.p, 0, s.nheavy * sizeof(int), st));
            KS_CHECK(hipMemsetAsync(s.inbox.p, 0, (size_t)s.nheavy * SHARDS * sizeof(long long), st));
            hipLaunchKernelGGL(k_set_hidx, dim3((s.nheavy + BLK - 1) / BLK), dim3(BLK), 0, st, s.nheavy, s.heavy.p,
                               s.hidx.p);
            KS_CHECK(hipStreamSynchronize(st));
        }
    }
    KS_CHECK(hipEventRecord(s.ev[1], st));

    // ------------------------------------------------------------ phases ---
    DG g = s.dg();
    const int sgrid = s.sweep_grid();
    const int K = std::max(2, std::min(MAXB, s.opts.sweeps_per_batch > 0 ? s.opts.sweeps_per_batch : 32)) & ~1;
    const int GK = 16;
    const int alpha = s.opts.alpha >= 2 ? s.opts.alpha : 16;
    const int gu_interval = s.opts.gu_interval > 0 ? s.opts.gu_interval : 48;
    const int ngrid = grid_for(n, 2048);
    long long eps = std::max<long long>(1, (long long)s.maxc * mult);
    uint64_t sweeps = 0, gus = 0, gu_iters = 0, sweep_launches = 0, gu_launches = 0;
    double ms_sweep_k = 0, ms_gu_k = 0;
    int phases = 0;
    double ms_sat = 0, ms_sweep = 0, ms_gu = 0;
    const int* one = reinterpret_cast<const int*>(&s.h_scr[1]);
    int status = KS_OK;

    auto read_ctl = [&]() -> hipError_t {
        hipError_t e = hipMemcpyAsync(s.h_ctl, s.ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) return e;
        return hipStreamSynchronize(st);
    };

    auto global_update = [&]() -> int {
        hipLaunchKernelGGL(k_drain_all, dim3((std::max(1, s.nheavy) + BLK - 1) / BLK), dim3(BLK), 0, st, g);
        hipLaunchKernelGGL(k_gu_init, dim3(ngrid), dim3(BLK), 0, st, g);
        for (int rounds = 0;; ++rounds) {
            KS_CHECK(hipMemsetAsync(s.ctl.p->gu_changed, 0, sizeof(int) * GK, st));
            KS_CHECK(hipMemcpyAsync(&s.ctl.p->gu_prev, one, sizeof(int), hipMemcpyHostToDevice, st));
            KS_CHECK(hipEventRecord(s.kev[0], st));
            for (int k = 0; k < GK; ++k) hipLaunchKernelGGL(k_gu_relax, dim3(sgrid), dim3(BLK), 0, st, g, k);
            KS_CHECK(hipEventRecord(s.kev[1], st));
            KS_CHECK(read_ctl());
            gu_launches += GK;
            ms_gu_k += ev_ms(s.kev[0], s.kev[1]);
            int it = 0;
            for (int k = 0; k < GK; ++k) it += s.h_ctl->gu_changed[k] ? 1 : 0;
            gu_iters += it;
            if (!s.h_ctl->gu_changed[GK - 1]) break;
            if (rounds > 1 + (int)(4 * n / GK) ||
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t_host0).count() >
                    kSolveWallLimitS) {
                err = "global price update did not converge";
                return KS_E_DEVICE;
            }
        }
        hipLaunchKernelGGL(k_gu_maxd, dim3(ngrid), dim3(BLK), 0, st, g, s.part.p);
        hipLaunchKernelGGL(k_gu_apply, dim3(ngrid), dim3(BLK), 0, st, g, (const long long*)s.part.p, ngrid);
        ++gus;
        return KS_OK;
    };

    do {
        eps = std::max<long long>(1, eps / alpha);
        ++phases;
        s.h_scr[0] = eps;
        KS_CHECK(hipMemcpyAsync(&s.ctl.p->eps, &s.h_scr[0], sizeof(long long), hipMemcpyHostToDevice, st));
        KS_CHECK(hipEventRecord(s.ev[2], st));
        hipLaunchKernelGGL(k_saturate, dim3(sgrid), dim3(BLK), 0, st, g);
        KS_CHECK(hipEventRecord(s.ev[3], st));
        ptrace.push_back(PhaseRec{eps, sweep_launches, 0, {}});
        int rc = global_update();
        if (rc) return rc;
        KS_CHECK(hipEventRecord(s.ev[4], st));
        uint64_t phase_sweeps = 0;
        int since_gu = 0;
        for (;;) {
            KS_CHECK(hipMemsetAsync(s.ctl.p->active, 0, sizeof(int) * K, st));
            KS_CHECK(hipMemcpyAsync(&s.ctl.p->active_prev, one, sizeof(int), hipMemcpyHostToDevice, st));
            KS_CHECK(hipEventRecord(s.kev[2], st));
            for (int k = 0; k < K; ++k) {
                const long long ti = (long long)sweep_launches + k;
                hipLaunchKernelGGL(k_sweep, dim3(sgrid), dim3(BLK), 0, st, g, k,
                                   (g.trace && ti < kTraceMax) ? (int)ti : -1);
            }
            KS_CHECK(hipEventRecord(s.kev[3], st));
            KS_CHECK(read_ctl());
            sweep_launches += K;
            ms_sweep_k += ev_ms(s.kev[2], s.kev[3]);
            if (s.h_ctl->infeasible) {
                status = KS_E_INFEASIBLE;
                break;
            }
            int did = 0;
            for (int k = 0; k < K; ++k) did += s.h_ctl->active[k] ? 1 : 0;
            phase_sweeps += did;
            if (!s.h_ctl->active[K - 1]) break;
            since_gu += K;
            if (since_gu >= gu_interval) {
                ptrace.back().gu_at.push_back(sweep_launches);
                KS_CHECK(hipEventRecord(s.ev[6], st));
                rc = global_update();
                if (rc) return rc;
                KS_CHECK(hipEventRecord(s.ev[7], st));
                KS_CHECK(hipEventSynchronize(s.ev[7]));
                ms_gu += ev_ms(s.ev[6], s.ev[7]);
                since_gu = 0;
                KS_CHECK(read_ctl());
                if (s.h_ctl->infeasible) {
                    status = KS_E_INFEASIBLE;
                    break;
                }
            }
            const double wall_s =
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t_host0).count();
            if (phase_sweeps > (uint64_t)(64 * (n + 64)) || wall_s > kSolveWallLimitS) {
                err = "push/relabel did not converge (sweeps " + std::to_string(phase_sweeps) + ", " +
                      std::to_string(wall_s) + " s)";
                return KS_E_DEVICE;
            }
        }
        KS_CHECK(hipEventRecord(s.ev[5], st));
        KS_CHECK(hipEventSynchronize(s.ev[5]));
        ptrace.back().end = sweep_launches;
        ms_sat += ev_ms(s.ev[2], s.ev[3]);
        ms_gu += ev_ms(s.ev[3], s.ev[4]);
        ms_sweep += ev_ms(s.ev[4], s.ev[5]);
        sweeps += phase_sweeps;
        if (status) break;
        if (s.h_ctl->infeasible) {
            status = KS_E_INFEASIBLE;
            break;
        }
    } while (eps > 1);

    if (status == KS_E_INFEASIBLE) {
        err = "infeasible: some supply cannot reach a demand node";
    }

    // ------------------------------------------------------------ verify ---
    KS_CHECK(hipEventRecord(s.ev[6], st));
    const int vgrid = grid_for(m, 2048);
    long long tot_cost = 0;
    if (status == KS_OK) {
        hipLaunchKernelGGL(k_drain_all, dim3((std::max(1, s.nheavy) + BLK - 1) / BLK), dim3(BLK), 0, st, g);
        if (m) {
            hipLaunchKernelGGL(k_verify_arcs, dim3(vgrid), dim3(BLK), 0, st, g, (const int*)s.fwd.p,
                               (const long long*)s.a_low.p, (const long long*)s.a_cap.p,
                               (const long long*)s.a_cost.p, s.flows.p, s.part.p);
            hipLaunchKernelGGL(k_verify_opt, dim3(grid_for(m2, 2048)), dim3(BLK), 0, st, g, (long long)m2);
        }
        hipLaunchKernelGGL(k_verify_nodes, dim3(ngrid), dim3(BLK), 0, st, g);
        std::vector<long long> parts(m ? vgrid : 0);
        if (m) KS_CHECK(hipMemcpyAsync(parts.data(), s.part.p, vgrid * sizeof(long long), hipMemcpyDeviceToHost, st));
        KS_CHECK(read_ctl());
        for (long long x : parts) tot_cost += x;
        if (s.h_ctl->verify_bad && s.opts.verify) {
            status = KS_E_VERIFY;
            err = std::string("on-device verification failed (") +
                  ((s.h_ctl->verify_bad & 1) ? "capacity " : "") + ((s.h_ctl->verify_bad & 2) ? "optimality " : "") +
                  ((s.h_ctl->verify_bad & 4) ? "conservation" : "") + ")";
        }
    }
    KS_CHECK(hipEventRecord(s.ev[7], st));
    unsigned long long hc[CTR_SHARDS * NCTR];
    KS_CHECK(hipMemcpyAsync(hc, s.ctr.p, sizeof(hc), hipMemcpyDeviceToHost, st));
    KS_CHECK(hipStreamSynchronize(st));
    unsigned long long tc[NCTR] = {0};
    for (int i = 0; i < CTR_SHARDS; ++i)
        for (int k = 0; k < NCTR; ++k) tc[k] += hc[i * NCTR + k];

    if (trace_path && *trace_path && s.trace.n) {
        const uint64_t nt = std::min<uint64_t>(sweep_launches, kTraceMax);
        std::vector<unsigned> ht(4 * nt);
        if (nt) KS_CHECK(hipMemcpy(ht.data(), s.trace.p, 4 * nt * sizeof(unsigned), hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(trace_path, "a")) {
            std::fprintf(f, "{\"n\": %lld, \"m\": %lld, \"phases\": [", (long long)n, (long long)m);
            for (size_t i = 0; i < ptrace.size(); ++i) {
                std::fprintf(f, "%s{\"eps\": %lld, \"begin\": %llu, \"end\": %llu, \"gu_at\": [", i ? ", " : "",
                             ptrace[i].eps, (unsigned long long)ptrace[i].begin, (unsigned long long)ptrace[i].end);
                for (size_t k = 0; k < ptrace[i].gu_at.size(); ++k)
                    std::fprintf(f, "%s%llu", k ? ", " : "", (unsigned long long)ptrace[i].gu_at[k]);
                std::fprintf(f, "]}");
            }
            std::fprintf(f, "], ");
            const char* names[4] = {"visits", "relabels", "medium", "heavy"};
            for (int k = 0; k < 4; ++k) {
                std::fprintf(f, "%s\"%s\": [", k ? "], " : "", names[k]);
                for (uint64_t i = 0; i < nt; ++i) std::fprintf(f, "%s%u", i ? ", " : "", ht[4 * i + k]);
            }
            std::fprintf(f, "]}\n");
            std::fclose(f);
        }
    }
    res.total_cost = tot_cost;
    res.phases = phases;
    res.sweeps = sweeps;
    res.arc_scans = tc[C_SCAN];
    res.node_visits = tc[C_VISIT];
    res.pushes = tc[C_PUSH];
    res.relabels = tc[C_RELABEL];
    res.global_updates = gus;
    res.gu_iterations = gu_iters;
    res.ms_phase[0] = ev_ms(s.ev[0], s.ev[1]);
    res.ms_phase[1] = ms_sat;
    res.ms_phase[2] = ms_sweep;
    res.ms_phase[3] = ms_gu;
    res.ms_phase[4] = ev_ms(s.ev[6], s.ev[7]);
    res.ms_phase[5] =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    res.gu_arc_scans = tc[C_GUSCAN];
    res.sweep_launches = sweep_launches;
    res.ms_sweep_kernels = ms_sweep_k;
    res.gu_launches = gu_launches;
    res.ms_gu_kernels = ms_gu_k;
    res.status = status;
    if (status == KS_OK) s.solved = true;
    return status;
}

int Engine::download_flows(int64_t* out, std::string& err) {
    EngineImpl& s = *p_;
    if (!s.solved) {
        err = "no successful solve";
        return KS_E_INVALID;
    }
    KS_CHECK(hipSetDevice(s.device));
    if (s.m) {
        KS_CHECK(hipMemcpyAsync(out, s.flows.p, s.m * sizeof(long long), hipMemcpyDeviceToHost, s.stream));
        KS_CHECK(hipStreamSynchronize(s.stream));
    }
    return KS_OK;
}

}  // namespace ks
