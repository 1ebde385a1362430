// ks_store.hip — on-device application of ksched's incremental change stream
// (the k_apply_deltas of SURVEY §7; ks_store.h has the data model).
//
// A stream of k records is applied by six short kernels, all O(k) except the
// liveness scan (O(arc slots), ≈ 10 µs at config 3):
//   1. k_mark_removed     per node edit: its last REMOVE position (n_lastrm)
//   2. k_hash_records     per arc record: find-or-insert its (src, dst) key with a
//                         CAS into the open-addressing index; atomicMax of the
//                         record position → the entry's LAST record
//   3. k_kill_scan        per live arc slot touching a removed node: its flow goes
//                         back to the endpoints' excess and its residual pair turns
//                         inert; the slot is freed unless a record after the removal
//                         re-creates the arc (then it is re-inserted in step 6)
//   4. k_node_edits       per node edit: liveness, type, supply (excess follows)
//   5. k_arc_deletes      per LAST record that deletes its arc (UPDATE 0/0) or that
//                         a later removal of an endpoint kills
//   6. k_arc_upserts      per LAST record that upserts: in-place edit of capacity,
//                         bounds and cost (flow clamped, excess adjusted), or a new
//                         arc inserted into free positions of both endpoints'
//                         segments (atomicAdd on the segment fill counters; a full
//                         segment raises ctl->overflow and the host rebuilds the CSR
//                         from the arc table)
// Superseded records (not the LAST for their key) do nothing: this is the
// reference's mergeChangesToSameArc / removeDuplicateChanges /
// purgeChangesBeforeNodeRemoval (graph_change_manager.go:220-279) done on device.
// Deletes free slots (step 5) strictly before upserts allocate them (step 6):
// the free-slot stack is never pushed and popped in the same kernel.
#include "ks_store.h"

namespace ks {
namespace {

constexpr int SBLK = 256;

__device__ __forceinline__ unsigned hslot(unsigned long long k, int mask) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return (unsigned)k & (unsigned)mask;
}

// Index of key k's entry, inserting it (value −1) when absent. −1 if the table is full.
__device__ int h_find_or_insert(const StoreDev& d, unsigned long long k) {
    unsigned i = hslot(k, d.hmask);
    for (int probe = 0; probe <= d.hmask; ++probe, i = (i + 1) & (unsigned)d.hmask) {
        unsigned long long cur = __hip_atomic_load(&d.hkey[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == k) return (int)i;
        if (cur == HKEY_EMPTY) {
            const unsigned long long was = atomicCAS(&d.hkey[i], HKEY_EMPTY, k);
            if (was == HKEY_EMPTY || was == k) return (int)i;
        }
    }
    return -1;
}

__device__ int h_find(const StoreDev& d, unsigned long long k) {
    unsigned i = hslot(k, d.hmask);
    for (int probe = 0; probe <= d.hmask; ++probe, i = (i + 1) & (unsigned)d.hmask) {
        const unsigned long long cur = d.hkey[i];
        if (cur == k) return (int)i;
        if (cur == HKEY_EMPTY) return -1;
    }
    return -1;
}

// Wave-aggregated counter updates and slot allocation. A round's delta stream
// deletes and inserts tens of thousands of arcs (config 4: ~25k of each), and
// one atomic per record on the same control word serialises at the memory-side
// atomic unit (~10 ns each: k_arc_deletes took ~0.8 ms per config-4 round). The
// lanes of a wave that are active at the call combine into one atomic.
__device__ __forceinline__ void wave_count(int* ctr, bool pred, int sign = 1) {
    const unsigned long long m = __ballot(pred);
    if (m && (int)__lane_id() == __ffsll((long long)m) - 1) atomicAdd(ctr, sign * __popcll(m));
}
// pred lanes take consecutive values base, base + 1, … of *top (one atomicAdd of the count)
__device__ __forceinline__ int wave_take(int* top, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (!m) return -1;
    const int lead = __ffsll((long long)m) - 1;
    int base = 0;
    if ((int)__lane_id() == lead) base = atomicAdd(top, __popcll(m));
    base = __shfl(base, lead);
    return pred ? base + __popcll(m & ((1ULL << __lane_id()) - 1)) : -1;
}

__device__ __forceinline__ int h_tomb(const StoreDev& d, int e) {   // 1 when the entry became a tombstone
    if (e < 0) return 0;
    const unsigned long long was = atomicExch(&d.hkey[e], HKEY_TOMB);
    d.hval[e] = -1;
    return was != HKEY_TOMB;
}

__device__ __forceinline__ void inert(const StoreDev& d, int p, int owner) {
    d.ent[p] = -1;
    d.pos[p].rcap = 0;
    d.pos[p].ucap = 0;
    d.pos[p].cost = DEAD_COST;
    d.pos[p].head = owner;
    d.pos[p].rev = p;
}

__device__ __forceinline__ int perm_of(const StoreDev& d, int slot) { return slot < d.ncap ? d.perm[slot] : -1; }

// Return arc slot s's flow (and its lower bound) to its endpoints and make its
// residual pair inert. Only when the CSR is valid and the arc has positions.
__device__ void kill_positions(const StoreDev& d, int s) {
    if (!d.csr_valid) return;
    const int p = d.fwd[s];
    if (p < 0) return;
    d.fwd[s] = -1;
    const int q = d.pos[p].rev;
    const long long f = d.pos[q].rcap + d.a_low[s];
    const int xs = perm_of(d, d.a_src[s]), xd = perm_of(d, d.a_dst[s]);
    if (f) {
        atomicAdd((unsigned long long*)&d.excess[xs], (unsigned long long)f);
        atomicAdd((unsigned long long*)&d.excess[xd], (unsigned long long)(-f));
    }
    inert(d, p, xs);
    inert(d, q, xd);
}

// Free arc slot s on the lanes where fr is set (every active lane of the wave
// calls it: the stack slots and the counters are taken once per wave).
__device__ __forceinline__ void free_slots(const StoreDev& d, int s, bool fr) {
    if (fr) {
        d.a_alive[s] = 0;
        d.fwd[s] = -1;
    }
    const int t = wave_take(&d.ctl->free_top, fr);
    if (fr) d.free_stack[t] = s;
    wave_count(&d.ctl->live, fr, -1);
    wave_count(&d.ctl->killed, fr);
}

// A free (inert, ent = −1) position in node x's segment, claimed for the entry
// tag with a CAS on ent, or −1 when the segment has none. First the next never
// used position (the fill counter), then — once the segment has been filled —
// the positions that removed arcs left inert, found by scanning 64-position
// chunks from a per-node cursor (inserts and removals balance in a churning
// cell, so hubs such as the cluster aggregator and the sink keep their slack
// instead of forcing a CSR rebuild every few rounds).
// used[x]++ for every active lane, one atomic per distinct x in the wave: the
// lanes of one segment take consecutive values (new tasks' arcs into the cluster
// aggregator and their unscheduled aggregators meet in one wave). The leaders are
// found first and then add together, so the atomics' round trips overlap.
__device__ __forceinline__ int wave_fill(int* used, int x) {
    const int me = (int)__lane_id();
    unsigned long long rem = __ballot(1);
    int lead = me, rank = 0, cnt = 0;
    while (rem) {
        const int l = __ffsll((long long)rem) - 1;
        const int xl = __shfl(x, l);
        const unsigned long long same = __ballot(x == xl) & rem;
        if ((same >> me) & 1) {
            lead = l;
            rank = __popcll(same & ((1ULL << me) - 1));
        }
        if (me == l) cnt = __popcll(same);
        rem &= ~same;
    }
    int base = 0;
    if (me == lead) base = atomicAdd(&used[x], cnt);
    return __shfl(base, lead) + rank;
}

__device__ int claim_pos(const StoreDev& d, int x, int tag) {
    const int b = d.first[x], e = d.first[x + 1], cap = e - b;
    const int ps = wave_fill(d.used, x);
    if (ps < cap && atomicCAS(&d.ent[b + ps], -1, tag) == -1) return b + ps;
    constexpr int SCAN = 64;
    const int chunks = (cap + SCAN - 1) / SCAN;
    for (int k = 0; k < chunks && k < 64; ++k) {
        const int c = (int)((unsigned)atomicAdd(&d.scur[x], 1) % (unsigned)chunks);
        const int lo = b + c * SCAN, hi = min(e, lo + SCAN);
        for (int p = lo; p < hi; ++p)
            if (__hip_atomic_load(&d.ent[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1 &&
                atomicCAS(&d.ent[p], -1, tag) == -1)
                return p;
    }
    return -1;
}

__device__ __forceinline__ bool is_arc_record(const ks_delta& x) {
    return x.kind == KS_ADD_ARC || x.kind == KS_UPDATE_ARC;
}

// --------------------------------------------------------------- kernels ---
__global__ void k_reset_counters(StoreDev d) {
    if (threadIdx.x == 0) {
        d.ctl->killed = d.ctl->inserted = d.ctl->updated = d.ctl->superseded = 0;
    }
}

__global__ void k_mark_removed(StoreDev d, const NodeEdit* __restrict__ e, int ne, int value) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < ne; i += gridDim.x * SBLK)
        if (e[i].last_rm >= 0) d.n_lastrm[e[i].slot] = value ? e[i].last_rm : -1;
}

__global__ void k_hash_records(StoreDev d, const ks_delta* __restrict__ r, int k, int* __restrict__ rec_ent) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < k; i += gridDim.x * SBLK) {
        const ks_delta x = r[i];
        int e = -1;
        if (is_arc_record(x)) {
            e = h_find_or_insert(d, arc_hkey((long long)x.src, (long long)x.dst));
            if (e < 0) d.ctl->overflow |= 4;
            else atomicMax(&d.hlast[e], i);
        }
        rec_ent[i] = e;
    }
}

__global__ void k_kill_scan(StoreDev d, int hi) {
    for (int s = blockIdx.x * SBLK + threadIdx.x; s < hi; s += gridDim.x * SBLK) {
        bool fr = false;
        int e = -1;
        if (d.a_alive[s]) {
            const int lr = max(d.n_lastrm[d.a_src[s]], d.n_lastrm[d.a_dst[s]]);
            if (lr >= 0) {
                e = h_find(d, arc_hkey((long long)d.a_src[s] + 1, (long long)d.a_dst[s] + 1));
                const int last = e >= 0 ? d.hlast[e] : -1;
                kill_positions(d, s);
                fr = last < lr;   // no record after the removal re-creates it; else alive with
            }                     // fwd = −1, re-inserted by k_arc_upserts
        }
        free_slots(d, s, fr);
        wave_count(&d.ctl->tombs, fr && h_tomb(d, e));
    }
}

// The same per removed node, over its own CSR segment (when the CSR is valid every
// live arc has its two positions, and a removed node's arcs are in its segment):
// one thread per node edit, the wave's lanes stepping through their segments
// together (so the slot frees and counters of 64 nodes share each wave's atomics).
// An arc whose two endpoints are both removed is handled once, from its tail's
// segment. Config 4: ~5k removed tasks of a few positions each instead of a pass
// over every arc slot.
__device__ void kill_node_segment(const StoreDev& d, const NodeEdit* __restrict__ e, int ne, int i) {
    int b = 0, len = 0;
    if (i < ne) {
        const NodeEdit x = e[i];
        const int v = (x.last_rm >= 0 && x.was_alive) ? perm_of(d, x.slot) : -1;
        if (v >= 0) {
            b = d.first[v];
            len = d.first[v + 1] - b;
        }
    }
    int steps = len;
    for (int off = 32; off > 0; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
    for (int j = 0; j < steps; ++j) {
        bool fr = false;
        int h = -1, s = 0;
        const int t = j < len ? d.ent[b + j] : -1;
        if (t >= 0) {
            s = t >> 1;
            const int sl = d.a_src[s], dl = d.a_dst[s];
            const int lr = max(d.n_lastrm[sl], d.n_lastrm[dl]);
            // (t odd: this node is the head; the tail's thread handles the arc when the tail is removed too)
            if (d.a_alive[s] && lr >= 0 && (!(t & 1) || d.n_lastrm[sl] < 0)) {
                h = h_find(d, arc_hkey((long long)sl + 1, (long long)dl + 1));
                const int last = h >= 0 ? d.hlast[h] : -1;
                kill_positions(d, s);
                fr = last < lr;   // no record after the removal re-creates it
            }
        }
        free_slots(d, s, fr);
        wave_count(&d.ctl->tombs, fr && h_tomb(d, h));
    }
}

__global__ void k_kill_nodes(StoreDev d, const NodeEdit* __restrict__ e, int ne) {
    for (int i0 = blockIdx.x * SBLK; i0 < ne; i0 += gridDim.x * SBLK)   // (uniform per workgroup)
        kill_node_segment(d, e, ne, i0 + (int)threadIdx.x);
}

__global__ void k_reset_used(StoreDev d, const NodeEdit* __restrict__ e, int ne) {
    if (!d.csr_valid) return;
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < ne; i += gridDim.x * SBLK) {
        if (e[i].last_rm < 0 || !e[i].was_alive) continue;
        const int x = perm_of(d, e[i].slot);
        if (x >= 0) d.used[x] = 0;   // every incident arc is gone: the segment is free again
    }
}

__global__ void k_node_edits(StoreDev d, const NodeEdit* __restrict__ e, int ne) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < ne; i += gridDim.x * SBLK) {
        const NodeEdit x = e[i];
        const long long sup = x.alive ? x.supply : 0;
        const int p = perm_of(d, x.slot);
        if (x.alive && p < 0) d.ctl->overflow |= 2;   // a node id beyond the build
        if (d.csr_valid && p >= 0) {
            if (x.last_rm >= 0 || !x.was_alive) d.excess[p] = sup;
            else d.excess[p] += sup - d.n_supply[x.slot];
        }
        d.n_supply[x.slot] = sup;
        d.n_alive[x.slot] = x.alive;
        d.n_type[x.slot] = x.type;
        if (x.alive && (x.last_rm >= 0 || !x.was_alive)) d.n_fresh[x.slot] = 1;
        if (x.last_rm >= 0 || !x.alive) d.n_bind[x.slot] = 0;   // a removed task is unbound (scheduler.go:106-132)
    }
}

// Is record i (an arc record, the LAST for its key) killed by a later removal
// of one of its endpoints?
__device__ __forceinline__ bool killed_later(const StoreDev& d, const ks_delta& x, int i) {
    return d.n_lastrm[x.src - 1] > i || d.n_lastrm[x.dst - 1] > i;
}

__global__ void k_arc_deletes(StoreDev d, const ks_delta* __restrict__ r, int k, const int* __restrict__ rec_ent) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < k; i += gridDim.x * SBLK) {
        const int e = rec_ent[i];
        bool sup = false, fr = false, tomb = false;
        int s = -1;
        if (e >= 0) {
            sup = d.hlast[e] != i;
            if (!sup) {
                const ks_delta x = r[i];
                const bool del = x.kind == KS_UPDATE_ARC && x.low == 0 && x.cap == 0;
                if (del || killed_later(d, x, i)) {
                    s = d.hval[e];
                    fr = s >= 0 && d.a_alive[s];   // (a slot killed by k_kill_scan is already free)
                    if (fr) kill_positions(d, s);
                    tomb = h_tomb(d, e);
                }
            }
        }
        wave_count(&d.ctl->superseded, sup);
        free_slots(d, s, fr);
        wave_count(&d.ctl->tombs, tomb);
    }
}

// Record x applied to arc slot s: 1 edited in place, 2 inserted into the CSR, 0 otherwise.
__device__ int upsert_slot(const StoreDev& d, const ks_delta& x, int s) {
    const int sl = (int)x.src - 1, dl = (int)x.dst - 1;
    const long long low = (long long)x.low, cap = (long long)x.cap, u = cap - low;
    const long long low_old = d.a_low[s], cost_old = d.a_cost[s];
    d.a_src[s] = sl;
    d.a_dst[s] = dl;
    d.a_low[s] = low;
    d.a_cap[s] = cap;
    d.a_cost[s] = x.cost;
    d.a_type[s] = (unsigned char)(x.type < 0 ? 0 : (x.type > 255 ? 255 : x.type));
    if (!d.csr_valid) return 0;
    const int xs = perm_of(d, sl), xd = perm_of(d, dl);
    if (xs < 0 || xd < 0) {
        d.ctl->overflow |= 2;
        return 0;
    }
    const int p0 = d.fwd[s];
    if (p0 >= 0) {                  // in place: same endpoints, new bounds / cost
        const int q0 = d.pos[p0].rev;
        const long long f = d.pos[q0].rcap;
        const long long fn = f < 0 ? 0 : (f > u ? u : f);
        d.pos[p0].rcap = u - fn;
        d.pos[q0].rcap = fn;
        d.pos[p0].ucap = u;
        d.pos[q0].ucap = u;
        d.pos[p0].cost = x.cost * d.mult;
        d.pos[q0].cost = -x.cost * d.mult;
        const long long back = (f - fn) - (low - low_old);   // units returned to the tail
        if (back) {
            atomicAdd((unsigned long long*)&d.excess[xs], (unsigned long long)back);
            atomicAdd((unsigned long long*)&d.excess[xd], (unsigned long long)(-back));
        }
        // a cost rise on an arc that keeps its flow (ksched's ageing of the
        // arcs to the unscheduled aggregators, graph_manager.go:462-475): the
        // warm start lowers the tail's price by it, so the arc keeps its reduced
        // cost and only the tail's other arcs lose that much slack
        if (fn > 0 && x.cost > cost_old)
            atomicMax(&d.n_cshift[sl], (unsigned long long)(x.cost - cost_old));
        return 1;
    }
    // both endpoints claim (so a full segment is flagged at each end at once); a
    // claim that cannot be paired is given back
    const int p = claim_pos(d, xs, 2 * s), q = claim_pos(d, xd, 2 * s + 1);
    if (p < 0 || q < 0) {
        d.ctl->overflow |= 1;       // a full segment: the host rebuilds from the table
        if (p < 0) d.n_grow[sl] = 1;
        if (q < 0) d.n_grow[dl] = 1;
        if (p >= 0) atomicExch(&d.ent[p], -1);
        if (q >= 0) atomicExch(&d.ent[q], -1);
        return 0;
    }
    d.pos[p].head = xd;
    d.pos[p].rev = q;
    d.pos[p].rcap = u;
    d.pos[p].ucap = u;
    d.pos[p].cost = x.cost * d.mult;
    d.ent[p] = 2 * s;
    d.pos[q].head = xs;
    d.pos[q].rev = p;
    d.pos[q].rcap = 0;
    d.pos[q].ucap = u;
    d.pos[q].cost = -x.cost * d.mult;
    d.ent[q] = 2 * s + 1;
    d.fwd[s] = p;
    if (low) {                      // lower-bound transform
        atomicAdd((unsigned long long*)&d.excess[xs], (unsigned long long)(-low));
        atomicAdd((unsigned long long*)&d.excess[xd], (unsigned long long)low);
    }
    return 2;
}

__global__ void k_arc_upserts(StoreDev d, const ks_delta* __restrict__ r, int k, const int* __restrict__ rec_ent) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < k; i += gridDim.x * SBLK) {
        const int e = rec_ent[i];
        bool up = e >= 0 && d.hlast[e] == i;
        ks_delta x{};
        if (up) {
            x = r[i];
            up = !((x.kind == KS_UPDATE_ARC && x.low == 0 && x.cap == 0) || killed_later(d, x, i));
        }
        int s = up ? d.hval[e] : -1;
        // a new arc: a free slot, else a fresh one. The free-slot stack is popped and
        // fresh slots are handed out once per wave; the stack top may run below zero
        // (those lanes take fresh slots; k_finish resets it), as with one pop per lane.
        const bool fresh = up && s < 0;
        const unsigned long long fm = __ballot(fresh);
        if (fm) {
            const int lead = __ffsll((long long)fm) - 1;
            int top = 0;
            if ((int)__lane_id() == lead) top = atomicSub(&d.ctl->free_top, __popcll(fm));
            top = __shfl(top, lead);
            const int t = top - 1 - __popcll(fm & ((1ULL << __lane_id()) - 1));   // this lane's stack entry
            const int h = wave_take(&d.ctl->hi, fresh && t < 0);
            if (fresh) s = t >= 0 ? d.free_stack[t] : h;
        }
        int res = 0;
        if (fresh && s >= d.acap) {   // the host sizes the table first; never expected
            d.ctl->overflow |= 8;
            up = false;
        } else if (fresh) {
            d.hval[e] = s;
            d.a_alive[s] = 1;
            d.fwd[s] = -1;
        }
        if (up) res = upsert_slot(d, x, s);
        wave_count(&d.ctl->live, fresh && up);
        wave_count(&d.ctl->updated, res == 1);
        wave_count(&d.ctl->inserted, res == 2);
    }
}

__global__ void k_finish(StoreDev d, const int* __restrict__ rec_ent, int k) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i < k; i += gridDim.x * SBLK) {
        const int e = rec_ent[i];
        if (e >= 0) d.hlast[e] = -1;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && d.ctl->free_top < 0) d.ctl->free_top = 0;
}

__global__ void k_hash_clear(StoreDev d) {
    for (int i = blockIdx.x * SBLK + threadIdx.x; i <= d.hmask; i += gridDim.x * SBLK) {
        d.hkey[i] = HKEY_EMPTY;
        d.hval[i] = -1;
        d.hlast[i] = -1;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) d.ctl->tombs = 0;
}

__global__ void k_hash_fill(StoreDev d, int hi) {
    for (int s = blockIdx.x * SBLK + threadIdx.x; s < hi; s += gridDim.x * SBLK) {
        if (!d.a_alive[s]) continue;
        const int e = h_find_or_insert(d, arc_hkey((long long)d.a_src[s] + 1, (long long)d.a_dst[s] + 1));
        if (e < 0) d.ctl->overflow |= 4;
        else d.hval[e] = s;
    }
}

inline int grid(long long n) {
    long long b = (n + SBLK - 1) / SBLK;
    return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

hipError_t store_apply(const StoreDev& d, const ks_delta* recs, int k, int* rec_ent, const NodeEdit* edits, int ne,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_reset_counters, dim3(1), dim3(64), 0, st, d);
    if (ne) hipLaunchKernelGGL(k_mark_removed, dim3(grid(ne)), dim3(SBLK), 0, st, d, edits, ne, 1);
    if (k) hipLaunchKernelGGL(k_hash_records, dim3(grid(k)), dim3(SBLK), 0, st, d, recs, k, rec_ent);
    if (ne) {
        if (d.csr_valid)
            hipLaunchKernelGGL(k_kill_nodes, dim3(grid(ne)), dim3(SBLK), 0, st, d, edits, ne);
        else
            hipLaunchKernelGGL(k_kill_scan, dim3(grid(d.acap)), dim3(SBLK), 0, st, d, d.acap);
        hipLaunchKernelGGL(k_reset_used, dim3(grid(ne)), dim3(SBLK), 0, st, d, edits, ne);
        hipLaunchKernelGGL(k_node_edits, dim3(grid(ne)), dim3(SBLK), 0, st, d, edits, ne);
    }
    if (k) {
        hipLaunchKernelGGL(k_arc_deletes, dim3(grid(k)), dim3(SBLK), 0, st, d, recs, k, (const int*)rec_ent);
        hipLaunchKernelGGL(k_arc_upserts, dim3(grid(k)), dim3(SBLK), 0, st, d, recs, k, (const int*)rec_ent);
    }
    hipLaunchKernelGGL(k_finish, dim3(grid(k)), dim3(SBLK), 0, st, d, (const int*)rec_ent, k);
    if (ne) hipLaunchKernelGGL(k_mark_removed, dim3(grid(ne)), dim3(SBLK), 0, st, d, edits, ne, 0);
    return hipGetLastError();
}

hipError_t store_rehash(const StoreDev& d, hipStream_t st) {
    hipLaunchKernelGGL(k_hash_clear, dim3(grid((long long)d.hmask + 1)), dim3(SBLK), 0, st, d);
    hipLaunchKernelGGL(k_hash_fill, dim3(grid(d.acap)), dim3(SBLK), 0, st, d, d.acap);
    return hipGetLastError();
}

}  // namespace ks
