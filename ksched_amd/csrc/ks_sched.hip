// ks_sched.hip — the scheduler-side sweeps of a ksched round, on the
// device-resident graph (SURVEY §8 row f: the per-round O(T) CPU work that
// remains around Solve once the solve itself is fast):
//
//   scheduling deltas   NodeBindingToSchedulingDelta + SchedulingDeltasForPreemptedTasks
//                       (flowmanager/graph_manager.go:253-295, :297-339): the new
//                       task→PU mapping against the bindings kept per task slot →
//                       PREEMPT / PLACE / MIGRATE records; every destination must be
//                       a PU (:259-262)
//   topology statistics ComputeTopologyStatistics (graph_manager.go:480-511) with the
//                       trivial model's PrepareStats / GatherStats
//                       (costmodel/trivial_cost_modeler.go:147-176): BFS from the
//                       sink over in-arcs, level-synchronous
//   unscheduled costs   UpdateAllCostsToUnscheduledAggs (graph_manager.go:462-475):
//                       every task's arc into its unscheduled aggregator re-costed
//                       in place (residual pair included), running tasks' running
//                       arcs set to the continuation cost
#include "ks_sched.h"

namespace ks {
namespace {

constexpr int SB = 256;

inline int grid(long long n) {
    long long b = (n + SB - 1) / SB;
    return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

// ---------------------------------------------------------- scheduling deltas ---
// kind per task slot: 0 none, 1 + pb.SchedulingDelta type (PLACE 0, PREEMPT 1, MIGRATE 2)
__global__ void k_delta_kinds(int ncap, const int* __restrict__ is_task, const int* __restrict__ rank,
                              const unsigned long long* __restrict__ newpu, const unsigned long long* __restrict__ bind,
                              const unsigned char* __restrict__ type, long long nstore, int* __restrict__ pre,
                              int* __restrict__ other, int* __restrict__ bad) {
    for (long long v = blockIdx.x * (long long)SB + threadIdx.x; v < ncap; v += (long long)gridDim.x * SB) {
        int p = 0, o = 0;
        if (is_task[v]) {
            const unsigned long long nw = newpu[rank[v]], old = bind[v];
            if (nw && ((long long)nw > nstore || type[nw - 1] != KS_NODE_PU)) atomicOr(bad, 1);   // :259-262
            if (nw == 0 && old != 0) p = 1;                // PREEMPT: running, absent from the mapping
            else if (nw != 0 && old == 0) o = 1;           // PLACE
            else if (nw != 0 && old != nw) o = 2;          // MIGRATE
        }
        pre[v] = p;
        other[v] = o;
    }
}

// Records at their scanned positions: preemptions first (the reference emits them
// before the mapping's deltas, flowscheduler/scheduler.go:356-365), then
// placements and migrations, each in task-slot order.
__global__ void k_delta_emit(int ncap, const int* __restrict__ rank, const unsigned long long* __restrict__ newpu,
                             const unsigned long long* __restrict__ bind, const int* __restrict__ pre,
                             const int* __restrict__ pre_pos, const int* __restrict__ other,
                             const int* __restrict__ other_pos, int npre, ks_sched_delta* __restrict__ out,
                             unsigned long long* __restrict__ bind_out, int commit) {
    for (long long v = blockIdx.x * (long long)SB + threadIdx.x; v < ncap; v += (long long)gridDim.x * SB) {
        if (pre[v]) {
            ks_sched_delta d{KS_DELTA_PREEMPT, 0, (uint64_t)v + 1, bind[v]};
            out[pre_pos[v]] = d;
            if (commit) bind_out[v] = 0;
        } else if (other[v]) {
            const unsigned long long nw = newpu[rank[v]];
            ks_sched_delta d{other[v] == 1 ? KS_DELTA_PLACE : KS_DELTA_MIGRATE, 0, (uint64_t)v + 1, nw};
            out[npre + other_pos[v]] = d;
            if (commit) bind_out[v] = nw;
        }
    }
}

// ------------------------------------------------------- topology statistics ---
// Level-synchronous BFS from the sink over in-arcs. Every node first reached at
// level L + 1 is zeroed (PrepareStats; the arrays start at 0) and pushed; then
// each in-arc source gathers from the node being expanded: a PU from the sink
// takes (len(CurrentRunningTasks), maxTasksPerPu), any other accumulating node
// adds the expanded node's sums (GatherStats). Accumulating nodes: PUs,
// machines, intermediate resources, and type-0 nodes (the coordinator; ECs and
// aggregators only ever see non-resource sources and stay 0).
__device__ __forceinline__ bool accum(unsigned char t) {
    return t == KS_NODE_PU || t == KS_NODE_MACHINE || t == KS_NODE_INTERMEDIATE || t == KS_NODE_OTHER;
}

__global__ void k_topo_level(SchedDev d, const int* __restrict__ front, int nfront, int level, int* __restrict__ lvl,
                             int* __restrict__ next, int* __restrict__ nnext, unsigned long long mtpp,
                             const unsigned long long* __restrict__ pu_running, unsigned long long* __restrict__ slots,
                             unsigned long long* __restrict__ running) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * SB + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * SB) >> 6;
    for (int i = wave; i < nfront; i += nwaves) {
        const int x = front[i];                 // internal id
        const int v = d.iperm[x];               // its slot
        const unsigned char tx = d.n_type[v];
        const bool cur_sink = tx == KS_NODE_SINK;
        const bool cur_res = accum(tx);
        for (int p = d.first[x] + lane; p < d.first[x + 1]; p += 64) {
            const int e = d.ent[p];
            if (e < 0 || !(e & 1)) continue;    // live in-arcs only (reverse positions)
            const int u = d.pos[p].head;
            const int us = d.iperm[u];
            if (atomicCAS(&lvl[u], -1, level + 1) == -1) next[atomicAdd(nnext, 1)] = u;
            const unsigned char tu = d.n_type[us];
            if (!accum(tu)) continue;
            if (cur_sink) {
                if (tu == KS_NODE_PU) {
                    running[us] = pu_running[us];
                    slots[us] = mtpp;
                }
            } else if (cur_res) {
                atomicAdd(&running[us], running[v]);
                atomicAdd(&slots[us], slots[v]);
            }
        }
    }
}

// running arcs (type 1) into each PU slot: len(CurrentRunningTasks) by default
__global__ void k_running_into(int hi, const unsigned char* __restrict__ alive, const unsigned char* __restrict__ atype,
                               const int* __restrict__ dst, unsigned long long* __restrict__ cnt) {
    for (long long s = blockIdx.x * (long long)SB + threadIdx.x; s < hi; s += (long long)gridDim.x * SB)
        if (alive[s] && atype[s] == 1) atomicAdd(&cnt[dst[s]], 1ULL);
}

__global__ void k_scatter_running(int k, const unsigned long long* __restrict__ ids,
                                  const unsigned long long* __restrict__ vals, unsigned long long* __restrict__ cnt) {
    for (long long i = blockIdx.x * (long long)SB + threadIdx.x; i < k; i += (long long)gridDim.x * SB)
        cnt[ids[i] - 1] = vals[i];
}

// ----------------------------------------------------- unscheduled-arc costs ---
// flag bits per node slot: 1 unscheduled aggregator, 2 task with a running arc
// (type 1), 4 task with an arc into an unscheduled aggregator
__global__ void k_mark_unsched_auto(int hi, const unsigned char* __restrict__ alive, const int* __restrict__ src,
                                    const int* __restrict__ dst, const unsigned char* __restrict__ type,
                                    unsigned char* __restrict__ fl) {
    // type-0 nodes with an arc into a sink (graph_manager.go:1291-1305)
    for (long long s = blockIdx.x * (long long)SB + threadIdx.x; s < hi; s += (long long)gridDim.x * SB)
        if (alive[s] && type[dst[s]] == KS_NODE_SINK && type[src[s]] == KS_NODE_OTHER) fl[src[s]] = 1;
}

__global__ void k_mark_ids(int k, const unsigned long long* __restrict__ ids, unsigned char* __restrict__ fl) {
    for (long long i = blockIdx.x * (long long)SB + threadIdx.x; i < k; i += (long long)gridDim.x * SB)
        fl[ids[i] - 1] = 1;
}

__global__ void k_mark_tasks(SchedDev d, int hi, unsigned char* __restrict__ fl) {
    for (long long s = blockIdx.x * (long long)SB + threadIdx.x; s < hi; s += (long long)gridDim.x * SB) {
        if (!d.a_alive[s]) continue;
        const int t = d.a_src[s];
        if (d.n_type[t] != KS_NODE_TASK) continue;
        if (d.a_type[s] == 1) atomicOr((unsigned*)&fl[t & ~3], 2u << (8 * (t & 3)));
        if (fl[d.a_dst[s]] & 1) atomicOr((unsigned*)&fl[t & ~3], 4u << (8 * (t & 3)));
    }
}

__device__ __forceinline__ void set_cost(const SchedDev& d, int s, long long c, int* changed) {
    if (d.a_cost[s] == c) return;           // ChangeArcCost emits nothing then (graph_change_manager.go:171-182)
    d.a_cost[s] = c;
    const int p = d.fwd[s];
    if (d.csr_valid && p >= 0) {
        d.pos[p].cost = c * d.mult;
        d.pos[d.pos[p].rev].cost = -c * d.mult;
    }
    atomicAdd(changed, 1);
}

// For each U_j and each task t with an arc t→U_j (U_j's IncomingArcMap): a
// running t gets its running arc set to the continuation cost
// (updateRunningTaskNode, :1140-1158), any other t its t→U_j arc set to (SET) or
// raised by (ADD) the unscheduled cost (updateTaskToUnscheduledAggArc, :1270-1285).
__global__ void k_unsched_costs(SchedDev d, int hi, const unsigned char* __restrict__ fl, int mode, long long ucost,
                                long long ccost, int* __restrict__ changed) {
    for (long long s = blockIdx.x * (long long)SB + threadIdx.x; s < hi; s += (long long)gridDim.x * SB) {
        if (!d.a_alive[s]) continue;
        const int t = d.a_src[s];
        const unsigned char ft = fl[t];
        if (d.n_type[t] != KS_NODE_TASK || !(ft & 4)) continue;
        if (fl[d.a_dst[s]] & 1) {
            if (!(ft & 2)) set_cost(d, (int)s, mode == KS_COST_ADD ? d.a_cost[s] + ucost : ucost, changed);
        } else if (d.a_type[s] == 1) {
            set_cost(d, (int)s, ccost, changed);
        }
    }
}

}  // namespace

// ------------------------------------------------------------------ launchers ---
hipError_t sched_delta_kinds(const SchedDev& d, const int* is_task, const int* rank, const unsigned long long* newpu,
                             int* pre, int* other, int* bad, hipStream_t st) {
    hipLaunchKernelGGL(k_delta_kinds, dim3(grid(d.ncap)), dim3(SB), 0, st, d.ncap, is_task, rank, newpu,
                       (const unsigned long long*)d.n_bind, d.n_type, (long long)d.nstore, pre, other, bad);
    return hipGetLastError();
}

hipError_t sched_delta_emit(const SchedDev& d, const int* rank, const unsigned long long* newpu, const int* pre,
                            const int* pre_pos, const int* other, const int* other_pos, int npre, ks_sched_delta* out,
                            int commit, hipStream_t st) {
    hipLaunchKernelGGL(k_delta_emit, dim3(grid(d.ncap)), dim3(SB), 0, st, d.ncap, rank, newpu,
                       (const unsigned long long*)d.n_bind, pre, pre_pos, other, other_pos, npre, out, d.n_bind,
                       commit);
    return hipGetLastError();
}

hipError_t sched_running_counts(const SchedDev& d, const unsigned long long* ids, const unsigned long long* vals,
                                int k, unsigned long long* cnt, hipStream_t st) {
    if (ids) {
        if (k) hipLaunchKernelGGL(k_scatter_running, dim3(grid(k)), dim3(SB), 0, st, k, ids, vals, cnt);
    } else if (d.hi) {
        hipLaunchKernelGGL(k_running_into, dim3(grid(d.hi)), dim3(SB), 0, st, d.hi, d.a_alive, d.a_type, d.a_dst, cnt);
    }
    return hipGetLastError();
}

hipError_t sched_topo_level(const SchedDev& d, const int* front, int nfront, int level, int* lvl, int* next,
                            int* nnext, unsigned long long mtpp, const unsigned long long* pu_running,
                            unsigned long long* slots, unsigned long long* running, hipStream_t st) {
    const int blocks = std::max(1, std::min(4096, (nfront + 3) / 4));
    hipLaunchKernelGGL(k_topo_level, dim3(blocks), dim3(SB), 0, st, d, front, nfront, level, lvl, next, nnext, mtpp,
                       pu_running, slots, running);
    return hipGetLastError();
}

hipError_t sched_unsched_costs(const SchedDev& d, const unsigned long long* ids, int k, unsigned char* fl, int mode,
                               long long ucost, long long ccost, int* changed, hipStream_t st) {
    if (ids) {
        if (k) hipLaunchKernelGGL(k_mark_ids, dim3(grid(k)), dim3(SB), 0, st, k, ids, fl);
    } else if (d.hi) {
        hipLaunchKernelGGL(k_mark_unsched_auto, dim3(grid(d.hi)), dim3(SB), 0, st, d.hi, d.a_alive, d.a_src, d.a_dst,
                           d.n_type, fl);
    }
    if (d.hi) {
        hipLaunchKernelGGL(k_mark_tasks, dim3(grid(d.hi)), dim3(SB), 0, st, d, d.hi, fl);
        hipLaunchKernelGGL(k_unsched_costs, dim3(grid(d.hi)), dim3(SB), 0, st, d, d.hi, (const unsigned char*)fl, mode,
                           ucost, ccost, changed);
    }
    return hipGetLastError();
}

}  // namespace ks
