// ks_store.h — device-resident graph store of libksmcmf (internal).
//
// The flow graph lives in HBM between scheduling rounds: an arc table indexed by
// arc slot, an open-addressing (src, dst) → slot hash index, and the residual
// CSR the solver runs on, whose per-node segments carry slack so incremental
// deltas are applied IN PLACE (SURVEY §7 k_apply_deltas; the reference stream
// they replace is placement/solver.go:118-123 → dimacs/export.go:31-38). The
// host validates a delta stream against node liveness (flowgraph/graph.go
// semantics) and hands the device the raw records plus the final state of every
// node the stream touched; the device resolves the records in stream order:
//   last record per (src, dst) wins            (mergeChangesToSameArc)
//   records before a node's removal are dead   (purgeChangesBeforeNodeRemoval)
//   REMOVE_NODE drops every incident arc       (graph_change_manager.go:129-139)
// i.e. the change optimisers of graph_change_manager.go:220-279 run on the device
// as part of applying the stream.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ksmcmf.h"
#include "ks_pos.h"

namespace ks {

constexpr unsigned long long HKEY_EMPTY = 0ULL;
constexpr unsigned long long HKEY_TOMB = ~0ULL;
constexpr long long DEAD_COST = 1LL << 60;   // inert residual position: never admissible

// Final state of one node slot touched by a delta stream (computed on the host,
// which validates the stream sequentially against node liveness).
struct NodeEdit {
    int32_t slot;        // node id − 1
    int32_t last_rm;     // stream position of the node's last REMOVE_NODE, −1 = none
    int64_t supply;      // final supply (0 when not alive)
    uint8_t alive;       // final liveness
    uint8_t type;        // final DIMACS type
    uint8_t was_alive;   // alive before the stream
    uint8_t _pad[5];
};

// Device counters of the store (one per context).
struct StoreCtl {
    int free_top;        // entries on the free-slot stack
    int hi;              // arc slots handed out at least once: [0, hi)
    int live;            // live arc slots
    int tombs;           // hash tombstones
    int overflow;        // 1: a segment, the node map or the slot table ran out → rebuild
    int killed;          // arcs dropped by this apply
    int inserted;        // arcs inserted in place by this apply
    int updated;         // arcs edited in place by this apply
    int superseded;      // arc records superseded by a later record for the same arc
};

// Raw pointers of the store and of the residual CSR it maintains.
struct StoreDev {
    // node store, by slot (id − 1)
    int ncap;                     // slots covered by the build (perm valid below)
    long long* n_supply;
    unsigned char* n_type;
    unsigned char* n_alive;
    unsigned char* n_fresh;       // per slot: (re)created since the last solve (warm start)
    unsigned long long* n_cshift; // per slot: the largest cost increase on one of its flow-carrying
                                  // out-arcs since the last solve (warm start: its price drops by it)
    int* n_lastrm;                // per slot: last REMOVE position of the current apply, −1
    unsigned char* n_grow;        // per slot: an insert did not fit its segment (next build doubles it)
    unsigned long long* n_bind;   // per slot: bound PU node id (task bindings), 0 = none
    const int* perm;              // slot → internal id
    // arc table, by slot
    int acap;
    int* a_src;
    int* a_dst;
    long long* a_low;
    long long* a_cap;
    long long* a_cost;
    unsigned char* a_type;        // flowgraph.ArcType (1 = running)
    unsigned char* a_alive;
    int* fwd;                     // forward residual position, −1 = none
    int* free_stack;
    // hash index
    int hmask;                    // capacity − 1 (power of two)
    unsigned long long* hkey;
    int* hval;                    // arc slot, −1 = none yet
    int* hlast;                   // last record of the current apply, −1
    // residual CSR (internal ids)
    int nn;
    const int* first;             // segment starts, first[v + 1] − first[v] = capacity
    int* used;                    // positions handed out in each segment
    int* scur;                    // per node: chunk cursor of the inert-position scan
    Pos* pos;                     // residual positions (ks_pos.h)
    int* ent;                     // position → 2·slot + (reverse ? 1 : 0), −1 = dead
    long long* excess;
    long long mult;               // cost multiplier (node capacity + 1)
    int csr_valid;                // 0: table-only apply (a rebuild follows)
    StoreCtl* ctl;
};

__host__ __device__ inline unsigned long long arc_hkey(long long src_id, long long dst_id) {
    return ((unsigned long long)src_id << 32) | (unsigned long long)dst_id;
}

// Launchers (ks_store.hip). All run on `st` and return hipGetLastError().
// Apply k device-resident delta records (recs) and ne node edits; rec_ent is
// scratch of k ints. The StoreCtl counters killed..superseded are reset first.
hipError_t store_apply(const StoreDev& d, const ks_delta* recs, int k, int* rec_ent, const NodeEdit* edits,
                       int ne, hipStream_t st);
// Empty the hash index and re-insert every live arc slot (growth, tombstones).
hipError_t store_rehash(const StoreDev& d, hipStream_t st);

}  // namespace ks
