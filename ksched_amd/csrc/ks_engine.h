// ks_engine.h — device engine of libksmcmf (gfx950). Internal to the library:
// the public boundary is include/ksmcmf.h.
//
// The engine owns the device-resident graph (ks_store.h: node store, arc table,
// hash index, residual CSR with slack), the solver state (excess,
// double-buffered prices, frontiers) and the control block the host polls
// between kernel batches. See DESIGN.md §3-§4 for the algorithm.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ksmcmf.h"
#include "ks_store.h"

namespace ks {

struct EngineImpl;

class Engine {
public:
    Engine();
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    int init(int device, const ks_opts& opts, std::string& err);

    // Replace the device store: node slots [0, nslots) (slot = NodeID − 1) with
    // their supply, DIMACS type and liveness, and the arcs (1-based ids, already
    // validated; a repeated (src, dst) pair: the last one wins).
    int load(int64_t nslots, const int64_t* supply, const uint8_t* type, const uint8_t* alive, const ks_arc* arcs,
             size_t m, std::string& err);

    // Apply a validated delta stream on the device (ks_store.h): the final state
    // of every node it touches plus the raw records; nslots = node slots in use.
    int apply(const NodeEdit* edits, size_t ne, const ks_delta* recs, size_t k, int64_t nslots, std::string& err);

    // The graph is a disjoint union of independent cells: cell i owns the node ids
    // (off[i], off[i+1]] (k + 1 offsets; no arc may cross two cells). Cells the cell
    // solver holds are then solved one workgroup each in ONE launch (ks_cell.h);
    // k = 0 forgets the partition (the whole graph is one cell).
    void set_cells(const int64_t* off, size_t k);

    // Node state changes outside a stream (the auto-sink demand).
    int set_nodes(const NodeEdit* edits, size_t ne, std::string& err);

    // ε-scaling push-relabel to optimality on the device-resident graph, then
    // on-device verification. Fills r. warm: start from the flow and prices in
    // place (the previous solve's, edited by the deltas since).
    int solve(ks_result& r, bool warm, std::string& err);

    // Per-partition sums of the last solve for a disjoint union of graphs: graph i
    // owns node ids (off[i], off[i+1]]; cost[i] = Σ flow·cost over its arcs, flow[i] =
    // net inflow into its demand nodes. off has k+1 entries (host); outputs are
    // device pointers (k int64 each).
    int cell_sums(const int64_t* off, size_t k, int64_t* dev_cost, int64_t* dev_flow, std::string& err);
    hipStream_t stream() const;

    // Live arcs of the store (1-based ids), arc-slot order.
    int arcs(std::vector<ks_arc>& out, std::string& err);

    // Arcs with positive flow in the last solve (the "f" lines), arc-slot order.
    int flows(std::vector<ks_flow>& out, std::string& err);

    // Task → PU placement of the last solve, decomposed on device: for the i-th
    // live task slot in slot order, the node id of the last PU its flow unit
    // crosses, 0 when unscheduled. *count = n_tasks; dev_out (device memory,
    // ≥ n_tasks entries) may be null to query the count.
    int task_pu(uint64_t* dev_out, size_t cap, size_t* count, int64_t n_tasks, std::string& err);

    // Engine-owned device scratch of n uint64 (valid until the next call).
    int scratch(uint64_t** dev, size_t n, std::string& err);
    int download(void* host_dst, const void* dev_src, size_t bytes, std::string& err);

    int64_t live_arcs() const;
    bool solved() const;
    void store_stats(ks_store_stats* out) const;

    // Scheduler-side sweeps of a round (ks_sched.hip); see include/ksmcmf.h.
    int set_bindings(const uint64_t* task, const uint64_t* pu, size_t k, std::string& err);
    int sched_deltas(int commit, std::vector<ks_sched_delta>* out, size_t* count, int64_t n_tasks, std::string& err);
    int unsched_costs(const uint64_t* ids, size_t k, int mode, int64_t ucost, int64_t ccost, size_t* changed,
                      std::string& err);
    int topology_stats(uint64_t mtpp, const uint64_t* pu_ids, const uint64_t* pu_running, size_t k, int64_t sink_slot,
                       uint64_t* slots_below, uint64_t* running_below, std::string& err);
    int device() const;

private:
    EngineImpl* p_;
};

}  // namespace ks
