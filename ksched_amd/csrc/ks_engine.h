// ks_engine.h — device engine of libksmcmf (gfx950). Internal to the library:
// the public boundary is include/ksmcmf.h.
//
// The engine owns one solve's device state: the input arc arrays (uploaded by
// the host graph store), the residual CSR built from them on device, the
// node state (excess, double-buffered prices) and the control block the host
// polls between kernel batches. See DESIGN.md §3-§4 for the algorithm.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ksmcmf.h"

namespace ks {

struct EngineImpl;

class Engine {
public:
    Engine();
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    int init(int device, const ks_opts& opts, std::string& err);

    // Copy a compacted graph (0-based node slots) into device input arrays.
    // supply[n] is the node excess after any auto-sink adjustment. For a warm
    // start, prev_idx[m] gives each arc's index in the previous upload (−1 = new)
    // and fresh[n] marks node slots created since the previous solve; both may
    // be null (no warm start for this graph).
    int upload(int64_t n, int64_t m, const int32_t* src, const int32_t* dst,
               const int64_t* low, const int64_t* cap, const int64_t* cost,
               const int64_t* supply, const uint8_t* type, const int32_t* prev_idx,
               const uint8_t* fresh, std::string& err);

    // Build the residual CSR on device and run ε-scaling push-relabel to
    // optimality, then verify on device. Fills r (never NULL here).
    // warm: start from the previous solution when one maps onto this graph.
    int solve(ks_result& r, bool warm, std::string& err);

    // Flow on every input arc (input order) from the last successful solve.
    int download_flows(int64_t* flows, std::string& err);

    // Task → PU placement of the last solve, decomposed on device: for the i-th
    // task slot (DIMACS type 1) in slot order, the node id (slot + 1) of the last
    // PU its flow unit crosses, 0 when unscheduled. *count = number of tasks;
    // dev_out (device memory, ≥ count entries) may be null to query the count.
    int task_pu(uint64_t* dev_out, size_t cap, size_t* count, std::string& err);

    // Engine-owned device scratch of n uint64 (valid until the next call).
    int scratch(uint64_t** dev, size_t n, std::string& err);
    int download(void* host_dst, const void* dev_src, size_t bytes, std::string& err);


    int device() const;

private:
    EngineImpl* p_;
};

}  // namespace ks
