// ks_ctx.h — the C-ABI context (internal to libksmcmf): node-level host state
// plus the device engine that owns the graph. Shared by ks_host.cpp (the
// single-graph API) and ks_batch.hip (config 5, several devices).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ksmcmf.h"
#include "ks_engine.h"

struct NodeRec {   // one NodeID: supply, DIMACS type, liveness
    int64_t excess = 0;
    int32_t type = 0;
    bool alive = false;
    bool pad = false;
};

struct ks_ctx {
    ks::Engine eng;
    ks_opts opts{};

    std::string err;

    std::vector<NodeRec> nodes;            // index = NodeID (slot 0 unused)
    // per id, the stamps of the current apply in one record next to nothing else
    // (a stream's node records touch them at scattered ids)
    struct IdStamp {
        uint32_t epoch = 0;     // last apply that touched the id
        int32_t lastrm = -1;    // last REMOVE position in that apply
    };
    std::vector<IdStamp> ids;
    uint32_t epoch = 0;
    int64_t sum_others = 0;                // Σ supply of live non-sink nodes
    int64_t n_sinks = 0;
    uint64_t sink_id = 0;                  // the sink (when n_sinks == 1)
    int64_t n_tasks = 0;                   // live task nodes
    int64_t dev_sink_supply = 0;           // the sink's supply as the device has it
    bool have_solution = false;
    bool flows_fresh = false;
    bool map_fresh = false;                // map_dense holds the current solve's task→PU vector
    std::vector<uint64_t> map_dense;       // per live task slot in slot order: its PU (0: none)
    bool store_bad = false;                // a load / apply failed on the device: reload first
    std::vector<ks_flow> flows;

    int fail(int code, const std::string& msg) {
        err = msg;
        return code;
    }
    int64_t nslots() const { return (int64_t)nodes.size() - 1; }
};
