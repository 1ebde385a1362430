// ks_host.cpp — host runtime and C-ABI of libksmcmf (include/ksmcmf.h).
//
// Mirrors the reference's solver boundary, scheduling/flow/placement/solver.go:
//   ks_create         ↔ NewSolver (:49-55) + startSolver (:92-109)
//   ks_load_graph     ↔ writeGraph → dimacs.Export (:111-116, dimacs/export.go:11-29)
//   ks_apply_deltas   ↔ writeIncremental → dimacs.ExportIncremental (:118-123)
//   ks_solve          ↔ the Flowlessly solve
//   ks_get_flows      ↔ the "f" lines consumed by readFlowGraph (:134-179)
//   ks_get_task_mapping ↔ parseFlowToMapping (:183-269)
// The graph itself lives on the device (ks_store.h): arc table, (src, dst) hash
// index and residual CSR, edited in place by ks_apply_deltas. The host keeps only
// node-level state — liveness, supply, type per NodeID (flowgraph/graph.go:27-182
// semantics: ids index slots, REMOVE_NODE drops incident arcs, ids are reused) —
// which is all a stream needs to be validated in order, sequentially, before the
// device resolves it in parallel.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ksmcmf.h"
#include "ks_ctx.h"

namespace {




constexpr uint64_t kMaxId = (1ULL << 30);

inline uint64_t arc_key(uint64_t s, uint64_t d) { return (s << 32) | d; }

// (src, dst) → record index for ks_coalesce_deltas: open addressing with linear
// probing and backward-shift deletion (no tombstones), power-of-two capacity
// kept under 1/2 load. Keys are never 0 (node ids start at 1), so 0 marks an
// empty bucket.
class ArcIndex {
public:
    void clear() {
        keys_.assign(16, 0);
        vals_.assign(16, -1);
        size_ = 0;
    }
    void reserve(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 2) cap <<= 1;
        if (cap > keys_.size()) rehash(cap);
    }
    int find(uint64_t k) const {
        size_t i = slot(k);
        while (keys_[i]) {
            if (keys_[i] == k) return vals_[i];
            i = (i + 1) & mask();
        }
        return -1;
    }
    void insert(uint64_t k, int v) {   // k must be absent
        if (2 * (size_ + 1) > keys_.size()) rehash(keys_.size() * 2);
        size_t i = slot(k);
        while (keys_[i]) i = (i + 1) & mask();
        keys_[i] = k;
        vals_[i] = v;
        ++size_;
    }
    void erase(uint64_t k) {
        size_t i = slot(k);
        while (keys_[i] && keys_[i] != k) i = (i + 1) & mask();
        if (!keys_[i]) return;
        // backward shift: pull later members of the probe run into the hole
        size_t j = i;
        for (;;) {
            j = (j + 1) & mask();
            if (!keys_[j]) break;
            const size_t h = slot(keys_[j]);
            const bool between = (i <= j) ? (i < h && h <= j) : (i < h || h <= j);
            if (between) continue;
            keys_[i] = keys_[j];
            vals_[i] = vals_[j];
            i = j;
        }
        keys_[i] = 0;
        vals_[i] = -1;
        --size_;
    }

private:
    std::vector<uint64_t> keys_ = std::vector<uint64_t>(16, 0);
    std::vector<int> vals_ = std::vector<int>(16, -1);
    size_t size_ = 0;
    size_t mask() const { return keys_.size() - 1; }
    size_t slot(uint64_t k) const {
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdULL;
        k ^= k >> 33;
        return (size_t)k & mask();
    }
    void rehash(size_t cap) {
        std::vector<uint64_t> ok;
        std::vector<int> ov;
        ok.swap(keys_);
        ov.swap(vals_);
        keys_.assign(cap, 0);
        vals_.assign(cap, -1);
        size_ = 0;
        for (size_t i = 0; i < ok.size(); ++i)
            if (ok[i]) insert(ok[i], ov[i]);
    }
};

}  // namespace

namespace {

void ensure_node(ks_ctx* c, uint64_t id) {
    if (id >= c->nodes.size()) {
        c->nodes.resize(id + 1);
        c->ids.resize(id + 1);
    }
}

bool node_alive(const ks_ctx* c, uint64_t id) { return id < c->nodes.size() && c->nodes[id].alive; }

// Node-level aggregates (auto-sink demand, task count) follow every change.
void account(ks_ctx* c, uint64_t id, const NodeRec& r, int sign) {
    if (!r.alive) return;
    if (r.type == KS_NODE_SINK) {
        c->n_sinks += sign;
        if (sign > 0) c->sink_id = id;
    } else {
        c->sum_others += sign * r.excess;
    }
    if (r.type == KS_NODE_TASK) c->n_tasks += sign;
}

// Validate one arc against a node table (the context's, or a load's new one).
int check_arc(ks_ctx* c, const std::vector<NodeRec>& tab, uint64_t s, uint64_t d, uint64_t low, uint64_t cap,
              int64_t cost) {
    auto alive = [&](uint64_t id) { return id < tab.size() && tab[id].alive; };
    if (s == 0 || d == 0 || s >= kMaxId || d >= kMaxId) return c->fail(KS_E_RANGE, "arc endpoint id out of range");
    if (!alive(s) || !alive(d))
        return c->fail(KS_E_INVALID, "arc " + std::to_string(s) + "->" + std::to_string(d) + " has a missing endpoint");
    if (s == d) return c->fail(KS_E_INVALID, "self-loop arc at node " + std::to_string(s));
    if (low > (uint64_t)INT64_MAX || cap > (uint64_t)INT64_MAX) return c->fail(KS_E_RANGE, "arc bound exceeds int64");
    if (low > cap)
        return c->fail(KS_E_INVALID, "arc " + std::to_string(s) + "->" + std::to_string(d) + " has low > cap");
    if (cap > (uint64_t(1) << 53) || cost > (int64_t(1) << 40) || cost < -(int64_t(1) << 40))
        return c->fail(KS_E_RANGE, "arc capacity or cost outside the supported range");
    return KS_OK;
}
int check_arc(ks_ctx* c, uint64_t s, uint64_t d, uint64_t low, uint64_t cap, int64_t cost) {
    return check_arc(c, c->nodes, s, d, low, cap, cost);
}

// A device-side failure inside an apply or a load leaves the device store in an
// unknown state: every call that would read it refuses until the next load.
int store_guard(ks_ctx* c) {
    if (!c->store_bad) return KS_OK;
    return c->fail(KS_E_INVALID, "the device graph store is inconsistent after a failed load or apply: "
                                 "reload the graph (ks_load_graph)");
}

}  // namespace

extern "C" {

int ks_abi_version(void) { return KSMCMF_ABI_VERSION; }

void ks_default_opts(ks_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->alpha = 0;   // the library's size-dependent default (ks_engine.hip)
    o->verify = 1;
    o->auto_sink = 1;
    o->price_refine = 1;
    o->gu_interval = 24;   // 24 vs 32 on config 3: ≈ 2 ms lower median; config 5 ≈ 3 % faster (profiles/r01f_gu_interval.txt)
    o->warm_start = 0;
}

ks_ctx* ks_create(int device, const ks_opts* opts) {
    ks_ctx* c = new (std::nothrow) ks_ctx;
    if (!c) return nullptr;
    if (opts) c->opts = *opts;
    else ks_default_opts(&c->opts);
    std::string err;
    if (c->eng.init(device, c->opts, err) != KS_OK) {
        delete c;
        return nullptr;
    }
    c->nodes.resize(1);
    c->ids.resize(1);
    return c;
}

void ks_destroy(ks_ctx* c) { delete c; }

const char* ks_last_error(ks_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ks_load_graph(ks_ctx* c, const ks_node* nodes, size_t n, const ks_arc* arcs, size_t m) {
    if (!c) return KS_E_INVALID;
    if ((n && !nodes) || (m && !arcs)) return c->fail(KS_E_INVALID, "null input array");
    uint64_t maxid = 0;
    for (size_t i = 0; i < n; ++i) {
        if (nodes[i].id == 0 || nodes[i].id >= kMaxId)
            return c->fail(KS_E_RANGE, "node id " + std::to_string(nodes[i].id) + " out of range");
        maxid = std::max<uint64_t>(maxid, nodes[i].id);
    }
    std::vector<NodeRec> fresh(maxid + 1);
    for (size_t i = 0; i < n; ++i) {
        NodeRec& r = fresh[nodes[i].id];
        if (r.alive)   // graph.go:95-98
            return c->fail(KS_E_INVALID, "node " + std::to_string(nodes[i].id) + " already present");
        r = NodeRec{nodes[i].excess, nodes[i].type, true, true};
    }
    // every arc is checked against the new table BEFORE anything changes: a bad
    // arc leaves the context (host and device) exactly as it was
    for (size_t i = 0; i < m; ++i) {
        const ks_arc& a = arcs[i];
        int rc = check_arc(c, fresh, a.src, a.dst, a.low, a.cap, a.cost);
        if (rc) return rc;
    }
    c->nodes.swap(fresh);
    c->ids.assign(maxid + 1, ks_ctx::IdStamp{});
    c->sum_others = c->n_sinks = c->n_tasks = 0;
    c->sink_id = 0;
    for (uint64_t id = 1; id <= maxid; ++id) account(c, id, c->nodes[id], 1);
    c->have_solution = false;
    c->map_fresh = false;
    c->flows_fresh = false;
    std::vector<int64_t> supply(maxid);
    std::vector<uint8_t> type(maxid), alive(maxid);
    for (uint64_t id = 1; id <= maxid; ++id) {
        const NodeRec& r = c->nodes[id];
        supply[id - 1] = r.alive ? r.excess : 0;
        type[id - 1] = (uint8_t)std::min<int32_t>(std::max<int32_t>(r.type, 0), 255);
        alive[id - 1] = r.alive ? 1 : 0;
    }
    c->dev_sink_supply = (c->n_sinks == 1) ? c->nodes[c->sink_id].excess : 0;
    c->eng.set_cells(nullptr, 0);   // a plain load is one graph (ks_batch_load sets its cells after)
    const int rc = c->eng.load((int64_t)maxid, supply.data(), type.data(), alive.data(), arcs, m, c->err);
    c->store_bad = rc != KS_OK;   // the upload failed part-way: nothing may read the store
    return rc;
}

// Validate the stream in order against node liveness (graph.go / the change
// manager's preconditions), all or nothing: on an error the host state is rolled
// back and nothing reaches the device. The device then resolves the records.
int ks_apply_deltas(ks_ctx* c, const ks_delta* d, size_t k) {
    if (!c) return KS_E_INVALID;
    if (k && !d) return c->fail(KS_E_INVALID, "null delta array");
    if (k > (size_t)INT32_MAX) return c->fail(KS_E_RANGE, "delta stream too long");
    if (int g = store_guard(c)) return g;
    const auto t_in = std::chrono::steady_clock::now();
    if (++c->epoch == 0) {   // epoch wrapped: forget old stamps
        for (auto& st : c->ids) st.epoch = 0;
        c->epoch = 1;
    }
    std::vector<std::pair<uint64_t, NodeRec>> saved;   // first-touch state of every touched node
    auto touch = [&](uint64_t id) {
        ensure_node(c, id);
        if (c->ids[id].epoch != c->epoch) {
            c->ids[id].epoch = c->epoch;
            c->ids[id].lastrm = -1;
            saved.emplace_back(id, c->nodes[id]);
        }
    };
    int rc = KS_OK;
    for (size_t i = 0; i < k && rc == KS_OK; ++i) {
        const ks_delta& x = d[i];
        switch (x.kind) {
            case KS_ADD_NODE:
                if (x.id == 0 || x.id >= kMaxId) {
                    rc = c->fail(KS_E_RANGE, "node id " + std::to_string(x.id) + " out of range");
                    break;
                }
                if (node_alive(c, x.id)) {   // graph.go:95-98
                    rc = c->fail(KS_E_INVALID, "node " + std::to_string(x.id) + " already present");
                    break;
                }
                touch(x.id);
                c->nodes[x.id] = NodeRec{x.excess, x.type, true, true};
                break;
            case KS_REMOVE_NODE:
                if (!node_alive(c, x.id)) {
                    rc = c->fail(KS_E_INVALID, "remove of missing node " + std::to_string(x.id));
                    break;
                }
                touch(x.id);
                c->nodes[x.id] = NodeRec{};
                c->ids[x.id].lastrm = (int32_t)i;
                break;
            case KS_ADD_ARC:
                rc = check_arc(c, x.src, x.dst, x.low, x.cap, x.cost);
                break;
            case KS_UPDATE_ARC:
                if (x.low == 0 && x.cap == 0) {   // DeleteArc / ChangeArc(0,0): the arc goes
                    if (x.src == 0 || x.dst == 0 || x.src >= kMaxId || x.dst >= kMaxId)
                        rc = c->fail(KS_E_RANGE, "arc endpoint id out of range");
                    else if (!node_alive(c, x.src) || !node_alive(c, x.dst))
                        rc = c->fail(KS_E_INVALID, "update of arc with a missing endpoint");
                    break;
                }
                rc = check_arc(c, x.src, x.dst, x.low, x.cap, x.cost);
                break;
            case KS_SET_EXCESS:
                if (!node_alive(c, x.id)) {
                    rc = c->fail(KS_E_INVALID, "excess of missing node " + std::to_string(x.id));
                    break;
                }
                touch(x.id);
                c->nodes[x.id].excess = x.excess;
                break;
            default:
                rc = c->fail(KS_E_INVALID, "unknown delta kind " + std::to_string(x.kind));
        }
    }
    if (rc) {   // roll back: the stream is applied entirely or not at all
        for (auto it = saved.rbegin(); it != saved.rend(); ++it) c->nodes[it->first] = it->second;
        return rc;
    }
    std::vector<ks::NodeEdit> edits;
    edits.reserve(saved.size());
    const int64_t sum0 = c->sum_others, sinks0 = c->n_sinks, tasks0 = c->n_tasks, dsink0 = c->dev_sink_supply;
    const uint64_t sink0 = c->sink_id;
    for (const auto& sv : saved) {
        const uint64_t id = sv.first;
        const NodeRec& now = c->nodes[id];
        account(c, id, sv.second, -1);
        account(c, id, now, 1);
        ks::NodeEdit e;
        std::memset(&e, 0, sizeof(e));
        e.slot = (int32_t)(id - 1);
        e.last_rm = c->ids[id].lastrm;
        e.supply = now.alive ? now.excess : 0;
        e.alive = now.alive ? 1 : 0;
        e.type = (uint8_t)std::min<int32_t>(std::max<int32_t>(now.type, 0), 255);
        e.was_alive = sv.second.alive ? 1 : 0;
        edits.push_back(e);
        if (now.alive && now.type == KS_NODE_SINK) c->dev_sink_supply = now.excess;
    }
    c->have_solution = false;
    c->map_fresh = false;
    c->flows_fresh = false;
    const auto t_dev = std::chrono::steady_clock::now();
    rc = c->eng.apply(edits.data(), edits.size(), d, k, c->nslots(), c->err);
    if (c->opts.log_cycles) {   // (ks_opts.log_cycles: the host's and the device's share of an apply)
        const auto t_out = std::chrono::steady_clock::now();
        std::fprintf(stderr, "apply: %zu records, %zu node edits, host %.3f ms, device %.3f ms\n", k, edits.size(),
                     std::chrono::duration<double, std::milli>(t_dev - t_in).count(),
                     std::chrono::duration<double, std::milli>(t_out - t_dev).count());
    }
    if (rc) {
        // the device may have applied part of the stream: the host goes back to its
        // state before the call (nodes and aggregates) and the store is marked
        // unusable until the next ks_load_graph
        for (auto it = saved.rbegin(); it != saved.rend(); ++it) c->nodes[it->first] = it->second;
        c->sum_others = sum0;
        c->n_sinks = sinks0;
        c->n_tasks = tasks0;
        c->sink_id = sink0;
        c->dev_sink_supply = dsink0;
        c->store_bad = true;
    }
    return rc;
}

// Coalescing follows the store's semantics above: ADD_ARC and UPDATE_ARC are both
// upserts of the full (low, cap, cost, type) and UPDATE_ARC 0/0 deletes, so the
// last record of an arc decides its state (mergeChangesToSameArc and
// removeDuplicateChanges); REMOVE_NODE drops every incident arc, so arc and
// excess records touching the node before its removal are dead
// (purgeChangesBeforeNodeRemoval). Survivors keep their relative order and a
// kept record sits at its own position, after the ADD_NODEs of its endpoints.
int ks_coalesce_deltas(const ks_delta* in, size_t k, ks_delta* out, size_t cap, size_t* count) {
    if (!count || (k && !in) || k > (size_t)INT32_MAX) return KS_E_INVALID;
    for (size_t i = 0; i < k; ++i) {             // ids as the store accepts them (hash keys ≠ 0)
        const ks_delta& x = in[i];
        const bool arc = x.kind == KS_ADD_ARC || x.kind == KS_UPDATE_ARC;
        const uint64_t a = arc ? x.src : x.id, b = arc ? x.dst : 1;
        if (a == 0 || b == 0 || a >= kMaxId || b >= kMaxId) return KS_E_INVALID;
    }
    std::vector<uint8_t> keep(k, 1);
    ArcIndex last_arc;                           // (src, dst) → index of its live record
    last_arc.reserve(k);
    // node id → slot: direct when ids are dense (the FIFO-reused ids of a cell), else hashed
    uint64_t max_id = 0;
    for (size_t i = 0; i < k; ++i) {
        const ks_delta& x = in[i];
        const bool arc = x.kind == KS_ADD_ARC || x.kind == KS_UPDATE_ARC;
        max_id = std::max(max_id, arc ? std::max(x.src, x.dst) : x.id);
    }
    const bool direct = max_id <= 4 * (uint64_t)k + 65536;
    ArcIndex slot_of;                            // sparse ids: id → slot (key (id, 0))
    std::vector<int> head(direct ? max_id + 1 : 0, -1);   // slot → newest record touching it
    std::vector<int> last_exc(direct ? max_id + 1 : 0, -1);  // slot → live SET_EXCESS record
    std::vector<int> link(2 * k, -1);            // record i: next older record at src (2i) / dst (2i+1)
    auto slot = [&](uint64_t id) -> int {
        if (direct) return (int)id;
        int s = slot_of.find(arc_key(id, 0));
        if (s < 0) {
            s = (int)head.size();
            slot_of.insert(arc_key(id, 0), s);
            head.push_back(-1);
            last_exc.push_back(-1);
        }
        return s;
    };
    // the list entry 2i+e belongs to node (e ? dst : src) of record i
    auto push = [&](int s, int i, int e) {
        link[2 * i + e] = head[s];
        head[s] = 2 * i + e;
    };
    for (size_t i = 0; i < k; ++i) {
        const ks_delta& x = in[i];
        switch (x.kind) {
            case KS_ADD_ARC:
            case KS_UPDATE_ARC: {
                const uint64_t key = arc_key(x.src, x.dst);
                const int j = last_arc.find(key);
                if (j >= 0) {
                    keep[j] = 0;
                    last_arc.erase(key);
                }
                last_arc.insert(key, (int)i);
                push(slot(x.src), (int)i, 0);
                if (x.dst != x.src) push(slot(x.dst), (int)i, 1);
                break;
            }
            case KS_SET_EXCESS: {
                const int s = slot(x.id);
                if (last_exc[s] >= 0) keep[last_exc[s]] = 0;
                last_exc[s] = (int)i;
                break;
            }
            case KS_REMOVE_NODE: {
                const int s = slot(x.id);
                for (int e = head[s]; e >= 0; e = link[e]) {
                    const int j = e >> 1;
                    if (!keep[j]) continue;
                    keep[j] = 0;
                    last_arc.erase(arc_key(in[j].src, in[j].dst));
                }
                head[s] = -1;
                if (last_exc[s] >= 0) keep[last_exc[s]] = 0;
                last_exc[s] = -1;
                break;
            }
            default:
                break;                           // ADD_NODE and unknown kinds pass through
        }
    }
    size_t n = 0;
    for (size_t i = 0; i < k; ++i) {
        if (!keep[i]) continue;
        if (out && n < cap) out[n] = in[i];      // n ≤ i: in-place (out == in) is safe
        ++n;
    }
    *count = n;
    return KS_OK;
}

int ks_solve(ks_ctx* c, ks_result* out) {
    if (!c) return KS_E_INVALID;
    if (int g = store_guard(c)) {
        if (out) {
            std::memset(out, 0, sizeof(*out));
            out->status = g;
        }
        return g;
    }
    ks_result r;
    std::memset(&r, 0, sizeof(r));
    c->have_solution = false;
    c->map_fresh = false;
    c->flows_fresh = false;
    int rc = KS_OK;
    // auto-sink: the sink absorbs every other supply (its demand drifts without a
    // message in the reference, graph_manager.go:640, 808)
    if (c->opts.auto_sink && c->n_sinks == 1 && c->dev_sink_supply != -c->sum_others) {
        ks::NodeEdit e;
        std::memset(&e, 0, sizeof(e));
        e.slot = (int32_t)(c->sink_id - 1);
        e.last_rm = -1;
        e.supply = -c->sum_others;
        e.alive = 1;
        e.type = KS_NODE_SINK;
        e.was_alive = 1;
        rc = c->eng.set_nodes(&e, 1, c->err);
        if (rc == KS_OK) c->dev_sink_supply = -c->sum_others;
    }
    if (rc == KS_OK) rc = c->eng.solve(r, c->opts.warm_start != 0, c->err);
    c->map_fresh = false;
    if (rc == KS_OK) c->have_solution = true;   // r.flow_value: measured on device from the resident flow
    r.status = rc;
    if (out) *out = r;
    return rc;
}

int ks_solve_many(ks_ctx* const* ctxs, size_t k, int workers, ks_result* results) {
    if (k && !ctxs) return KS_E_INVALID;
    for (size_t i = 0; i < k; ++i)
        if (!ctxs[i]) return KS_E_INVALID;
    std::vector<int> rcs(k, KS_OK);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < k;) rcs[i] = ks_solve(ctxs[i], results ? &results[i] : nullptr);
    };
    size_t nw = workers > 0 ? (size_t)workers : 4;
    nw = std::min(nw, k);
    std::vector<std::thread> pool;
    for (size_t w = 1; w < nw; ++w) pool.emplace_back(work);
    if (nw) work();
    for (auto& t : pool) t.join();
    for (int rc : rcs)
        if (rc != KS_OK) return rc;
    return KS_OK;
}

int ks_get_flows(ks_ctx* c, ks_flow* out, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    if (!c->flows_fresh) {
        int rc = c->eng.flows(c->flows, c->err);
        if (rc) return rc;
        c->flows_fresh = true;
    }
    if (out) std::memcpy(out, c->flows.data(), std::min(cap, c->flows.size()) * sizeof(ks_flow));
    *count = c->flows.size();
    return KS_OK;
}

// Pairs from the device decomposition (Engine::task_pu): the i-th live task slot
// in slot order ↔ the i-th entry of the device vector.
int ks_get_task_mapping(ks_ctx* c, uint64_t* task, uint64_t* pu, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    // one device decomposition per solve: the usual count-then-fill call pair
    // reuses it
    if (!c->map_fresh) {
        size_t nt = 0;
        int rc = c->eng.task_pu(nullptr, 0, &nt, c->n_tasks, c->err);
        if (rc) return rc;
        uint64_t* dev = nullptr;
        rc = c->eng.scratch(&dev, nt, c->err);
        if (rc == KS_OK) rc = c->eng.task_pu(dev, nt, &nt, c->n_tasks, c->err);
        c->map_dense.resize(nt);
        if (rc == KS_OK) rc = c->eng.download(c->map_dense.data(), dev, nt * sizeof(uint64_t), c->err);
        if (rc) return rc;
        c->map_fresh = true;
    }
    const std::vector<uint64_t>& dense = c->map_dense;
    const size_t nt = dense.size();
    size_t k = 0, ti = 0;
    for (uint64_t id = 1; id < c->nodes.size() && ti < nt; ++id) {
        const NodeRec& r = c->nodes[id];
        if (!r.alive || r.type != KS_NODE_TASK) continue;
        const uint64_t p = dense[ti++];
        if (!p) continue;
        if (task && pu && k < cap) {
            task[k] = id;
            pu[k] = p;
        }
        ++k;
    }
    *count = k;
    return KS_OK;
}

int ks_get_task_pu_device(ks_ctx* c, uint64_t* dev_out, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    return c->eng.task_pu(dev_out, cap, count, c->n_tasks, c->err);
}

int ks_set_bindings(ks_ctx* c, const uint64_t* task, const uint64_t* pu, size_t k) {
    if (!c) return KS_E_INVALID;
    if (int g = store_guard(c)) return g;
    if (k && (!task || !pu)) return c->fail(KS_E_INVALID, "null binding array");
    for (size_t i = 0; i < k; ++i) {
        if (!node_alive(c, task[i]) || c->nodes[task[i]].type != KS_NODE_TASK)
            return c->fail(KS_E_INVALID, "binding of a node that is not a live task: " + std::to_string(task[i]));
        if (pu[i] && (!node_alive(c, pu[i]) || c->nodes[pu[i]].type != KS_NODE_PU))
            return c->fail(KS_E_INVALID, "binding to a node that is not a live PU: " + std::to_string(pu[i]));
    }
    return c->eng.set_bindings(task, pu, k, c->err);
}

int ks_scheduling_deltas(ks_ctx* c, int commit, ks_sched_delta* out, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    size_t n = 0;
    int rc = c->eng.sched_deltas(0, nullptr, &n, c->n_tasks, c->err);   // count (nothing committed)
    if (rc || !out) {
        *count = n;
        return rc;
    }
    if (cap < n) {
        *count = n;
        return c->fail(KS_E_INVALID, "output buffer smaller than the delta count");
    }
    std::vector<ks_sched_delta> v;
    rc = c->eng.sched_deltas(commit, &v, &n, c->n_tasks, c->err);
    if (rc) return rc;
    if (!v.empty()) std::memcpy(out, v.data(), v.size() * sizeof(ks_sched_delta));
    *count = v.size();
    return KS_OK;
}

int ks_update_unsched_costs(ks_ctx* c, const uint64_t* ids, size_t k, int32_t mode, int64_t unsched_cost,
                            int64_t continuation_cost, size_t* changed) {
    if (!c) return KS_E_INVALID;
    if (int g = store_guard(c)) return g;
    if (mode != KS_COST_SET && mode != KS_COST_ADD) return c->fail(KS_E_INVALID, "unknown cost mode");
    const int64_t lim = int64_t(1) << 40;
    if (unsched_cost > lim || unsched_cost < -lim || continuation_cost > lim || continuation_cost < -lim)
        return c->fail(KS_E_RANGE, "cost outside the supported range");
    for (size_t i = 0; ids && i < k; ++i)
        if (!node_alive(c, ids[i])) return c->fail(KS_E_INVALID, "unscheduled aggregator " + std::to_string(ids[i]) +
                                                                     " is not a live node");
    size_t ch = 0;
    int rc = c->eng.unsched_costs(ids, ids ? k : 0, mode, unsched_cost, continuation_cost, &ch, c->err);
    if (rc == KS_OK && ch) {
        c->have_solution = false;
        c->map_fresh = false;
        c->flows_fresh = false;
    }
    if (changed) *changed = ch;
    return rc;
}

int ks_topology_stats(ks_ctx* c, uint64_t max_tasks_per_pu, const uint64_t* pu_ids, const uint64_t* pu_running,
                      size_t k, uint64_t* slots_below, uint64_t* running_below, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (int g = store_guard(c)) return g;
    const size_t n = (size_t)c->nslots();
    *count = n;
    if (!slots_below || !running_below) return KS_OK;
    if (cap < n) return c->fail(KS_E_INVALID, "output buffers smaller than the node id range");
    if (pu_ids && k && !pu_running) return c->fail(KS_E_INVALID, "null running-count array");
    for (size_t i = 0; pu_ids && i < k; ++i)
        if (!node_alive(c, pu_ids[i]) || c->nodes[pu_ids[i]].type != KS_NODE_PU)
            return c->fail(KS_E_INVALID, "running count for a node that is not a live PU");
    const int64_t sink = c->n_sinks == 1 ? (int64_t)c->sink_id - 1 : -1;
    int rc = c->eng.topology_stats(max_tasks_per_pu, pu_ids, pu_running, pu_ids ? k : 0, sink, slots_below,
                                   running_below, c->err);
    if (!c->eng.solved()) c->have_solution = c->flows_fresh = c->map_fresh = false;   // a pending CSR rebuild ran
    return rc;
}

int ks_get_graph(ks_ctx* c, ks_node* nodes, size_t ncap, size_t* n, ks_arc* arcs, size_t acap, size_t* m) {
    if (!c || !n || !m) return KS_E_INVALID;
    if (int g = store_guard(c)) return g;
    size_t k = 0;
    for (uint64_t id = 1; id < c->nodes.size(); ++id) {
        const NodeRec& r = c->nodes[id];
        if (!r.alive) continue;
        if (nodes && k < ncap) nodes[k] = ks_node{id, r.excess, r.type, 0};
        ++k;
    }
    *n = k;
    std::vector<ks_arc> v;
    int rc = c->eng.arcs(v, c->err);
    if (rc) return rc;
    if (arcs) std::memcpy(arcs, v.data(), std::min(acap, v.size()) * sizeof(ks_arc));
    *m = v.size();
    return KS_OK;
}

int ks_get_store_stats(ks_ctx* c, ks_store_stats* out) {
    if (!c || !out) return KS_E_INVALID;
    c->eng.store_stats(out);
    return KS_OK;
}

}  // extern "C"
