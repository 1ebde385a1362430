// ks_host.cpp — host runtime and C-ABI of libksmcmf (include/ksmcmf.h).
//
// Mirrors the reference's solver boundary, scheduling/flow/placement/solver.go:
//   ks_create         ↔ NewSolver (:49-55) + startSolver (:92-109)
//   ks_load_graph     ↔ writeGraph → dimacs.Export (:111-116, dimacs/export.go:11-29)
//   ks_apply_deltas   ↔ writeIncremental → dimacs.ExportIncremental (:118-123)
//   ks_solve          ↔ the Flowlessly solve
//   ks_get_flows      ↔ the "f" lines consumed by readFlowGraph (:134-179)
//   ks_get_task_mapping ↔ parseFlowToMapping (:183-269)
// The graph store keeps ksched's node/arc semantics (flowgraph/graph.go:27-182):
// NodeIDs index node slots directly, at most one arc per (src, dst), REMOVE_NODE
// drops incident arcs. The device engine (ks_engine.hip) solves the compacted graph.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ksmcmf.h"
#include "ks_engine.h"

namespace {

struct NodeRec {
    int64_t excess = 0;
    int32_t type = 0;
    bool alive = false;
    bool fresh = true;     // created since the last successful solve (warm start)
};

struct ArcRec {
    uint64_t src = 0, dst = 0;
    int64_t low = 0, cap = 0, cost = 0;
    int32_t type = 0;
    bool alive = false;
    int prev_up = -1;      // index in the last solved upload; −1 = new since (warm start)
};

constexpr uint64_t kMaxId = (1ULL << 30);

inline uint64_t arc_key(uint64_t s, uint64_t d) { return (s << 32) | d; }

// (src, dst) → arc slot: open addressing with linear probing and backward-shift
// deletion (no tombstones), power-of-two capacity kept under 1/2 load. Keys are
// never 0 (node ids start at 1), so 0 marks an empty bucket. The incremental
// stream of a scheduling round (~80k upserts/deletes at config 4) is dominated
// by these lookups.
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

struct ks_ctx {
    ks::Engine eng;
    ks_opts opts{};
    std::string err;

    std::vector<NodeRec> nodes;            // index = NodeID (slot 0 unused)
    std::vector<ArcRec> arcs;
    std::vector<int> free_arcs;
    ArcIndex arc_of;
    std::vector<std::vector<int>> inc;     // per node: incident arc slots (lazy, see push_incident)
    std::vector<uint32_t> live_deg;        // per node: live incident arcs
    bool dirty = true;
    bool reloaded = true;                  // ks_load_graph since the last solve: no warm start

    // last upload (compact arrays) and solve outputs
    std::vector<int> up_arc;               // compact index → arc slot
    std::vector<int32_t> c_src, c_dst;
    std::vector<int64_t> c_low, c_cap, c_cost, c_supply;
    std::vector<int32_t> c_prev;
    std::vector<uint8_t> c_fresh, c_type;
    std::vector<int64_t> flows;
    bool have_solution = false;
    bool flows_fresh = false;
    int64_t n_slots = 0;

    int fail(int code, const std::string& msg) {
        err = msg;
        return code;
    }
};

namespace {

void ensure_node(ks_ctx* c, uint64_t id) {
    if (id >= c->nodes.size()) {
        c->nodes.resize(id + 1);
        c->inc.resize(id + 1);
        c->live_deg.resize(id + 1, 0);
    }
}

bool node_alive(const ks_ctx* c, uint64_t id) { return id < c->nodes.size() && c->nodes[id].alive; }

void kill_arc(ks_ctx* c, int slot) {
    ArcRec& a = c->arcs[slot];
    if (!a.alive) return;
    a.alive = false;
    a.prev_up = -1;
    c->arc_of.erase(arc_key(a.src, a.dst));
    c->free_arcs.push_back(slot);
    --c->live_deg[a.src];
    --c->live_deg[a.dst];
}

// Incidence lists are append-only between compactions: a killed arc's slot stays
// in both endpoints' lists (and may later be reused by an arc of other nodes).
// Long-lived hubs (sink, aggregators) would otherwise grow with history, so a
// list is compacted to its live arcs once it exceeds twice its live degree.
void push_incident(ks_ctx* c, uint64_t v, int slot) {
    std::vector<int>& l = c->inc[v];
    if (l.size() >= 2 * (size_t)c->live_deg[v] + 16) {
        size_t k = 0;
        for (int t : l) {
            const ArcRec& a = c->arcs[t];
            if (a.alive && (a.src == v || a.dst == v)) l[k++] = t;
        }
        l.resize(k);
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
    }
    l.push_back(slot);
}

int upsert_arc(ks_ctx* c, uint64_t s, uint64_t d, int64_t low, int64_t cap, int64_t cost, int32_t type) {
    if (!node_alive(c, s) || !node_alive(c, d))
        return c->fail(KS_E_INVALID, "arc " + std::to_string(s) + "->" + std::to_string(d) + " has a missing endpoint");
    if (s == d) return c->fail(KS_E_INVALID, "self-loop arc at node " + std::to_string(s));
    if (low < 0 || cap < 0 || low > cap)
        return c->fail(KS_E_INVALID, "arc " + std::to_string(s) + "->" + std::to_string(d) + " has low > cap");
    if (cap > (int64_t(1) << 53) || cost > (int64_t(1) << 40) || cost < -(int64_t(1) << 40))
        return c->fail(KS_E_RANGE, "arc capacity or cost outside the supported range");
    int slot = c->arc_of.find(arc_key(s, d));
    if (slot < 0) {
        if (!c->free_arcs.empty()) {
            slot = c->free_arcs.back();
            c->free_arcs.pop_back();
        } else {
            slot = (int)c->arcs.size();
            c->arcs.emplace_back();
        }
        c->arc_of.insert(arc_key(s, d), slot);
        c->arcs[slot].prev_up = -1;
        c->arcs[slot].alive = false;       // not yet: compaction below must skip it
        push_incident(c, s, slot);
        push_incident(c, d, slot);
        ++c->live_deg[s];
        ++c->live_deg[d];
    }
    ArcRec& a = c->arcs[slot];
    a.src = s;
    a.dst = d;
    a.low = low;
    a.cap = cap;
    a.cost = cost;
    a.type = type;
    a.alive = true;
    return KS_OK;
}

int add_node(ks_ctx* c, uint64_t id, int64_t excess, int32_t type) {
    if (id == 0 || id >= kMaxId) return c->fail(KS_E_RANGE, "node id " + std::to_string(id) + " out of range");
    ensure_node(c, id);
    if (c->nodes[id].alive)
        return c->fail(KS_E_INVALID, "node " + std::to_string(id) + " already present");  // graph.go:95-98
    c->nodes[id] = NodeRec{excess, type, true, true};
    return KS_OK;
}

int remove_node(ks_ctx* c, uint64_t id) {
    if (!node_alive(c, id)) return c->fail(KS_E_INVALID, "remove of missing node " + std::to_string(id));
    for (int slot : c->inc[id]) {
        const ArcRec& a = c->arcs[slot];
        if (a.alive && (a.src == id || a.dst == id)) kill_arc(c, slot);
    }
    c->inc[id].clear();
    c->live_deg[id] = 0;
    c->nodes[id] = NodeRec{};
    return KS_OK;
}

// Compact the live graph into device input arrays (node slot = id − 1).
int upload(ks_ctx* c) {
    uint64_t maxid = 0;
    for (uint64_t id = c->nodes.size(); id-- > 1;)
        if (c->nodes[id].alive) {
            maxid = id;
            break;
        }
    const int64_t n = (int64_t)maxid;
    c->n_slots = n;
    c->c_supply.assign(n, 0);
    c->c_type.assign(n, 0);
    int64_t others = 0;
    int64_t sink = -1, nsinks = 0;
    for (int64_t v = 0; v < n; ++v) {
        const NodeRec& r = c->nodes[v + 1];
        if (!r.alive) continue;
        c->c_supply[v] = r.excess;
        c->c_type[v] = (uint8_t)std::min<int32_t>(std::max<int32_t>(r.type, 0), 255);
        if (r.type == KS_NODE_SINK) {
            sink = v;
            ++nsinks;
        } else {
            others += r.excess;
        }
    }
    if (c->opts.auto_sink && nsinks == 1) c->c_supply[sink] = -others;
    const bool warm = c->opts.warm_start && !c->reloaded;
    const size_t live = c->arcs.size() - c->free_arcs.size();
    c->up_arc.resize(live);
    c->c_src.resize(live);
    c->c_dst.resize(live);
    c->c_low.resize(live);
    c->c_cap.resize(live);
    c->c_cost.resize(live);
    c->c_prev.resize(warm ? live : 0);
    size_t k = 0;
    for (int slot = 0; slot < (int)c->arcs.size(); ++slot) {
        const ArcRec& a = c->arcs[slot];
        if (!a.alive) continue;
        c->up_arc[k] = slot;
        c->c_src[k] = (int32_t)(a.src - 1);
        c->c_dst[k] = (int32_t)(a.dst - 1);
        c->c_low[k] = a.low;
        c->c_cap[k] = a.cap;
        c->c_cost[k] = a.cost;
        if (warm) c->c_prev[k] = a.prev_up;
        ++k;
    }
    if (k != live) return c->fail(KS_E_INVALID, "internal: arc free list out of sync");
    if (warm) {
        c->c_fresh.assign(n, 0);
        for (int64_t v = 0; v < n; ++v) c->c_fresh[v] = c->nodes[v + 1].alive && c->nodes[v + 1].fresh;
    }
    const int64_t m = (int64_t)c->up_arc.size();
    int rc = c->eng.upload(n, m, c->c_src.data(), c->c_dst.data(), c->c_low.data(), c->c_cap.data(),
                           c->c_cost.data(), c->c_supply.data(), c->c_type.data(), warm ? c->c_prev.data() : nullptr,
                           warm ? c->c_fresh.data() : nullptr, c->err);
    if (rc == KS_OK) c->dirty = false;
    return rc;
}

int fetch_flows(ks_ctx* c) {
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    if (c->flows_fresh) return KS_OK;
    c->flows.assign(c->up_arc.size(), 0);
    int rc = c->eng.download_flows(c->flows.data(), c->err);
    if (rc == KS_OK) c->flows_fresh = true;
    return rc;
}

}  // namespace

extern "C" {

int ks_abi_version(void) { return KSMCMF_ABI_VERSION; }

void ks_default_opts(ks_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->alpha = 8;
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
    c->inc.resize(1);
    c->live_deg.resize(1, 0);
    return c;
}

void ks_destroy(ks_ctx* c) { delete c; }

const char* ks_last_error(ks_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ks_load_graph(ks_ctx* c, const ks_node* nodes, size_t n, const ks_arc* arcs, size_t m) {
    if (!c) return KS_E_INVALID;
    if ((n && !nodes) || (m && !arcs)) return c->fail(KS_E_INVALID, "null input array");
    c->nodes.assign(1, NodeRec{});
    c->inc.assign(1, {});
    c->live_deg.assign(1, 0);
    c->arcs.clear();
    c->free_arcs.clear();
    c->arc_of.clear();
    c->arc_of.reserve(m);
    c->arcs.reserve(m);
    c->have_solution = false;
    c->dirty = true;
    c->reloaded = true;
    uint64_t maxid = 0;
    for (size_t i = 0; i < n; ++i) maxid = std::max<uint64_t>(maxid, nodes[i].id);
    if (maxid < kMaxId) {
        c->nodes.reserve(maxid + 1);
        c->inc.reserve(maxid + 1);
        c->live_deg.reserve(maxid + 1);
    }
    for (size_t i = 0; i < n; ++i) {
        int rc = add_node(c, nodes[i].id, nodes[i].excess, nodes[i].type);
        if (rc) return rc;
    }
    {   // size the incidence lists once (one pass over the arcs)
        std::vector<uint32_t> deg(c->nodes.size(), 0);
        for (size_t i = 0; i < m; ++i) {
            if (arcs[i].src < deg.size()) ++deg[arcs[i].src];
            if (arcs[i].dst < deg.size()) ++deg[arcs[i].dst];
        }
        for (size_t v = 0; v < deg.size(); ++v)
            if (deg[v]) c->inc[v].reserve(deg[v]);
    }
    for (size_t i = 0; i < m; ++i) {
        const ks_arc& a = arcs[i];
        if (a.low > (uint64_t)INT64_MAX || a.cap > (uint64_t)INT64_MAX)
            return c->fail(KS_E_RANGE, "arc bound exceeds int64");
        int rc = upsert_arc(c, a.src, a.dst, (int64_t)a.low, (int64_t)a.cap, a.cost, a.type);
        if (rc) return rc;
    }
    return KS_OK;
}

int ks_apply_deltas(ks_ctx* c, const ks_delta* d, size_t k) {
    if (!c) return KS_E_INVALID;
    if (k && !d) return c->fail(KS_E_INVALID, "null delta array");
    c->dirty = true;
    c->have_solution = false;
    for (size_t i = 0; i < k; ++i) {
        const ks_delta& x = d[i];
        int rc = KS_OK;
        switch (x.kind) {
            case KS_ADD_NODE:
                rc = add_node(c, x.id, x.excess, x.type);
                break;
            case KS_REMOVE_NODE:
                rc = remove_node(c, x.id);
                break;
            case KS_ADD_ARC:
                if (x.low > (uint64_t)INT64_MAX || x.cap > (uint64_t)INT64_MAX) {
                    rc = c->fail(KS_E_RANGE, "arc bound exceeds int64");
                    break;
                }
                rc = upsert_arc(c, x.src, x.dst, (int64_t)x.low, (int64_t)x.cap, x.cost, x.type);
                break;
            case KS_UPDATE_ARC: {
                if (x.src == 0 || x.dst == 0 || x.src >= kMaxId || x.dst >= kMaxId) {
                    rc = c->fail(KS_E_RANGE, "arc endpoint id out of range");
                    break;
                }
                if (x.low == 0 && x.cap == 0) {  // DeleteArc / ChangeArc(0,0): no capacity left
                    const int slot = c->arc_of.find(arc_key(x.src, x.dst));
                    if (slot >= 0) kill_arc(c, slot);
                    else if (!node_alive(c, x.src) || !node_alive(c, x.dst))
                        rc = c->fail(KS_E_INVALID, "update of arc with a missing endpoint");
                    break;
                }
                if (x.low > (uint64_t)INT64_MAX || x.cap > (uint64_t)INT64_MAX) {
                    rc = c->fail(KS_E_RANGE, "arc bound exceeds int64");
                    break;
                }
                rc = upsert_arc(c, x.src, x.dst, (int64_t)x.low, (int64_t)x.cap, x.cost, x.type);
                break;
            }
            case KS_SET_EXCESS:
                if (!node_alive(c, x.id)) rc = c->fail(KS_E_INVALID, "excess of missing node " + std::to_string(x.id));
                else c->nodes[x.id].excess = x.excess;
                break;
            default:
                rc = c->fail(KS_E_INVALID, "unknown delta kind " + std::to_string(x.kind));
        }
        if (rc) return rc;
    }
    return KS_OK;
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
    ks_result r;
    std::memset(&r, 0, sizeof(r));
    c->have_solution = false;
    c->flows_fresh = false;
    int rc = KS_OK;
    if (c->dirty) rc = upload(c);
    if (rc == KS_OK) rc = c->eng.solve(r, c->opts.warm_start != 0, c->err);
    if (rc == KS_OK) {
        // remember which upload index every arc had, for the next warm start
        for (size_t i = 0; i < c->up_arc.size(); ++i) c->arcs[c->up_arc[i]].prev_up = (int)i;
        for (auto& nd : c->nodes) nd.fresh = false;
        c->reloaded = false;
        c->have_solution = true;   // r.flow_value: measured on device from the resident flow
    }
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
    int rc = fetch_flows(c);
    if (rc) return rc;
    size_t k = 0;
    for (size_t i = 0; i < c->flows.size(); ++i)
        if (c->flows[i] > 0) {
            if (out && k < cap) {
                const ArcRec& a = c->arcs[c->up_arc[i]];
                out[k] = ks_flow{a.src, a.dst, c->flows[i]};
            }
            ++k;
        }
    *count = k;
    return KS_OK;
}

// Pairs from the device decomposition (Engine::task_pu): the i-th task slot in
// slot order ↔ the i-th entry of the device vector.
int ks_get_task_mapping(ks_ctx* c, uint64_t* task, uint64_t* pu, size_t cap, size_t* count) {
    if (!c || !count) return KS_E_INVALID;
    if (!c->have_solution) return c->fail(KS_E_INVALID, "no successful solve on this context");
    size_t nt = 0;
    int rc = c->eng.task_pu(nullptr, 0, &nt, c->err);
    if (rc) return rc;
    uint64_t* dev = nullptr;
    rc = c->eng.scratch(&dev, nt, c->err);
    if (rc == KS_OK) rc = c->eng.task_pu(dev, nt, &nt, c->err);
    std::vector<uint64_t> dense(nt);
    if (rc == KS_OK) rc = c->eng.download(dense.data(), dev, nt * sizeof(uint64_t), c->err);
    if (rc) return rc;
    size_t k = 0, ti = 0;
    for (int64_t v = 0; v < c->n_slots && ti < nt; ++v) {
        const NodeRec& r = c->nodes[v + 1];
        if (!r.alive || r.type != KS_NODE_TASK) continue;
        const uint64_t p = dense[ti++];
        if (!p) continue;
        if (task && pu && k < cap) {
            task[k] = (uint64_t)v + 1;
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
    return c->eng.task_pu(dev_out, cap, count, c->err);
}

}  // extern "C"
