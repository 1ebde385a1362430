// ks_flow_scheduler — a flow_scheduler-compatible DIMACS daemon over libksmcmf.
//
// ksched talks to its solver through a child process (placement/solver.go:92-109:
// flow_scheduler --graph_has_node_types=true --algorithm=... --print_assignments=false
// --debug_output=true [--daemon=false]). This binary speaks that protocol, so an
// unmodified ksched (FlowlesslyBinary pointed here) schedules on the GPU:
//
//   stdin, first iteration   full graph (dimacs/export.go:11-76): "p min n m",
//                            "n id excess type", "a src dst low cap cost", comments
//                            ("c ..."), terminated by "c EOI"
//   stdin, later iterations  change records (dimacs/*_change.go GenerateChange):
//                            "n id excess type", "r id", "a src dst low cap cost type",
//                            "x src dst low cap cost type oldcost", then "c EOI"
//   stdout, per iteration    "f src dst flow" for every arc carrying flow, "s cost",
//                            "c EOI" — exactly what readFlowGraph accepts
//                            (placement/solver.go:134-179)
//
// --daemon=false solves the first graph only. --device=N picks the HIP device.
// --parse-only parses the stream and prints per-iteration counts without a
// device (used by the CPU tests). --coalesce runs each change block through
// ks_coalesce_deltas before applying it (the reference's optimizeChanges switches,
// graph_change_manager.go:220-229; off by default there too). Errors go to stderr with a non-zero exit, the
// way the reference panics when the pipe breaks.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ksmcmf.h"

namespace {

struct Stream {
    std::vector<ks_node> nodes;
    std::vector<ks_arc> arcs;
    std::vector<ks_delta> deltas;
    bool eoi = false;
};

// Parse up to 8 integer fields after the record letter; returns the count.
int fields(const char* p, long long* out, int max) {
    int k = 0;
    while (k < max) {
        while (*p == ' ' || *p == '\t') ++p;
        if (*p == '\0' || *p == '\n' || *p == '\r') break;
        char* end = nullptr;
        errno = 0;
        const long long v = std::strtoll(p, &end, 10);
        if (end == p || errno) return -1;
        out[k++] = v;
        p = end;
    }
    while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') ++p;
    return *p ? -1 : k;
}

[[noreturn]] void die(const std::string& msg, long long line) {
    std::fprintf(stderr, "ks_flow_scheduler: line %lld: %s\n", line, msg.c_str());
    std::exit(2);
}

// Read one iteration (up to "c EOI"). full = the first, whole-graph iteration.
bool read_iteration(FILE* in, bool full, Stream& s, long long& lineno) {
    s.nodes.clear();
    s.arcs.clear();
    s.deltas.clear();
    s.eoi = false;
    static std::vector<char> buf(1 << 16);
    bool any = false;
    while (std::fgets(buf.data(), (int)buf.size(), in)) {
        ++lineno;
        any = true;
        const char* l = buf.data();
        const size_t len = std::strlen(l);
        if (len + 1 == buf.size() && l[len - 1] != '\n') die("line too long", lineno);
        long long f[8];
        switch (l[0]) {
            case 'c':
                if (std::strncmp(l, "c EOI", 5) == 0 && (l[5] == '\n' || l[5] == '\r' || l[5] == '\0')) {
                    s.eoi = true;
                    return true;
                }
                break;   // comments and "c nd ..." descriptors
            case 'p':
                break;   // "p min n m": sizes are taken from the records
            case '\n':
            case '\r':
                break;
            case 'n': {
                const int k = fields(l + 1, f, 8);
                if (k != 3) die("expected 'n id excess type'", lineno);
                if (full) {
                    s.nodes.push_back(ks_node{(uint64_t)f[0], f[1], (int32_t)f[2], 0});
                } else {
                    ks_delta d{};
                    d.kind = KS_ADD_NODE;
                    d.id = (uint64_t)f[0];
                    d.excess = f[1];
                    d.type = (int32_t)f[2];
                    s.deltas.push_back(d);
                }
                break;
            }
            case 'a': {
                const int k = fields(l + 1, f, 8);
                if (k != 5 && k != 6) die("expected 'a src dst low cap cost [type]'", lineno);
                if (f[0] < 0 || f[1] < 0 || f[2] < 0 || f[3] < 0) die("negative id or bound", lineno);
                const int32_t type = k == 6 ? (int32_t)f[5] : 0;
                if (full) {
                    s.arcs.push_back(ks_arc{(uint64_t)f[0], (uint64_t)f[1], (uint64_t)f[2], (uint64_t)f[3], f[4], type, 0});
                } else {
                    ks_delta d{};
                    d.kind = KS_ADD_ARC;
                    d.src = (uint64_t)f[0];
                    d.dst = (uint64_t)f[1];
                    d.low = (uint64_t)f[2];
                    d.cap = (uint64_t)f[3];
                    d.cost = f[4];
                    d.type = type;
                    s.deltas.push_back(d);
                }
                break;
            }
            case 'x': {
                const int k = fields(l + 1, f, 8);
                if (k != 7 && k != 6) die("expected 'x src dst low cap cost type oldcost'", lineno);
                if (full) die("change record in the full graph", lineno);
                ks_delta d{};
                d.kind = KS_UPDATE_ARC;
                d.src = (uint64_t)f[0];
                d.dst = (uint64_t)f[1];
                d.low = (uint64_t)f[2];
                d.cap = (uint64_t)f[3];
                d.cost = f[4];
                d.type = (int32_t)f[5];
                d.old_cost = k == 7 ? f[6] : 0;
                s.deltas.push_back(d);
                break;
            }
            case 'r': {
                const int k = fields(l + 1, f, 8);
                if (k != 1) die("expected 'r id'", lineno);
                if (full) die("change record in the full graph", lineno);
                ks_delta d{};
                d.kind = KS_REMOVE_NODE;
                d.id = (uint64_t)f[0];
                s.deltas.push_back(d);
                break;
            }
            default:
                die(std::string("unknown record '") + l[0] + "'", lineno);
        }
    }
    return any;   // EOF: true when a partial iteration (no "c EOI") was read
}

void emit(ks_ctx* ctx, FILE* out) {
    size_t count = 0;
    if (ks_get_flows(ctx, nullptr, 0, &count) != KS_OK) {
        std::fprintf(stderr, "ks_flow_scheduler: %s\n", ks_last_error(ctx));
        std::exit(3);
    }
    std::vector<ks_flow> fl(count);
    if (count && ks_get_flows(ctx, fl.data(), count, &count) != KS_OK) {
        std::fprintf(stderr, "ks_flow_scheduler: %s\n", ks_last_error(ctx));
        std::exit(3);
    }
    for (const ks_flow& f : fl)
        std::fprintf(out, "f %llu %llu %lld\n", (unsigned long long)f.src, (unsigned long long)f.dst, (long long)f.flow);
}

}  // namespace

int main(int argc, char** argv) {
    bool daemon = true, parse_only = false, coalesce = false;
    int device = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--daemon=false") daemon = false;
        else if (a == "--parse-only") parse_only = true;
        else if (a == "--coalesce") coalesce = true;   // graph_change_manager.go:220-229 optimizeChanges
        else if (a.rfind("--device=", 0) == 0) device = std::atoi(a.c_str() + 9);
        // the reference's other flags (--graph_has_node_types, --algorithm,
        // --print_assignments, --debug_output) need no action here
    }
    ks_ctx* ctx = nullptr;
    if (!parse_only) {
        ks_opts o;
        ks_default_opts(&o);
        ctx = ks_create(device, &o);
        if (!ctx) {
            std::fprintf(stderr, "ks_flow_scheduler: no usable HIP device %d\n", device);
            return 3;
        }
    }
    Stream s;
    long long lineno = 0;
    bool first = true;
    while (read_iteration(stdin, first, s, lineno)) {
        if (!s.eoi) die("input ended inside an iteration (no 'c EOI')", lineno);
        if (coalesce && !first) {
            size_t kept = 0;
            if (ks_coalesce_deltas(s.deltas.data(), s.deltas.size(), s.deltas.data(), s.deltas.size(), &kept) != KS_OK)
                die("invalid node id in change records", lineno);
            s.deltas.resize(kept);
        }
        if (parse_only) {
            std::printf("iteration %s nodes %zu arcs %zu deltas %zu\n", first ? "full" : "incremental", s.nodes.size(),
                        s.arcs.size(), s.deltas.size());
            std::fflush(stdout);
        } else {
            int rc = first ? ks_load_graph(ctx, s.nodes.data(), s.nodes.size(), s.arcs.data(), s.arcs.size())
                           : ks_apply_deltas(ctx, s.deltas.data(), s.deltas.size());
            ks_result r;
            if (rc == KS_OK) rc = ks_solve(ctx, &r);
            if (rc != KS_OK) {
                std::fprintf(stderr, "ks_flow_scheduler: %s\n", ks_last_error(ctx));
                ks_destroy(ctx);
                return 4;
            }
            emit(ctx, stdout);
            std::fprintf(stdout, "s %lld\nc EOI\n", (long long)r.total_cost);
            std::fflush(stdout);
        }
        first = false;
        if (!daemon) break;
    }
    if (ctx) ks_destroy(ctx);
    return 0;
}
