// Host-only stand-in for ks::Engine (profiling the graph store on a CPU box):
// keeps the uploaded sizes, "solves" instantly, reports zero flows and no tasks.
#include <vector>

#include "../../ksched_amd/csrc/ks_engine.h"

namespace ks {
struct EngineImpl {
    int64_t n = 0, m = 0;
    std::vector<uint64_t> scratch;
};
Engine::Engine() : p_(new EngineImpl) {}
Engine::~Engine() { delete p_; }
int Engine::init(int, const ks_opts&, std::string&) { return KS_OK; }
int Engine::upload(int64_t n, int64_t m, const int32_t*, const int32_t*, const int64_t*, const int64_t*,
                   const int64_t*, const int64_t*, const uint8_t*, const int32_t*, const uint8_t*, std::string&) {
    p_->n = n;
    p_->m = m;
    return KS_OK;
}
int Engine::solve(ks_result& r, bool, std::string&) {
    r.n_nodes = p_->n;
    r.n_arcs = p_->m;
    return KS_OK;
}
int Engine::download_flows(int64_t* f, std::string&) {
    for (int64_t i = 0; i < p_->m; ++i) f[i] = 0;
    return KS_OK;
}
int Engine::task_pu(uint64_t*, size_t, size_t* count, std::string&) {
    *count = 0;
    return KS_OK;
}
int Engine::scratch(uint64_t** dev, size_t n, std::string&) {
    p_->scratch.resize(n + 1);
    *dev = p_->scratch.data();
    return KS_OK;
}
int Engine::download(void*, const void*, size_t, std::string&) { return KS_OK; }
int Engine::device() const { return 0; }
}  // namespace ks
