// ks_batch.hip — config 5 behind the C-ABI: independent cell graphs sharded over
// GPUs, solved concurrently, and their task→PU mappings gathered to rank 0 over
// RCCL inside libksmcmf (SURVEY §7 step 6, §8 row e).
//
// A single solve does not shard, so multi-GPU throughput comes
// from independent graphs (cluster cells, what-if variants). Graph g belongs to
// global rank g mod world (round-robin); each device solves the
// disjoint union of its graphs as ONE device solve (the min-cost flow of a
// disjoint union is the union of the optima). After the solves every device
// packs one row per graph — [cost, flow value, PU id of each task (cell-local,
// 0 = unscheduled)] — and rank 0 receives every device's rows with
// ncclSend/ncclRecv in one group: a single collective, no data-path exchange.
// Two ways to build the communicator: ks_batch_create (one process, several
// devices: ncclCommInitAll) and ks_batch_create_rank (one process per GPU, e.g.
// under torch.distributed.run: ncclCommInitRank with an id from rank 0).
// RCCL is loaded with dlopen on the first batch (the single-graph API never
// needs it); a process that already holds RCCL (torch) shares its copy.
// A TEST build of the library (-DKS_FAKE_COMM: libksmcmf_fakecomm.so, made by
// ksched_amd/_build.py build_fake_comm, never the shipped libksmcmf.so) binds the
// same entry points to tests/fake_comm/fake_nccl.cpp compiled into it instead —
// the ranks of one process on one GPU — so the world > 1 path of ks_batch_gather
// runs on a one-GPU box.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifdef KS_FAKE_COMM
extern "C" {
ncclResult_t ks_fake_ncclGetUniqueId(ncclUniqueId*);
ncclResult_t ks_fake_ncclCommInitAll(ncclComm_t*, int, const int*);
ncclResult_t ks_fake_ncclCommInitRank(ncclComm_t*, int, ncclUniqueId, int);
ncclResult_t ks_fake_ncclCommDestroy(ncclComm_t);
ncclResult_t ks_fake_ncclGroupStart();
ncclResult_t ks_fake_ncclGroupEnd();
ncclResult_t ks_fake_ncclSend(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
ncclResult_t ks_fake_ncclRecv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
ncclResult_t ks_fake_ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
const char* ks_fake_ncclGetErrorString(ncclResult_t);
}
#endif

#include "ks_ctx.h"

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;

    bool load(std::string& err) {
        if (h) return true;
#ifdef KS_FAKE_COMM
        GetUniqueId = ks_fake_ncclGetUniqueId;
        CommInitAll = ks_fake_ncclCommInitAll;
        CommInitRank = ks_fake_ncclCommInitRank;
        CommDestroy = ks_fake_ncclCommDestroy;
        GroupStart = ks_fake_ncclGroupStart;
        GroupEnd = ks_fake_ncclGroupEnd;
        Send = ks_fake_ncclSend;
        Recv = ks_fake_ncclRecv;
        AllReduce = ks_fake_ncclAllReduce;
        GetErrorString = ks_fake_ncclGetErrorString;
        h = this;
        (void)err;
        return true;
#endif
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            err = std::string("RCCL not found: ") + dlerror();
            return false;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            ok = ok && fn;
        };
        sym(GetUniqueId, "ncclGetUniqueId");
        sym(CommInitAll, "ncclCommInitAll");
        sym(CommInitRank, "ncclCommInitRank");
        sym(CommDestroy, "ncclCommDestroy");
        sym(GroupStart, "ncclGroupStart");
        sym(GroupEnd, "ncclGroupEnd");
        sym(Send, "ncclSend");
        sym(Recv, "ncclRecv");
        sym(AllReduce, "ncclAllReduce");
        sym(GetErrorString, "ncclGetErrorString");
        if (!ok) err = "RCCL is missing a symbol";
        return ok;
    }
};

// RCCL, loaded on first use (the test build: the fake in-process ranks)
Rccl* comm_lib(std::string& err) {
    static Rccl r;
    return r.load(err) ? &r : nullptr;
}

// ---- row layout of ks_batch_gather (host code, shared by the packing, the
// unpacking and the CPU tests through the exported ks_batch_* layout calls) ----
// Graph g lives on global rank g mod world, as that rank's (g div world)-th
// graph. Every rank sends ONE block: [status word][slots rows], a row being
// [cost, flow value, PU id of each task (cell-local, 0 = unscheduled), padded to
// max_tasks]. Rank 0 receives the blocks in rank order.
inline size_t kb_slots(size_t ngraphs, int world) { return (ngraphs + (size_t)world - 1) / (size_t)std::max(1, world); }
inline size_t kb_rowlen(size_t max_tasks) { return 2 + max_tasks; }
inline size_t kb_block(size_t ngraphs, int world, size_t max_tasks) {
    return 1 + std::max<size_t>(1, kb_slots(ngraphs, world)) * kb_rowlen(max_tasks);
}
inline size_t kb_row_in_block(size_t slot, size_t max_tasks) { return 1 + slot * kb_rowlen(max_tasks); }

// row r: PU ids of its tasks made cell-local (subtract the cell's node offset)
__global__ void k_localize(int rows, int rowlen, const long long* __restrict__ off, long long* __restrict__ buf) {
    const int r = blockIdx.y;
    if (r >= rows) return;
    long long* row = buf + 1 + (size_t)r * rowlen;
    for (int i = 2 + blockIdx.x * blockDim.x + threadIdx.x; i < rowlen; i += gridDim.x * blockDim.x)
        if (row[i] > 0) row[i] -= off[r];
}

}  // namespace

struct ks_batch {
    struct Local {
        int device = 0;
        int grank = 0;                  // global rank
        ks_ctx* ctx = nullptr;
        ncclComm_t comm = nullptr;
        std::vector<int> graphs;        // graph ids solved here, in order
        std::vector<int64_t> off;       // node-id offset of each graph in the union (+ total)
        std::vector<int64_t> toff;      // task offset of each graph in the dense task vector (+ total)
        long long* rows = nullptr;      // device: graphs.size() × rowlen
        long long* scratch = nullptr;   // device: dense task→PU vector, offsets
        long long* stat = nullptr;      // device: this rank's status word for the status all-reduce
        size_t rows_cap = 0, scratch_cap = 0;
        ks_result res{};
    };
    std::vector<Local> loc;
    const Rccl* nccl = nullptr;         // the communication library behind this batch
    int world = 1;
    size_t ngraphs = 0;
    std::string err;
    long long* root_buf = nullptr;      // rank 0: world × slots × rowlen
    size_t root_cap = 0;
    int fault_pack = 0;                 // TESTS ONLY (ks_opts.fault_inject bit 2): global rank + 1 whose packing fails
    int fault_root = 0;                 // TESTS ONLY (ks_opts.fault_inject bit 3): rank 0's receive buffer allocation fails

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
};

namespace {

#define KB_HIP(expr)                                                          \
    do {                                                                      \
        hipError_t _e = (expr);                                               \
        if (_e != hipSuccess) return b->fail(KS_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

ks_batch* make_batch(const Rccl* api, int world, const ks_opts* opts, const std::vector<std::pair<int, int>>& dev_rank) {
    ks_batch* b = new (std::nothrow) ks_batch;
    if (!b) return nullptr;
    b->nccl = api;
    b->world = world;
    b->fault_pack = (opts && (opts->fault_inject & 4)) ? 1 : 0;   // TESTS ONLY: global rank 0's packing fails
    b->fault_root = (opts && (opts->fault_inject & 8)) ? 1 : 0;   // TESTS ONLY: rank 0's root buffer allocation fails
    for (auto [dev, rank] : dev_rank) {
        ks_batch::Local l;
        l.device = dev;
        l.grank = rank;
        l.ctx = ks_create(dev, opts);
        // the status word of the gather's all-reduce exists before any gather, so a
        // rank can always enter that collective
        if (!l.ctx || hipSetDevice(dev) != hipSuccess || hipMalloc(&l.stat, sizeof(long long)) != hipSuccess) {
            if (l.ctx) ks_destroy(l.ctx);
            for (auto& x : b->loc) {
                if (x.stat) (void)hipFree(x.stat);
                ks_destroy(x.ctx);
            }
            delete b;
            return nullptr;
        }
        b->loc.push_back(std::move(l));
    }
    return b;
}

}  // namespace

extern "C" {

size_t ks_batch_slots(size_t ngraphs, int world) { return world < 1 ? 0 : kb_slots(ngraphs, world); }

int ks_batch_owner(size_t g, int world, int* rank, size_t* slot) {
    if (world < 1 || !rank || !slot) return KS_E_INVALID;
    *rank = (int)(g % (size_t)world);
    *slot = g / (size_t)world;
    return KS_OK;
}

size_t ks_batch_block_len(size_t ngraphs, int world, size_t max_tasks) {
    return world < 1 ? 0 : kb_block(ngraphs, world, max_tasks);
}

int ks_batch_unpack(const int64_t* gathered, size_t ngraphs, int world, size_t max_tasks, uint64_t* pu,
                    int64_t* cost, int64_t* flow) {
    if (!gathered || world < 1) return KS_E_INVALID;
    const size_t block = kb_block(ngraphs, world, max_tasks);
    for (int r = 0; r < world; ++r)
        if (gathered[(size_t)r * block] != 0) return (int)gathered[(size_t)r * block];   // a rank's status
    for (size_t g = 0; g < ngraphs; ++g) {
        int r = 0;
        size_t slot = 0;
        ks_batch_owner(g, world, &r, &slot);
        const int64_t* row = gathered + (size_t)r * block + kb_row_in_block(slot, max_tasks);
        if (cost) cost[g] = row[0];
        if (flow) flow[g] = row[1];
        if (pu) std::memcpy(pu + g * max_tasks, row + 2, max_tasks * sizeof(uint64_t));
    }
    return KS_OK;
}

int ks_batch_unique_id(uint8_t* id) {
    std::string err;
    const Rccl* api = id ? comm_lib(err) : nullptr;
    if (!api) return KS_E_DEVICE;
    ncclUniqueId u;
    if (api->GetUniqueId(&u) != ncclSuccess) return KS_E_DEVICE;
    std::memcpy(id, u.internal, KS_UNIQUE_ID_BYTES);
    return KS_OK;
}

ks_batch* ks_batch_create(const int* devices, int ndev, const ks_opts* opts) {
    std::string err;
    const Rccl* api = devices && ndev >= 1 ? comm_lib(err) : nullptr;
    if (!api) return nullptr;
    std::vector<std::pair<int, int>> dr;
    for (int i = 0; i < ndev; ++i) dr.emplace_back(devices[i], i);
    ks_batch* b = make_batch(api, ndev, opts, dr);
    if (!b) return nullptr;
    std::vector<ncclComm_t> comms(ndev);
    if (api->CommInitAll(comms.data(), ndev, devices) != ncclSuccess) {
        ks_batch_destroy(b);
        return nullptr;
    }
    for (int i = 0; i < ndev; ++i) b->loc[i].comm = comms[i];
    return b;
}

ks_batch* ks_batch_create_rank(int device, int nranks, int rank, const uint8_t* id, const ks_opts* opts) {
    std::string err;
    const Rccl* api = id && nranks >= 1 && rank >= 0 && rank < nranks ? comm_lib(err) : nullptr;
    if (!api) return nullptr;
    ks_batch* b = make_batch(api, nranks, opts, {{device, rank}});
    if (!b) return nullptr;
    ncclUniqueId u;
    std::memcpy(u.internal, id, KS_UNIQUE_ID_BYTES);
    if (hipSetDevice(device) != hipSuccess || api->CommInitRank(&b->loc[0].comm, nranks, u, rank) != ncclSuccess) {
        ks_batch_destroy(b);
        return nullptr;
    }
    return b;
}

void ks_batch_destroy(ks_batch* b) {
    if (!b) return;
    for (auto& l : b->loc) {
        (void)hipSetDevice(l.device);
        if (l.comm) b->nccl->CommDestroy(l.comm);
        if (l.rows) (void)hipFree(l.rows);
        if (l.scratch) (void)hipFree(l.scratch);
        if (l.stat) (void)hipFree(l.stat);
        ks_destroy(l.ctx);
    }
    if (b->root_buf) {
        (void)hipSetDevice(b->loc[0].device);
        (void)hipFree(b->root_buf);
    }
    delete b;
}

const char* ks_batch_last_error(ks_batch* b) { return b ? b->err.c_str() : "null batch"; }

int ks_batch_load(ks_batch* b, size_t ngraphs, const ks_node* const* nodes, const size_t* n,
                  const ks_arc* const* arcs, const size_t* m) {
    if (!b) return KS_E_INVALID;
    if (ngraphs && (!nodes || !n || !arcs || !m)) return b->fail(KS_E_INVALID, "null graph arrays");
    b->ngraphs = ngraphs;
    for (auto& l : b->loc) {
        l.graphs.clear();
        for (size_t g = 0; g < ngraphs; ++g) {
            int r = 0;
            size_t slot = 0;
            ks_batch_owner(g, b->world, &r, &slot);
            if (r == l.grank) l.graphs.push_back((int)g);   // slot = its index in l.graphs
        }
        if (l.graphs.size() > 1024) return b->fail(KS_E_INVALID, "more than 1024 graphs on one device");
        // the disjoint union of this device's graphs: node ids offset per graph
        std::vector<ks_node> un;
        std::vector<ks_arc> ua;
        l.off.assign(1, 0);
        l.toff.assign(1, 0);
        for (int g : l.graphs) {
            uint64_t maxid = 0;
            int64_t tasks = 0;
            for (size_t i = 0; i < n[g]; ++i) {
                ks_node x = nodes[g][i];
                maxid = std::max<uint64_t>(maxid, x.id);
                tasks += x.type == KS_NODE_TASK;
                x.id += (uint64_t)l.off.back();
                un.push_back(x);
            }
            for (size_t i = 0; i < m[g]; ++i) {
                ks_arc a = arcs[g][i];
                // an arc must stay inside its own graph: past its max id it would land
                // on a node of the next graph in the union and couple two cells
                if (a.src == 0 || a.dst == 0 || a.src > maxid || a.dst > maxid)
                    return b->fail(KS_E_INVALID, "graph " + std::to_string(g) + ": arc " + std::to_string(a.src) +
                                                     "->" + std::to_string(a.dst) + " outside its node id range");
                a.src += (uint64_t)l.off.back();
                a.dst += (uint64_t)l.off.back();
                ua.push_back(a);
            }
            l.off.push_back(l.off.back() + (int64_t)maxid);
            l.toff.push_back(l.toff.back() + tasks);
        }
        const int rc = ks_load_graph(l.ctx, un.data(), un.size(), ua.data(), ua.size());
        if (rc) return b->fail(rc, ks_last_error(l.ctx));
        // the union's cells: the cell solver runs each in its own workgroup (ks_cell.h)
        l.ctx->eng.set_cells(l.off.data(), l.graphs.size());
    }
    return KS_OK;
}

int ks_batch_solve(ks_batch* b, ks_result* results) {
    if (!b) return KS_E_INVALID;
    std::vector<int> rcs(b->loc.size(), KS_OK);
    std::vector<std::thread> th;
    for (size_t i = 0; i < b->loc.size(); ++i)
        th.emplace_back([&, i]() { rcs[i] = ks_solve(b->loc[i].ctx, &b->loc[i].res); });
    for (auto& t : th) t.join();
    for (size_t i = 0; i < b->loc.size(); ++i) {
        if (results) results[i] = b->loc[i].res;
        if (rcs[i]) return b->fail(rcs[i], ks_last_error(b->loc[i].ctx));
    }
    return KS_OK;
}

int ks_batch_gather(ks_batch* b, size_t max_tasks, uint64_t* pu, int64_t* cost, int64_t* flow) {
    if (!b) return KS_E_INVALID;
    const size_t rowlen = kb_rowlen(max_tasks);
    const size_t block = kb_block(b->ngraphs, b->world, max_tasks);   // elements per rank
    bool has_root = false;
    int root_loc = -1;   // the local device of global rank 0 once its receive buffer is ready
    // 1. every device packs its block: [status][rows: cost, flow value, cell-local PU per task].
    //    A rank that fails here — a logical error or ANY HIP failure — still takes part
    //    in the collective below with its status word set, so its peers never wait for
    //    a send that is not posted (no early return before the status all-reduce).
    std::vector<int> status(b->loc.size(), KS_OK);
    std::string first_err;
    for (size_t li = 0; li < b->loc.size(); ++li) {
        auto& l = b->loc[li];
        ks_ctx* c = l.ctx;
        if (l.grank == 0) has_root = true;
        const size_t k = l.graphs.size();
        hipStream_t st = c->eng.stream();
        int rc = KS_OK;
        // a HIP failure: this rank's status, then on to the collective
#define KB_TRY(expr)                                                                          \
    do {                                                                                      \
        if (rc == KS_OK) {                                                                    \
            const hipError_t _e = (expr);                                                     \
            if (_e != hipSuccess) {                                                           \
                rc = KS_E_DEVICE;                                                             \
                c->err = std::string(#expr) + ": " + hipGetErrorString(_e);                   \
            }                                                                                 \
        }                                                                                     \
    } while (0)
        KB_TRY(hipSetDevice(l.device));
        if (b->fault_pack == (int)l.grank + 1) {   // TESTS ONLY: this rank's packing fails
            rc = KS_E_DEVICE;
            c->err = "injected pack failure";
        }
        if (rc == KS_OK && l.rows_cap < block) {
            if (l.rows) (void)hipFree(l.rows);
            l.rows = nullptr;
            l.rows_cap = 0;
            KB_TRY(hipMalloc(&l.rows, block * sizeof(long long)));
            if (rc == KS_OK) l.rows_cap = block;
        }
        KB_TRY(hipMemsetAsync(l.rows, 0, block * sizeof(long long), st));
        for (size_t i = 0; i < k && rc == KS_OK; ++i)
            if ((size_t)(l.toff[i + 1] - l.toff[i]) > max_tasks) {
                rc = KS_E_INVALID;
                c->err = "a graph has more tasks than max_tasks";
            }
        const size_t need = (size_t)l.toff.back() + 3 * (k + 1);
        if (rc == KS_OK && l.scratch_cap < need) {
            if (l.scratch) (void)hipFree(l.scratch);
            l.scratch = nullptr;
            l.scratch_cap = 0;
            KB_TRY(hipMalloc(&l.scratch, std::max<size_t>(need, 1) * sizeof(long long)));
            if (rc == KS_OK) l.scratch_cap = need;
        }
        if (rc == KS_OK && k) {
            long long* dcost = l.scratch + l.toff.back();
            long long* dflow = dcost + (k + 1);
            long long* doff = dflow + (k + 1);
            rc = c->eng.cell_sums(l.off.data(), k, (int64_t*)dcost, (int64_t*)dflow, c->err);
            size_t cnt = 0;
            if (rc == KS_OK) rc = ks_get_task_pu_device(c, (uint64_t*)l.scratch, (size_t)l.toff.back(), &cnt);
            long long* rows = l.rows + kb_row_in_block(0, max_tasks);
            KB_TRY(hipMemcpy2DAsync(rows, rowlen * sizeof(long long), dcost, sizeof(long long), sizeof(long long), k,
                                    hipMemcpyDeviceToDevice, st));
            KB_TRY(hipMemcpy2DAsync(rows + 1, rowlen * sizeof(long long), dflow, sizeof(long long), sizeof(long long),
                                    k, hipMemcpyDeviceToDevice, st));
            for (size_t i = 0; i < k; ++i) {
                const size_t t = (size_t)(l.toff[i + 1] - l.toff[i]);
                if (t)
                    KB_TRY(hipMemcpyAsync(l.rows + kb_row_in_block(i, max_tasks) + 2, l.scratch + l.toff[i],
                                          t * sizeof(long long), hipMemcpyDeviceToDevice, st));
            }
            KB_TRY(hipMemcpyAsync(doff, l.off.data(), k * sizeof(long long), hipMemcpyHostToDevice, st));
            if (rc == KS_OK)
                hipLaunchKernelGGL(k_localize, dim3(std::max<size_t>(1, std::min<size_t>(64, (rowlen + 255) / 256)), k),
                                   dim3(256), 0, st, (int)k, (int)rowlen, (const long long*)doff, l.rows);
            KB_TRY(hipGetLastError());
        }
        // rank 0 also holds the receive buffer of step 3: allocated (and its own block
        // copied in) here, so a failure is this rank's status word like any other and
        // nothing between the status all-reduce and the send/receive group can fail
        if (rc == KS_OK && l.grank == 0) {
            const size_t need = block * (size_t)b->world;
            if (b->fault_root) {   // TESTS ONLY: the root buffer's allocation fails
                rc = KS_E_DEVICE;
                c->err = "injected root buffer allocation failure";
            } else if (b->root_cap < need) {
                if (b->root_buf) (void)hipFree(b->root_buf);
                b->root_buf = nullptr;
                b->root_cap = 0;
                KB_TRY(hipMalloc(&b->root_buf, need * sizeof(long long)));
                if (rc == KS_OK) b->root_cap = need;
            }
            if (rc == KS_OK) root_loc = (int)li;
            KB_TRY(hipMemcpyAsync(b->root_buf, l.rows, block * sizeof(long long), hipMemcpyDeviceToDevice, st));
        }
        // always drain the stream, also after a failure: the memset, the copies and
        // k_localize must be finished before the status word is written or we return
        {
            const hipError_t se = hipStreamSynchronize(st);
            if (se != hipSuccess && rc == KS_OK) {
                rc = KS_E_DEVICE;
                c->err = std::string("hipStreamSynchronize: ") + hipGetErrorString(se);
            }
        }
        if (rc != KS_OK) {
            status[li] = rc;
            if (first_err.empty()) first_err = "rank " + std::to_string(l.grank) + ": " + c->err;
            // the status word goes out in the block when the rows buffer exists
            // (written on the engine's stream, which the rows' producers used)
            if (l.rows) {
                const long long sw = rc;
                if (hipMemcpyAsync(l.rows, &sw, sizeof(long long), hipMemcpyHostToDevice, st) == hipSuccess)
                    (void)hipStreamSynchronize(st);
            }
        }
#undef KB_TRY
    }
    // 2. every rank learns whether any rank failed (min over the status words), so
    //    all of them return the same error instead of only the failing one
    if (b->world > 1) {
        for (size_t li = 0; li < b->loc.size(); ++li) {
            auto& l = b->loc[li];
            const long long sw = status[li];
            // (a failure to post the word is itself this rank's failure; it still enters)
            if ((hipSetDevice(l.device) != hipSuccess ||
                 hipMemcpy(l.stat, &sw, sizeof(long long), hipMemcpyHostToDevice) != hipSuccess) &&
                status[li] == KS_OK) {
                status[li] = KS_E_DEVICE;
                if (first_err.empty()) first_err = "rank " + std::to_string(l.grank) + ": status word not posted";
            }
        }
        {   // (the group is always closed: an RCCL error is returned after GroupEnd)
            ncclResult_t nr = b->nccl->GroupStart();
            for (auto& l : b->loc) {
                const ncclResult_t x = b->nccl->AllReduce(l.stat, l.stat, 1, ncclInt64, ncclMin, l.comm, l.ctx->eng.stream());
                if (nr == ncclSuccess) nr = x;
            }
            const ncclResult_t ge = b->nccl->GroupEnd();
            if (nr == ncclSuccess) nr = ge;
            if (nr != ncclSuccess) return b->fail(KS_E_DEVICE, std::string("status all-reduce: ") + b->nccl->GetErrorString(nr));
        }
        long long worst = 0;
        for (size_t li = 0; li < b->loc.size(); ++li) {
            auto& l = b->loc[li];
            long long sw = 0;
            if (hipSetDevice(l.device) != hipSuccess || hipStreamSynchronize(l.ctx->eng.stream()) != hipSuccess ||
                hipMemcpy(&sw, l.stat, sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
                sw = KS_E_DEVICE;
            worst = std::min<long long>(worst, std::min<long long>(sw, status[li]));
        }
        if (worst != 0)
            return b->fail((int)worst, first_err.empty() ? "another rank failed to pack its rows (status " +
                                                               std::to_string(worst) + ")"
                                                         : first_err);
    }
    // world 1: this process's own failure ends it here (no peer waits)
    for (int rc : status)
        if (rc != KS_OK) return b->fail(rc, first_err);
    // 3. one group: every rank's block to global rank 0. Nothing between the status
    //    all-reduce and GroupEnd returns early: an RCCL error is remembered and
    //    returned after the group, so no peer is left waiting in a send.
    long long* rbuf = root_loc >= 0 ? b->root_buf : nullptr;
    if (b->world > 1) {
        ncclResult_t nr = b->nccl->GroupStart();
        for (auto& l : b->loc) {
            hipStream_t st = l.ctx->eng.stream();
            if (l.grank == 0) {
                for (int r = 1; r < b->world; ++r) {
                    const ncclResult_t x = b->nccl->Recv(rbuf + (size_t)r * block, block, ncclInt64, r, l.comm, st);
                    if (nr == ncclSuccess) nr = x;
                }
            } else {
                const ncclResult_t x = b->nccl->Send(l.rows, block, ncclInt64, 0, l.comm, st);
                if (nr == ncclSuccess) nr = x;
            }
        }
        const ncclResult_t ge = b->nccl->GroupEnd();
        if (nr == ncclSuccess) nr = ge;
        if (nr != ncclSuccess) return b->fail(KS_E_DEVICE, std::string("ncclSend/ncclRecv group: ") + b->nccl->GetErrorString(nr));
    }
    for (auto& l : b->loc) {
        KB_HIP(hipSetDevice(l.device));
        KB_HIP(hipStreamSynchronize(l.ctx->eng.stream()));
    }
    for (int rc : status)
        if (rc != KS_OK) return b->fail(rc, first_err);   // this process's own failure, after the collective
    if (!has_root) return KS_OK;
    // 4. rank 0: every rank's status word, then the rows back in graph order
    std::vector<long long> host(block * (size_t)b->world);
    for (auto& l : b->loc)
        if (l.grank == 0) {
            KB_HIP(hipSetDevice(l.device));
            KB_HIP(hipMemcpy(host.data(), rbuf, host.size() * sizeof(long long), hipMemcpyDeviceToHost));
        }
    const int rc = ks_batch_unpack((const int64_t*)host.data(), b->ngraphs, b->world, max_tasks, pu, cost, flow);
    if (rc != KS_OK) return b->fail(rc, "a rank failed to pack its rows (status " + std::to_string(rc) + ")");
    return KS_OK;
}

}  // extern "C"
