// fake_nccl.cpp — TEST INFRASTRUCTURE: RCCL's entry points for the ranks of ONE
// process, so ks_batch_gather's world > 1 path (its status all-reduce, the
// send/receive group, the status protocol under fault_inject bits 2 and 3) runs on
// a one-GPU box. It is compiled only into the TEST build of
// the library, libksmcmf_fakecomm.so (-DKS_FAKE_COMM, ksched_amd/_build.py
// build_fake_comm), whose ks_batch.hip binds its communication calls to these
// ks_fake_nccl* functions instead of RCCL; the shipped libksmcmf.so never contains
// them and loads nothing but RCCL.
//
// ncclCommInitAll(comms, n, devs) makes n ranks of one clique (devices may repeat).
// Operations are queued between ncclGroupStart and ncclGroupEnd and run at the
// outermost GroupEnd, where the protocol is CHECKED, not assumed:
//   - an all-reduce runs only when every rank of its clique posted one in the group,
//     with the same count and type (int64, min or sum) — otherwise
//     ncclInvalidUsage, which is what a rank that skipped the collective would turn
//     into on real RCCL: a hang;
//   - every ncclRecv(peer p) of rank r needs an ncclSend(peer r) of rank p with the
//     same count, matched in posting order, and every send a receive.
// Data moves with device copies: the sender's stream is drained, then the copy is
// enqueued on the receiver's stream (so the receiver's later work sees it).
// ks_fake_nccl_stats() reports what ran, so a test can tell this library was used.
//
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

struct Clique {
    int n = 0;
    int refs = 0;
};

struct ncclComm {
    Clique* q;
    int rank;
    int dev;
};

namespace {

enum Kind { OP_ALLREDUCE, OP_SEND, OP_RECV };

struct Op {
    Kind kind;
    ncclComm* c;
    const void* sb;
    void* rb;
    size_t count;
    ncclDataType_t dt;
    ncclRedOp_t red;
    int peer;
    hipStream_t st;
};

std::mutex g_mu;
std::vector<Op> g_ops;
int g_depth = 0;
long long g_stats[4] = {0, 0, 0, 0};   // all-reduces, sends, receives, groups run

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt64:
        case ncclUint64:
        case ncclFloat64: return 8;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32: return 4;
        default: return 0;
    }
}

ncclResult_t run_allreduces(std::vector<Op>& ops) {
    std::vector<bool> done(ops.size(), false);
    for (size_t i = 0; i < ops.size(); ++i) {
        if (ops[i].kind != OP_ALLREDUCE || done[i]) continue;
        Clique* q = ops[i].c->q;
        std::vector<size_t> mine;   // one op per rank of this clique
        for (size_t j = i; j < ops.size(); ++j)
            if (ops[j].kind == OP_ALLREDUCE && !done[j] && ops[j].c->q == q) mine.push_back(j);
        if ((int)mine.size() != q->n) return ncclInvalidUsage;   // a rank did not enter the collective
        std::vector<bool> seen(q->n, false);
        for (size_t j : mine) {
            const Op& o = ops[j];
            if (seen[o.c->rank] || o.count != ops[i].count || o.dt != ncclInt64 ||
                (o.red != ncclMin && o.red != ncclSum))
                return ncclInvalidUsage;
            seen[o.c->rank] = true;
        }
        std::vector<long long> acc(ops[i].count), buf(ops[i].count);
        bool first = true;
        for (size_t j : mine) {
            const Op& o = ops[j];
            if (hipSetDevice(o.c->dev) != hipSuccess || hipStreamSynchronize(o.st) != hipSuccess ||
                hipMemcpy(buf.data(), o.sb, o.count * 8, hipMemcpyDeviceToHost) != hipSuccess)
                return ncclUnhandledCudaError;
            for (size_t k = 0; k < o.count; ++k)
                acc[k] = first ? buf[k] : (o.red == ncclMin ? std::min(acc[k], buf[k]) : acc[k] + buf[k]);
            first = false;
        }
        for (size_t j : mine) {
            const Op& o = ops[j];
            if (hipSetDevice(o.c->dev) != hipSuccess ||
                hipMemcpyAsync(o.rb, acc.data(), o.count * 8, hipMemcpyHostToDevice, o.st) != hipSuccess ||
                hipStreamSynchronize(o.st) != hipSuccess)
                return ncclUnhandledCudaError;
            done[j] = true;
        }
        ++g_stats[0];
    }
    return ncclSuccess;
}

ncclResult_t run_p2p(std::vector<Op>& ops) {
    std::vector<bool> used(ops.size(), false);
    for (size_t i = 0; i < ops.size(); ++i) {
        if (ops[i].kind != OP_RECV) continue;
        const Op& r = ops[i];
        size_t s = ops.size();
        for (size_t j = 0; j < ops.size(); ++j)
            if (ops[j].kind == OP_SEND && !used[j] && ops[j].c->q == r.c->q && ops[j].c->rank == r.peer &&
                ops[j].peer == r.c->rank) {
                s = j;
                break;
            }
        if (s == ops.size() || ops[s].count != r.count || ops[s].dt != r.dt) return ncclInvalidUsage;
        used[s] = true;
        const Op& x = ops[s];
        const size_t bytes = r.count * type_size(r.dt);
        if (hipSetDevice(x.c->dev) != hipSuccess || hipStreamSynchronize(x.st) != hipSuccess ||
            hipSetDevice(r.c->dev) != hipSuccess ||
            hipMemcpyAsync(r.rb, x.sb, bytes, hipMemcpyDeviceToDevice, r.st) != hipSuccess)
            return ncclUnhandledCudaError;
        ++g_stats[1];
        ++g_stats[2];
    }
    for (size_t j = 0; j < ops.size(); ++j)
        if (ops[j].kind == OP_SEND && !used[j]) return ncclInvalidUsage;   // a send nobody receives
    return ncclSuccess;
}

ncclResult_t post(const Op& o) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_depth == 0) return ncclInvalidUsage;   // only grouped operations (ks_batch always groups)
    if (!o.c || !o.c->q || type_size(o.dt) == 0) return ncclInvalidArgument;
    g_ops.push_back(o);
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ks_fake_ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof(id->internal));
    return ncclSuccess;
}

ncclResult_t ks_fake_ncclCommInitAll(ncclComm_t* comms, int n, const int* devs) {
    if (!comms || n < 1 || !devs) return ncclInvalidArgument;
    Clique* q = new Clique;
    q->n = n;
    q->refs = n;
    for (int i = 0; i < n; ++i) comms[i] = new ncclComm{q, i, devs[i]};
    return ncclSuccess;
}

// one process holds every rank here: a per-process rank of a larger world has no peers
ncclResult_t ks_fake_ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
    if (!comm || nranks != 1 || rank != 0) return ncclInvalidUsage;
    int dev = 0;
    (void)hipGetDevice(&dev);
    Clique* q = new Clique;
    q->n = 1;
    q->refs = 1;
    *comm = new ncclComm{q, 0, dev};
    return ncclSuccess;
}

ncclResult_t ks_fake_ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    if (--c->q->refs == 0) delete c->q;
    delete c;
    return ncclSuccess;
}

ncclResult_t ks_fake_ncclGroupStart() {
    std::lock_guard<std::mutex> lk(g_mu);
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ks_fake_ncclGroupEnd() {
    std::vector<Op> ops;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_depth == 0) return ncclInvalidUsage;
        if (--g_depth > 0) return ncclSuccess;
        ops.swap(g_ops);
        ++g_stats[3];
    }
    ncclResult_t r = run_allreduces(ops);
    if (r == ncclSuccess) r = run_p2p(ops);
    return r;
}

ncclResult_t ks_fake_ncclAllReduce(const void* sb, void* rb, size_t count, ncclDataType_t dt, ncclRedOp_t op, ncclComm_t c,
                           hipStream_t st) {
    return post(Op{OP_ALLREDUCE, c, sb, rb, count, dt, op, -1, st});
}

ncclResult_t ks_fake_ncclSend(const void* sb, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t st) {
    return post(Op{OP_SEND, c, sb, nullptr, count, dt, ncclSum, peer, st});
}

ncclResult_t ks_fake_ncclRecv(void* rb, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t st) {
    return post(Op{OP_RECV, c, nullptr, rb, count, dt, ncclSum, peer, st});
}

const char* ks_fake_ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake_nccl)";
        case ncclInvalidUsage: return "invalid usage: a rank skipped a collective or a send/recv is unmatched (fake_nccl)";
        case ncclInvalidArgument: return "invalid argument (fake_nccl)";
        case ncclUnhandledCudaError: return "HIP error (fake_nccl)";
        default: return "error (fake_nccl)";
    }
}

// [all-reduces run, sends, receives, groups closed]
void ks_fake_nccl_stats(long long* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < 4; ++i) out[i] = g_stats[i];
}

}  // extern "C"
