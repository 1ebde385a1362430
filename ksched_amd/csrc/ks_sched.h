// ks_sched.h — scheduler-side device sweeps of a round (ks_sched.hip), internal.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/ksmcmf.h"
#include "ks_pos.h"

namespace ks {

// Raw pointers the scheduler sweeps read or edit (a view of the engine's store).
struct SchedDev {
    int ncap;                      // node slots covered by the build (ids 1..ncap)
    long long nstore;              // allocated node slots
    const int* perm;               // slot → internal id
    const int* iperm;              // internal id → slot (−1 = padding)
    const unsigned char* n_alive;
    const unsigned char* n_type;
    unsigned long long* n_bind;    // per task slot: bound PU node id, 0 = none (TaskBindings)
    int hi;                        // arc slots handed out
    const unsigned char* a_alive;
    const unsigned char* a_type;
    const int* a_src;
    const int* a_dst;
    long long* a_cost;
    const int* fwd;
    const int* first;              // residual CSR (internal ids)
    Pos* pos;                      // residual positions (ks_pos.h)
    const int* ent;
    long long mult;
    int csr_valid;
};

hipError_t sched_delta_kinds(const SchedDev& d, const int* is_task, const int* rank, const unsigned long long* newpu,
                             int* pre, int* other, int* bad, hipStream_t st);
hipError_t sched_delta_emit(const SchedDev& d, const int* rank, const unsigned long long* newpu, const int* pre,
                            const int* pre_pos, const int* other, const int* other_pos, int npre, ks_sched_delta* out,
                            int commit, hipStream_t st);
hipError_t sched_running_counts(const SchedDev& d, const unsigned long long* ids, const unsigned long long* vals,
                                int k, unsigned long long* cnt, hipStream_t st);
hipError_t sched_topo_level(const SchedDev& d, const int* front, int nfront, int level, int* lvl, int* next,
                            int* nnext, unsigned long long mtpp, const unsigned long long* pu_running,
                            unsigned long long* slots, unsigned long long* running, hipStream_t st);
hipError_t sched_unsched_costs(const SchedDev& d, const unsigned long long* ids, int k, unsigned char* flags, int mode,
                               long long ucost, long long ccost, int* changed, hipStream_t st);

}  // namespace ks
