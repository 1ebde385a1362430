// ks_pos.h — one residual position of the device CSR (internal to libksmcmf).
//
// Every field a sweep, a Bellman-Ford relaxation or a walk reads about one
// residual arc sits in one 32-byte record (two 16-B loads, issued together),
// instead of five arrays (five loads from five cache lines): the arc's scaled
// cost, its residual capacity, the pair capacity ucap = rcap + rcap(rev)
// (constant per pair, so the reverse residual is ucap − rcap without a gather),
// the head and the reverse position. A push still writes only the two rcap
// fields (8-B stores).
#pragma once

namespace ks {

struct alignas(32) Pos {
    long long cost;   // scaled cost: +c·(n+1) forward, −c·(n+1) reverse, DEAD_COST when inert
    long long rcap;   // residual capacity
    long long ucap;   // pair capacity rcap(a) + rcap(rev a)
    int head;         // internal id of the head (inert: the owner)
    int rev;          // position of the reverse arc (inert: itself)
};
static_assert(sizeof(Pos) == 32, "a residual position is one 32-byte record");

}  // namespace ks
