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

// The multi-kernel engine's 16-byte copy of a position for the solve's hot kernels
// (sweeps, Bellman-Ford rounds, walks, forward searches). Packed
// from Pos before the phases when every scaled cost and capacity fits 32 bits, its
// residual written back before verification. The reverse position lives in a
// separate int array: only a push needs it (a Bellman-Ford relaxation reads one
// 16-B record, and a task's eight records are one 128-B line instead of two).
struct alignas(16) CPos {
    int rcap;         // residual capacity
    int ucap;         // pair capacity
    int cost;         // scaled cost; CPOS_DEAD for an inert position (never residual)
    int head;         // internal id of the head
};
static_assert(sizeof(CPos) == 16, "a compact position is one 16-byte record");
constexpr int CPOS_DEAD = 0x7fffffff;          // > every ε a compact solve uses (ε ≤ max|scaled cost|)
constexpr long long CPOS_MAX = 0x7ffffffeLL;   // largest |scaled cost| / capacity a compact record holds

}  // namespace ks
