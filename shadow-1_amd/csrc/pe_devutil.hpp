// pe_devutil.hpp -- device helpers shared by the sparse, batched and exact
// kernels (bit views of positive doubles, address-space casts).
#pragma once
#include <hip/hip_runtime.h>

#include "pe_device.hpp"

namespace shdpe {

// +inf as a u64 bit pattern: positive doubles order like their bit patterns,
// so an integer min on the pattern is an exact f64 min.
constexpr unsigned long long INF_BITS = 0x7FF0000000000000ull;

__device__ __forceinline__ double b2d(unsigned long long b) {
    return __longlong_as_double((long long)b);
}
__device__ __forceinline__ unsigned long long d2b(double d) {
    return (unsigned long long)__double_as_longlong(d);
}

// Pointers that arrive inside by-value structs lose their address space and
// would be accessed with flat_* instructions (which also make every wait a
// combined vmcnt+lgkmcnt wait).  Round-tripping them through address space 1
// lets the compiler emit global_* loads/stores/atomics.
template <class T>
__device__ __forceinline__ T* as_global(T* p) {
    return (T*)((__attribute__((address_space(1))) T*)p);
}

__device__ __forceinline__ DevGraph global_view(const DevGraph& g0) {
    DevGraph g = g0;
    g.rowPtr = as_global(g0.rowPtr);
    g.col = as_global(g0.col);
    g.arcs = as_global(g0.arcs);
    g.arc3 = as_global(g0.arc3);
    g.lat = as_global(g0.lat);
    g.rel = as_global(g0.rel);
    g.inPtr = as_global(g0.inPtr);
    g.inCol = as_global(g0.inCol);
    g.inLat = as_global(g0.inLat);
    g.inRel = as_global(g0.inRel);
    g.outToIn = as_global(g0.outToIn);
    g.vrel = as_global(g0.vrel);
    g.selfLat = as_global(g0.selfLat);
    g.selfRel = as_global(g0.selfRel);
    g.hasSelf = as_global(g0.hasSelf);
    g.selfMinLat = as_global(g0.selfMinLat);
    g.selfMinRel = as_global(g0.selfMinRel);
    g.attached = as_global(g0.attached);
    g.isAttached = as_global(g0.isAttached);
    g.heavyBits = as_global(g0.heavyBits);
    g.oldId = g0.oldId ? as_global(g0.oldId) : nullptr;
    return g;
}

__device__ __forceinline__ DevTable global_view(const DevTable& t0) {
    DevTable t = t0;
    t.lat = as_global(t0.lat);
    t.rel = as_global(t0.rel);
    t.hops = as_global(t0.hops);
    t.pred = t0.pred ? as_global(t0.pred) : nullptr;
    t.flags = as_global(t0.flags);
    return t;
}

__device__ __forceinline__ DevScratch global_view(const DevScratch& s0) {
    DevScratch s = s0;
    s.dist = as_global(s0.dist);
    s.hops = as_global(s0.hops);
    s.rel = as_global(s0.rel);
    s.pred = as_global(s0.pred);
    s.heapTail = as_global(s0.heapTail);
    s.index2 = as_global(s0.index2);
    s.queue = as_global(s0.queue);
    return s;
}

// Loads of data that other waves of the SAME workgroup update (atomics or
// stores).  A workgroup runs on one CU, so workgroup scope is the coherence
// level needed.  Never use agent scope for this on gfx950: agent-scope loads
// carry sc1 (they miss the XCD's L2) and agent-scope fences write back and
// invalidate the whole L2 (buffer_wbl2 / buffer_inv sc1).
template <class T>
__device__ __forceinline__ T ld_wg(T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void fence_wg() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

}  // namespace shdpe
