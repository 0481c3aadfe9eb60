// deep_fold.h -- the level-3 residual fold in the reference's order, shared by
// the two-launch coarse path (k_coarse.hip) and the sharded apply
// (k_shard.hip).  See k_coarse.hip's header for the algorithm.
#pragma once

#include "block_solve.h"

#ifndef MAS_STAMP
#define MAS_STAMP(kern, wave, k) \
    do {                         \
    } while (0)
#endif

namespace mas {

// write-through hand-off of a float4 (agent-scope relaxed atomic stores: sc1,
// no L2 writeback fence), drained before the arrival counter moves; the
// consumer reads it with sc1 loads (no invalidate fence).
//
// This is a HARDWARE protocol for gfx942/gfx950, not a C++/HIP memory-model
// guarantee: in the model, relaxed atomics to different locations give no
// happens-before edge between producer and consumer.  It rests on these rows
// of LLVM's AMDGPU memory model for GFX942 (AMDGPUUsage, "Memory Model GFX942",
// which gfx950 shares):
//   * store atomic monotonic, agent scope  -> global_store ... sc1: written
//     through the (per-XCD, non-coherent) L2 to memory-side coherence;
//   * load atomic monotonic, agent scope   -> global_load ... sc1: misses the
//     local L2 for that line, reads the coherent copy;
//   * atomicrmw monotonic, agent scope     -> global_atomic ... sc1, performed
//     at memory-side coherence.
// The producer issues its sc1 stores, waits for their completion
// (s_waitcnt vmcnt(0): the write-through acknowledgements), and only then
// issues the counter RMW; the consumer issues its sc1 loads only after that
// RMW has returned the count that makes it the last arriver.  Every datum
// involved is written and read with sc1, so no L2 copy of it is ever
// consulted, and the waitcnt orders completion before the count.  The
// formal alternative -- release fetch_add + acquire fence (buffer_wbl2 sc1 /
// buffer_inv sc1 on the whole L2) -- measured 4.8 us per hand-off here.
// Regression test with 18 level-3 blocks spread over every XCD:
// tests/test_gpu_restrict.py::test_level3_handoff_across_xcds_4m_tet.
__device__ __forceinline__ void st_wt(float4* p, float4 v) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, __builtin_bit_cast(unsigned long long, make_float2(v.x, v.y)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __builtin_bit_cast(unsigned long long, make_float2(v.z, v.w)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld_wt(const float4* p) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const float2 a = __builtin_bit_cast(float2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const float2 b =
        __builtin_bit_cast(float2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return make_float4(a.x, a.y, b.x, b.y);
}

// Left fold of n4 float4 (4 n4 floats, n4 a multiple of B) of one LDS row into
// acc, in order, B float4 per batch: the batch's B reads issue together and the
// adds wait for them one by one, so one LDS latency is exposed per 4 B adds
// (scripts/dev/fold_rate.hip: cycles per add for B = 8 / 16 / 32).
template <int B = 8>
__device__ __forceinline__ float fold_row(const float4* __restrict__ row, int n4, float acc) {
    for (int k0 = 0; k0 < n4; k0 += B) {
        float4 c[B];
#pragma unroll
        for (int k = 0; k < B; ++k) c[k] = row[k0 + k];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            acc = __fadd_rn(acc, c[k].x);
            acc = __fadd_rn(acc, c[k].y);
            acc = __fadd_rn(acc, c[k].z);
            acc = __fadd_rn(acc, c[k].w);
        }
    }
    return acc;
}

constexpr int kDeepChunk = 2048;  // list entries staged per step (8 per thread): one step at 1M

// R3 of node `node` folded from R1 (see the header), published; the block's
// last arriving node solves the block.  The whole workgroup (kApplyThreads)
// runs it.  List p of node T: T * stride + i.  INDEXED (the per-level form and
// the sharded apply): d.src[d.idx[p]] (-1: padding); else d.src[p] (deepR1).
template <bool INDEXED, bool PREFETCH = true, int THREADS = kApplyThreads>
__device__ __forceinline__ void deep_node(const float4* __restrict__ inv, int node, const DeepArgs& d,
                                          float4* __restrict__ rc, float4* __restrict__ zc, int begin1) {
    __shared__ __attribute__((aligned(16))) float st[3][kDeepChunk];  // b128 reads: 16-byte aligned rows
    __shared__ int last;
    constexpr int kPer = kDeepChunk / THREADS;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int T = node - d.lv3Begin, blk = node >> 5;
    [[maybe_unused]] const int pw = blockIdx.x * 4 + w;  // probe slot (k_solve123 grid order)
    MAS_STAMP(1, pw, 0);
    const size_t base = (size_t)T * d.stride;
    const int len = d.stride;
    float g[kRecord], tl[3];
    float4 v[kPer];
    auto load = [&](int b) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int i = b + t + THREADS * q;
            v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < len) {
                if (INDEXED) {
                    const int k = d.idx[base + i];
                    if (k >= 0) v[q] = d.src[k];
                } else {
                    v[q] = d.src[base + i];
                }
            }
        }
    };
    load(0);
#ifdef MAS_PROBE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic only: when the list has landed
    MAS_STAMP(1, pw, 5);
#endif
    float acc = 0.f;
    if (w == 0) __builtin_amdgcn_s_setprio(3);  // the fold is the launch's longest chain
    for (int b0 = 0; b0 < len; b0 += kDeepChunk) {
        if (b0 > 0) __syncthreads();  // the previous step's fold is done with st
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int i = t + THREADS * q;
            st[0][i] = v[q].x;
            st[1][i] = v[q].y;
            st[2][i] = v[q].z;
        }
        __syncthreads();
        if (b0 == 0) MAS_STAMP(1, pw, 1);
        // in case this node arrives last: the block's inverse, issued once the
        // list is staged and in flight during the fold (issued with the list
        // loads, the staging waits held the barrier: pre-fine 19.3 -> 18.4 us)
        if (PREFETCH && b0 == 0 && w == 1) load_record<true>(inv, blk, lane, g, tl);
        if (b0 + kDeepChunk < len) load(b0 + kDeepChunk);  // in flight during the fold
        if (t < 3) {
            // cnt is a multiple of 32 (stride): whole 8-float4 batches
            const int n4 = min(kDeepChunk, len - b0) / 4;
            acc = fold_row(reinterpret_cast<const float4*>(st[t]), n4, acc);
        }
    }
    MAS_STAMP(1, pw, 2);
    if (w == 0) {
        __builtin_amdgcn_s_setprio(0);
        const float ax = __shfl(acc, 0), ay = __shfl(acc, 1), az = __shfl(acc, 2);
        if (t == 0) {
            // publish R (write-through, drained), then count the arrival; the
            // block's last node reads the others' R with sc1 loads.  (An
            // acq_rel atomic instead -- an L2 writeback + invalidate -- took
            // 4.8 us here.)
            st_wt(rc + node - begin1, make_float4(ax, ay, az, 0.f));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int old = __hip_atomic_fetch_add(d.cnt + (blk - d.lv3Begin / 32), 1, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            last = old == 31;
        }
    }
    __syncthreads();
    MAS_STAMP(1, pw, 3);
    if (!last || w != 1) return;
    if (lane == 0) d.cnt[blk - d.lv3Begin / 32] = 0;  // for the next apply (visible after this kernel)
    if (!PREFETCH) load_record<true>(inv, blk, lane, g, tl);
    const int n = lane & 31;
    const float4 R = ld_wt(rc + blk * 32 + n - begin1);
    const float3 out = block_solve(g, tl, make_float3(R.x, R.y, R.z), lane);
    MAS_STAMP(1, pw, 4);
    if (lane < 32) zc[blk * 32 + n - begin1] = make_float4(out.x, out.y, out.z, 0.f);
}

}  // namespace mas
