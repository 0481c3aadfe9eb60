// block_solve.h -- the per-wave 32-node block solve shared by the apply
// kernels (k_apply.hip) and the sharded apply (k_shard.hip).  Layout of the
// packed inverse: layout.h.
#pragma once

#include "layout.h"
#include "mas_internal.h"

namespace mas {

constexpr int kApplyThreads = 256;  // 4 waves = 4 blocks per workgroup

// One rotation step: out += G r_src, and lane dst receives G^T r_own.
__device__ __forceinline__ void pair_step(float3& out, const float (&G)[9], float3 r, int src, int dst) {
    const float mx = __shfl(r.x, src), my = __shfl(r.y, src), mz = __shfl(r.z, src);
    out.x = __fmaf_rn(G[2], mz, __fmaf_rn(G[1], my, __fmaf_rn(G[0], mx, out.x)));
    out.y = __fmaf_rn(G[5], mz, __fmaf_rn(G[4], my, __fmaf_rn(G[3], mx, out.y)));
    out.z = __fmaf_rn(G[8], mz, __fmaf_rn(G[7], my, __fmaf_rn(G[6], mx, out.z)));
    const float cx = __fmaf_rn(G[6], r.z, __fmaf_rn(G[3], r.y, __fmul_rn(G[0], r.x)));
    const float cy = __fmaf_rn(G[7], r.z, __fmaf_rn(G[4], r.y, __fmul_rn(G[1], r.x)));
    const float cz = __fmaf_rn(G[8], r.z, __fmaf_rn(G[5], r.y, __fmul_rn(G[2], r.x)));
    out.x = __fadd_rn(out.x, __shfl(cx, dst));
    out.y = __fadd_rn(out.y, __shfl(cy, dst));
    out.z = __fadd_rn(out.z, __shfl(cz, dst));
}

// out = Inv_b r for the node this lane owns (layout.h).  g: the lane's
// 72-float record, tl: its tail row (half 0, lanes 0..15; zero elsewhere).
// Both halves return the same, complete result.
__device__ __forceinline__ float3 block_solve(const float (&g)[kRecord], const float (&tl)[3], float3 r, int lane) {
    const int n = lane & 31, hb = lane & 32;
    const bool h1 = hb != 0;
    float3 out;
    {  // D(n) r, half 0 only
        const float ox = __fmaf_rn(g[68], r.z, __fmaf_rn(g[67], r.y, __fmul_rn(g[66], r.x)));
        const float oy = __fmaf_rn(g[70], r.z, __fmaf_rn(g[69], r.y, __fmul_rn(g[67], r.x)));
        const float oz = __fmaf_rn(g[71], r.z, __fmaf_rn(g[70], r.y, __fmul_rn(g[68], r.x)));
        out = h1 ? make_float3(0.f, 0.f, 0.f) : make_float3(ox, oy, oz);
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const int s = h1 ? 8 + k : 1 + k;
        float G[9];
#pragma unroll
        for (int e = 0; e < 9; ++e) G[e] = g[9 * k + e];
        pair_step(out, G, r, hb | ((n + s) & 31), hb | ((n - s) & 31));
    }
    {  // k = 7: half 1 regular s = 15; half 0 the s = 16 pair (p, p+16) as a
       // rotation step with a per-lane 3x3: lane p = [row0; 0; row2],
       // lane p+16 = row1 in column 1 (so it adds r_p.y row1 and returns row1.r).
        const bool lo = n < 16;
        const float w0 = g[63], w1 = g[64], w2 = g[65];
        float G[9];
        if (h1) {
#pragma unroll
            for (int e = 0; e < 9; ++e) G[e] = g[63 + e];
        } else {
            G[0] = lo ? w0 : 0.f;  G[1] = lo ? w1 : w0;   G[2] = lo ? w2 : 0.f;
            G[3] = 0.f;            G[4] = lo ? 0.f : w1;  G[5] = 0.f;
            G[6] = lo ? tl[0] : 0.f; G[7] = lo ? tl[1] : w2; G[8] = lo ? tl[2] : 0.f;
        }
        const int s = h1 ? 15 : 16;
        pair_step(out, G, r, hb | ((n + s) & 31), hb | ((n - s) & 31));
    }
    // combine the halves (commutative add: both halves hold the same sum)
    const int other = lane ^ 32;
    out.x = __fadd_rn(out.x, __shfl(out.x, other));
    out.y = __fadd_rn(out.y, __shfl(out.y, other));
    out.z = __fadd_rn(out.z, __shfl(out.z, other));
    return out;
}

template <bool NT = false>
__device__ __forceinline__ void load_record(const float4* __restrict__ inv, int blk, int lane, float (&g)[kRecord],
                                            float (&tl)[3]) {
    const float4* b = inv + (size_t)blk * kBlockF4 + lane;
#pragma unroll
    for (int q = 0; q < kRecord / 4; ++q) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f* bp = reinterpret_cast<const v4f*>(b + q * 64);
        const v4f x = NT ? __builtin_nontemporal_load(bp) : *bp;
        g[4 * q + 0] = x.x;
        g[4 * q + 1] = x.y;
        g[4 * q + 2] = x.z;
        g[4 * q + 3] = x.w;
    }
    const float* t = reinterpret_cast<const float*>(inv + (size_t)blk * kBlockF4) + kMainFloats + 3 * (lane & 15);
    tl[0] = t[0];
    tl[1] = t[1];
    tl[2] = t[2];
    if (lane >= 16) tl[0] = tl[1] = tl[2] = 0.f;
}

}  // namespace mas
