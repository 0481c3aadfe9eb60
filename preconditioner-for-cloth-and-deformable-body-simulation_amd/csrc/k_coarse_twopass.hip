// k_coarse_twopass.hip -- the coarse levels of one Preconditioning
// (.cpp:1548-1696) in two launches instead of one per level (L >= 3).
//
// The per-level form runs level 1 (restrict from r + solve), then one launch
// per coarse level, each waiting for the previous level's R: at 1M that is
// 10.7 + 6.0 + 6.0 us of mostly latency (a level-2/3 launch solves 32 / 1
// blocks).  But only the RESTRICTIONS are chained; the solves of different
// levels are independent once R is known.  So:
//
//   k_restrict12   one half-wave per level-1 bank: lane j computes R1 of node
//                  j (its vertices' r through l1src, lane order from +0 as
//                  k_coarse_l1); the level-2 nodes of this bank are its
//                  components, each summed by its lowest lane in child-lane
//                  order from +0 (as k_coarse_up) into R2.
//   k_solve123     one wave per block of levels 1 and 2 (Z = Inv R, R from
//                  the first launch) and of level 3 (R3 summed from R2 as
//                  k_coarse_up, then Z3) -- all independent, one launch.
//   (L = 5: level 4 follows as one k_coarse_up launch.)
//
// Same sums in the same order, same solves: bitwise equal to the per-level
// form (tests/test_gpu_chain.py).
#include "block_solve.h"

namespace mas {

// R1 of every level-1 node and R2 of every level-2 node.  One half-wave per
// level-1 bank (32 nodes, lane j = node 32 b + j): R1 from the node's
// vertices (l1src, lane order from +0, as k_coarse_l1).  The level-2 nodes
// whose children live in this bank are its connected components (members:
// child bank = b, mask = the component's lanes), so each R2 is summed inside
// the half-wave by the component's lowest lane, in child-lane order from +0
// (as k_coarse_up).  The parent id and mask loads run beside the l1src load,
// so the r gather is the second dependent load.  128-thread workgroups spread
// the 512 waves (1M) over the CUs.
constexpr int kRestrictWaves = 2;  // waves per workgroup (1 measured 8.4 vs 8.1 us at 1M)
// Measured, not adopted: one wave per bank solving its level-1 block right
// here (record loaded beside the gathers, k_solve123 left with levels 2-3):
// 12.5 + 5.2 us vs 8.1 + 7.9 us -- 244 VGPRs and the gather chain in front of
// the solve make the fused wave slower than two short launches.

__global__ __launch_bounds__(64 * kRestrictWaves) void k_restrict12(int n1, int begin1, const int* __restrict__ l1src,
                                                    const int* __restrict__ goingNext,
                                                    const int2* __restrict__ members, const float4* __restrict__ r,
                                                    float4* __restrict__ rc, const int* __restrict__ done) {
    if (done && *done) return;
    __shared__ float4 red[kRestrictWaves][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, half = lane >> 5;
    const int c = ((blockIdx.x * kRestrictWaves + wave) * 2 + half) * 32 + j;  // level-1 local id
    const bool own = c < n1;
    const int parent = own ? goingNext[begin1 + c] - begin1 : 0;  // level-2 node id - begin1
    const unsigned msk = own ? (unsigned)members[parent].y : 0u;
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (own) {
        const int4* s4 = reinterpret_cast<const int4*>(l1src + (size_t)c * 32);
        int src[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int4 t = s4[q];
            src[4 * q + 0] = t.x;
            src[4 * q + 1] = t.y;
            src[4 * q + 2] = t.z;
            src[4 * q + 3] = t.w;
        }
        float vx[32], vy[32], vz[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const float4 v = r[src[k] >= 0 ? src[k] : 0];
            vx[k] = v.x;
            vy[k] = v.y;
            vz[k] = v.z;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (src[k] >= 0) {
                ax = __fadd_rn(ax, vx[k]);
                ay = __fadd_rn(ay, vy[k]);
                az = __fadd_rn(az, vz[k]);
            }
        }
        rc[c] = make_float4(ax, ay, az, 0.f);  // level-1 node id - begin1 == level-1 local id
    }
    red[wave][lane] = make_float4(ax, ay, az, 0.f);
    __syncthreads();
    if (own && (unsigned)(__ffs(msk) - 1) == (unsigned)j) {  // the component's lowest lane: R2
        float bx = 0.f, by = 0.f, bz = 0.f;
        for (int k = 0; k < 32; ++k) {
            if ((msk >> k) & 1u) {
                const float4 v = red[wave][32 * half + k];
                bx = __fadd_rn(bx, v.x);
                by = __fadd_rn(by, v.y);
                bz = __fadd_rn(bz, v.z);
            }
        }
        rc[parent] = make_float4(bx, by, bz, 0.f);
    }
}

struct Solve123 {
    int b1, nb1, n1;        // level-1 blocks [b1, b1 + nb1), n1 nodes
    int b2, nb2, n2;        // level 2
    int b3, nb3, n3;        // level 3 (R3 restricted here from R2)
    int lv1Begin, lv2Begin, lv3Begin, begin1;
};

__global__ __launch_bounds__(kApplyThreads) void k_solve123(const float4* __restrict__ inv,
                                                           const int2* __restrict__ members, float4* __restrict__ rc,
                                                           float4* __restrict__ zc, Solve123 q,
                                                           const int* __restrict__ done) {
    if (done && *done) return;
    const int lane = threadIdx.x & 63, n = lane & 31;
    int w = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= q.nb1 + q.nb2 + q.nb3) return;  // wave-uniform
    int blk, lvBegin, cnt;
    const bool top = w >= q.nb1 + q.nb2;
    if (w < q.nb1) {
        blk = q.b1 + w; lvBegin = q.lv1Begin; cnt = q.n1;
    } else if (!top) {
        blk = q.b2 + (w - q.nb1); lvBegin = q.lv2Begin; cnt = q.n2;
    } else {
        blk = q.b3 + (w - q.nb1 - q.nb2); lvBegin = q.lv3Begin; cnt = q.n3;
    }
    const int node = blk * 32 + n;
    const bool own = lane < 32 && node - lvBegin < cnt;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (!top) {
        if (own) {
            const float4 v = rc[node - q.begin1];
            ax = v.x; ay = v.y; az = v.z;
        }
    } else if (own) {  // R3 from R2, child-lane order from +0 (as k_coarse_up)
        const int2 mb = members[node - q.begin1];
        const unsigned msk = (unsigned)mb.y;
        const int base = q.lv2Begin + mb.x * 32 - q.begin1;
        float vx[32], vy[32], vz[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if ((msk >> k) & 1u) v = rc[base + k];
            vx[k] = v.x; vy[k] = v.y; vz[k] = v.z;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if ((msk >> k) & 1u) {
                ax = __fadd_rn(ax, vx[k]);
                ay = __fadd_rn(ay, vy[k]);
                az = __fadd_rn(az, vz[k]);
            }
        }
    }
    ax = __shfl(ax, n);  // half 1 takes node n's residual from lane n
    ay = __shfl(ay, n);
    az = __shfl(az, n);
    const float3 out = block_solve(g, tl, make_float3(ax, ay, az), lane);
    if (lane < 32) {
        if (top) rc[node - q.begin1] = make_float4(ax, ay, az, 0.f);
        zc[node - q.begin1] = make_float4(out.x, out.y, out.z, 0.f);
    }
}

// L >= 3: k_restrict12, k_solve123, and for L = 5 a k_coarse_up for level 4.
void launch_coarse_twopass(mas_context* h, const float4* r, hipStream_t s) {
    const int begin1 = h->levelSize[3];
    const int n2 = h->levelSize[4], lv2Begin = h->levelSize[5];
    const int n1 = h->levelSize[2];
    k_restrict12<<<cdiv(n1, 64 * kRestrictWaves), 64 * kRestrictWaves, 0, s>>>(n1, begin1, P<int>(h->l1src), P<int>(h->goingNext),
                                              P<int2>(h->members), r, P<float4>(h->Rc), h->applyDone);
    Solve123 q{};
    q.begin1 = begin1;
    q.lv1Begin = h->levelSize[3];
    q.n1 = h->levelSize[2];
    q.b1 = q.lv1Begin / 32;
    q.nb1 = ceil32(q.n1) / 32;
    q.lv2Begin = lv2Begin;
    q.n2 = n2;
    q.b2 = lv2Begin / 32;
    q.nb2 = ceil32(n2) / 32;
    if (h->L >= 4) {
        q.lv3Begin = h->levelSize[7];
        q.n3 = h->levelSize[6];
        q.b3 = q.lv3Begin / 32;
        q.nb3 = ceil32(q.n3) / 32;
    }
    k_solve123<<<cdiv(q.nb1 + q.nb2 + q.nb3, kApplyThreads / 64), kApplyThreads, 0, s>>>(
        P<float4>(h->inv), P<int2>(h->members), P<float4>(h->Rc), P<float4>(h->Zc), q, h->applyDone);
    if (h->L >= 5) launch_coarse_levels(h, 4, nullptr, s);
}

}  // namespace mas
