// k_coarse.hip -- the coarse levels of one Preconditioning
// (BuildResidualHierarchy .cpp:1548-1598, SchwarzLocalXSym .cpp:1600-1696)
// in two launches (L >= 3), the default coarse form (coarseMode 2).
//
// Only the RESTRICTIONS are chained; the solves of different levels are
// independent once R is known.  So:
//
//   k_restrict12   one wave per level-1 bank: R1 of its 32 nodes (their
//                  vertices' r, lane order from +0, as the reference's owner
//                  loop .cpp:1558-1574), then R2 of the level-2 nodes whose
//                  children live in the bank (level-1 id order from +0,
//                  .cpp:1577-1590).
//   k_solve123     one workgroup per level-3 node first (R3 folded from R1 in
//                  the reference's order, below; the block's last node solves
//                  it), then one wave per block of levels 1 and 2 (Z = Inv R
//                  from the first launch).  All independent.
//
// Level 3 in the reference's order.  BuildResidualHierarchy adds every
// level-1 R into each of its ancestors, walking the level-1 ids in order
// (.cpp:1581-1590), so R3 of node T is the left fold from +0 of R1 over T's
// level-1 descendants in ascending id order -- not the sum of its children's
// R2 (another association).  Each such fold is one dependent chain (~1 024
// adds per level-3 node at 1M, 3.9 us alone on an MI355X CU: the floor of this
// path), so the work is spread over workgroups, one per level-3 node:
// k_restrict12 also stores every R1 at its place in the descendant lists
// (deepR1: node T's list at T * stride, zero-padded to the longest list --
// adding +0.0 to a fold that starts at +0 is exact), so a node's values are
// one contiguous run at a position known without a load: the workgroup loads
// it coalesced into LDS and lanes 0..2 fold x, y, z.  The node's R is
// published with write-through stores and a relaxed agent-scope arrival
// counter per block (an acq_rel atomic measured 4.8 us); the block's last
// arriver reads the others' R with sc1 loads, solves the block (its wave 1
// prefetched the inverse) and resets the counter for the next apply.
// Levels >= 4 (L = 5) are not computed: CollectFinalZ prolongs only levels
// 1..3 (.cpp:1706-1717, B-6), so the reference's R4/Z4 never reach z; folding
// them in its order would be a chain over every level-1 node (n1 adds).
//
// Measured, replaced (scripts/dev/probe_coarse.py stamps, 1M + contacts):
// ONE launch in which level-1 waves hand levels 2 and 3 over by arrival
// counters (write-through stores, drained, then the atomic) -- 31 us: every
// hand-off costs a store drain and an atomic round trip on the longest path,
// and the level-1 inverse loads in the same phase as the r gathers made the
// first loads 6.6 us instead of 3.5 (profiles/round2/bench_fused_onelaunch.json).
#include <algorithm>

#include "block_solve.h"

namespace mas {

// Diagnostic stamps (build with -DMAS_PROBE; never in the product build):
// lane 0 of a wave writes the 100 MHz wall clock into probe slot
// [kernel][wave][k]; mas_probe_dump reads them back (scripts/dev/probe_coarse.py).
#ifdef MAS_PROBE
__device__ unsigned long long g_probe[2 * 4096 * 8];
#define MAS_STAMP(kern, wave, k)                                                                         \
    do {                                                                                                 \
        unsigned long long t_;                                                                           \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        if ((threadIdx.x & 63) == 0 && (wave) < 4096) g_probe[((kern) * 4096 + (wave)) * 8 + (k)] = t_; \
    } while (0)
#else
#define MAS_STAMP(kern, wave, k) \
    do {                         \
    } while (0)
#endif
}  // namespace mas

#include "deep_fold.h"

namespace mas {

// Exactness of the branch-free folds below: a left fold that starts at +0 in
// round-to-nearest never holds -0 (x + y is -0 only for -0 + -0), so adding
// +0.0 to it is the identity -- terms outside a mask are added as +0.0, and
// list padding is +0.0, without changing a bit of the result.

// left fold from +0 over 32 float4 in LDS, x/y/z; msk selects the terms (the
// others count as +0); one LDS round trip per 8 terms
template <bool MASKED>
__device__ __forceinline__ float3 fold32(const float4* __restrict__ row, unsigned msk) {
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 8) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = row[k0 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool in = !MASKED || ((msk >> (k0 + k)) & 1u);
            ax = __fadd_rn(ax, in ? v[k].x : 0.f);
            ay = __fadd_rn(ay, in ? v[k].y : 0.f);
            az = __fadd_rn(az, in ? v[k].z : 0.f);
        }
    }
    return make_float3(ax, ay, az);
}

// the same fold over 32 children stored component-major (three float rows)
__device__ __forceinline__ float3 fold32_soa(const float* __restrict__ rx, const float* __restrict__ ry,
                                             const float* __restrict__ rz) {
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 8) {
        float vx[8], vy[8], vz[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            vx[k] = rx[k0 + k];
            vy[k] = ry[k0 + k];
            vz[k] = rz[k0 + k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            ax = __fadd_rn(ax, vx[k]);
            ay = __fadd_rn(ay, vy[k]);
            az = __fadd_rn(az, vz[k]);
        }
    }
    return make_float3(ax, ay, az);
}

// R1 of level-1 bank `bank` (nodes c0 .. c0 + 31, c0 = 32 bank).  l1src holds
// 32 original vertex ids per node (-1 where the lane is not a child), so the
// bank's 1 024 slots are one contiguous 4 KiB run: lane L loads slots
// 64 q + L (node 2 q + L / 32, child L % 32), 16 coalesced loads, and gathers
// their r -- 64 lanes read the vertices of two Morton tiles per instruction
// (a few cache lines), where a lane-per-node gather touched 64 lines.  The
// values go through LDS to the node's lane, which folds its children in lane
// order from +0.  Every store comes after the last dependent load: a store
// counts in vmcnt like a load, so a wait for a later load would wait for the
// store's completion too (stamped: a fold followed by stores and a dependent
// load took 1.8 us).
constexpr int kRestrictWaves = 2;  // waves (level-1 banks) per workgroup

// SOA: the children's values staged component-major (12.7 KB of LDS per wave
// instead of 16.9): 3 waves per SIMD instead of 2 (LDS-bound), which matters
// when the launch has several rounds of waves (4M tet: 6 530 banks).
template <bool SOA, int WAVES = kRestrictWaves>
__global__ __launch_bounds__(64 * WAVES) void k_restrict12(int n1, int begin1, int L,
                                                                    const int* __restrict__ l1src,
                                                                    const int* __restrict__ goingNext,
                                                                    const int2* __restrict__ members,
                                                                    const float4* __restrict__ r,
                                                                    float4* __restrict__ rc,
                                                                    const int* __restrict__ deepPos,
                                                                    float4* __restrict__ deepR1,
                                                                    const int* __restrict__ done) {
    if (done && *done) return;
    constexpr int kRows = SOA ? 1 : WAVES;
    constexpr int kCols = SOA ? 1 : 33;
    __shared__ float4 sv[kRows][32][kCols];  // [node][child], padded row (!SOA)
    __shared__ float svs[SOA ? WAVES : 1][3][32][33];  // SOA: [component][node][child]
    __shared__ float4 red[WAVES][32];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane & 31;
    const int c0 = (blockIdx.x * WAVES + w) * 32;
    MAS_STAMP(0, c0 / 32, 0);
    if (c0 >= n1) return;  // wave-uniform; no workgroup barriers below
    const int* s = l1src + (size_t)c0 * 32;  // l1src covers ceil32(n1) nodes
    int src[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) src[q] = s[64 * q + lane];
    // independent of the gathers: the lane's own node, its level-2 parent, its list slot
    const int c = c0 + j;
    const bool own = lane < 32 && c < n1;
    const int parent = own && L >= 3 ? goingNext[begin1 + c] - begin1 : 0;
    const int dpos = own && L >= 4 && deepPos ? deepPos[c] : -1;  // null: grouped level 3, no lists
    float4 val[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) val[q] = src[q] >= 0 ? r[src[q]] : make_float4(0.f, 0.f, 0.f, 0.f);
    const unsigned pmsk = own && L >= 3 ? (unsigned)members[parent].y : 0u;  // the parent's children
    if (SOA) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            svs[w][0][2 * q + (lane >> 5)][j] = val[q].x;
            svs[w][1][2 * q + (lane >> 5)][j] = val[q].y;
            svs[w][2][2 * q + (lane >> 5)][j] = val[q].z;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) sv[w][2 * q + (lane >> 5)][j] = val[q];
    }
    MAS_STAMP(0, c0 / 32, 1);
    __builtin_amdgcn_wave_barrier();
    // R1: the node's children in lane order from +0 (non-children are +0.0)
    float3 a = make_float3(0.f, 0.f, 0.f);
    if (own) a = SOA ? fold32_soa(svs[w][0][j], svs[w][1][j], svs[w][2][j]) : fold32<false>(sv[w][j], 0u);
    if (lane < 32) red[w][j] = make_float4(a.x, a.y, a.z, 0.f);  // lanes j and 32 + j share the slot
    __builtin_amdgcn_wave_barrier();
    // R2 of the level-2 nodes whose children are this bank's components (lowest lane)
    const bool r2w = own && L >= 3 && (unsigned)(__ffs(pmsk) - 1) == (unsigned)j;
    float3 b = make_float3(0.f, 0.f, 0.f);
    if (r2w) b = fold32<true>(red[w], pmsk);
    if (own) {
        const float4 R1 = make_float4(a.x, a.y, a.z, 0.f);
        rc[c] = R1;  // level-1 node id - begin1 == level-1 local id
        if (dpos >= 0) deepR1[dpos] = R1;  // its place in its level-3 ancestor's list
    }
    if (r2w) rc[parent] = make_float4(b.x, b.y, b.z, 0.f);
    MAS_STAMP(0, c0 / 32, 2);
}

struct Solve12 {
    int b1, nb1, n1;  // level-1 blocks [b1, b1 + nb1), n1 nodes
    int b2, nb2, n2;  // level 2
    int lv1Begin, lv2Begin, begin1;
    int nDeepNodes;   // level-3 nodes lv3Begin .. + nDeepNodes: the first nDeepNodes workgroups
};

__device__ __forceinline__ void solve12_wave(const float4* __restrict__ inv, float4* __restrict__ rc,
                                             float4* __restrict__ zc, const Solve12& q, int w);

// Workgroups [0, nDeepNodes): one level-3 node each (R1 from deepR1).  The
// rest: one wave per block of levels 1 and 2, Z = Inv R with R from
// k_restrict12.
// PREFETCH (deep_node): the level-3 block's inverse in flight during the fold
// (182 VGPRs, 2 waves per SIMD); without it more waves per SIMD for the
// level-1 and level-2 solves, which matters once they take several rounds.
// THREADS = 512 (the wide form): with > 128 VGPRs per wave a workgroup
// then fills its CU, so a level-3 fold has its CU to itself.
template <bool PREFETCH, int THREADS = kApplyThreads>
__global__ __launch_bounds__(THREADS) void k_solve123(const float4* __restrict__ inv, DeepArgs d,
                                                     float4* __restrict__ rc, float4* __restrict__ zc,
                                                     Solve12 q, const int* __restrict__ done) {
    if (done && *done) return;
    if ((int)blockIdx.x < q.nDeepNodes) {  // workgroup-uniform
        deep_node<false, PREFETCH, THREADS>(inv, d.lv3Begin + blockIdx.x, d, rc, zc, q.begin1);
        return;
    }
    // The level-1/2 solves have slack (~4 us of work beside the ~11 us
    // level-3 chain): held back ~1.7 us (s_sleep 64 x 64 cycles), their 20 MB
    // of inverse loads no longer queue in front of the deep lists and the
    // fold's SIMDs stay quiet.  pre-fine 21.7 -> 19.4 us at 1M + contacts
    // (sleep 32 / 64 / 127: 19.9 / 19.4 / 19.9 us).
    if (q.nDeepNodes > 0) __builtin_amdgcn_s_sleep(64);
    const int w = (blockIdx.x - q.nDeepNodes) * (THREADS / 64) + (threadIdx.x >> 6);
    if (w >= q.nb1 + q.nb2) return;  // wave-uniform
    solve12_wave(inv, rc, zc, q, w);
}

// Grouped level 3 (mas_config.reference_restriction = 0, the default).  R3 of
// a level-3 node = its children's R2 -- the lanes of one component of one
// level-2 bank (members) -- folded in level-2 id order from +0, R2 from
// k_restrict12: a 32-add chain per node instead of the reference's 1 024-add
// fold over R1 (deep_fold.h), the same sum associated by level-2 node.  One
// wave per level-3 block: the 1 024 child slots of its 32 nodes are gathered
// 16 per lane (item 64 q + lane = node 2 q + lane / 32, child lane % 32;
// masked-out children +0.0, exact in a fold from +0) into LDS, lane n folds
// node n's row, then Z3 = Inv R3 with the inverse loaded at wave start.
struct Solve3 {
    int b3, nb3, n3;       // level-3 blocks [b3, b3 + nb3), n3 nodes
    int lv3Begin, lv2Begin;
};

__device__ __forceinline__ void solve3_grouped_wave(const float4* __restrict__ inv, const int2* __restrict__ members,
                                                    float4* __restrict__ rc, float4* __restrict__ zc, int begin1,
                                                    const Solve3& q3, int k, float (&sv)[3][32][33]) {
    const int lane = threadIdx.x & 63, n = lane & 31, j = lane & 31;
    const int blk = q3.b3 + k, node = blk * 32 + n;
    const bool own = lane < 32 && node - q3.lv3Begin < q3.n3;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    const int2 mb = own ? members[node - begin1] : make_int2(0, 0);
    const int base = q3.lv2Begin - begin1;  // Rc index of level-2 local id 0
    float4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int nn = 2 * q + (lane >> 5);
        const int bank = __shfl(mb.x, nn);
        const unsigned msk = (unsigned)__shfl(mb.y, nn);
        v[q] = (msk >> j) & 1u ? rc[base + bank * 32 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        sv[0][2 * q + (lane >> 5)][j] = v[q].x;
        sv[1][2 * q + (lane >> 5)][j] = v[q].y;
        sv[2][2 * q + (lane >> 5)][j] = v[q].z;
    }
    __builtin_amdgcn_wave_barrier();
    float3 a = make_float3(0.f, 0.f, 0.f);
    if (own) a = fold32_soa(sv[0][n], sv[1][n], sv[2][n]);
    const float ax = __shfl(a.x, n), ay = __shfl(a.y, n), az = __shfl(a.z, n);  // half 1 takes node n's R
    const float3 out = block_solve(g, tl, make_float3(ax, ay, az), lane);
    if (lane < 32) {
        rc[node - begin1] = make_float4(ax, ay, az, 0.f);
        zc[node - begin1] = make_float4(out.x, out.y, out.z, 0.f);
    }
}

// Grouped form of k_solve123: workgroups [0, nb3) give their wave 0 to a
// level-3 block (LDS for one), every other wave solves a level-1/2 block.
// Nothing waits on anything inside the launch.
__global__ __launch_bounds__(kApplyThreads) void k_solve123g(const float4* __restrict__ inv,
                                                            const int2* __restrict__ members,
                                                            float4* __restrict__ rc, float4* __restrict__ zc,
                                                            Solve12 q, Solve3 q3, const int* __restrict__ done) {
    if (done && *done) return;
    __shared__ float sv[3][32][33];
    const int wv = threadIdx.x >> 6, g = blockIdx.x;
    if (g < q3.nb3 && wv == 0) {  // wave-uniform
        solve3_grouped_wave(inv, members, rc, zc, q.begin1, q3, g, sv);
        return;
    }
    const int w = g * (kApplyThreads / 64) + wv - min(q3.nb3, g + 1);
    if (w >= q.nb1 + q.nb2) return;  // wave-uniform
    solve12_wave(inv, rc, zc, q, w);
}

// L = 3 (no level-3 nodes): one single-wave workgroup per level-1/2 block, so
// the few hundred block solves spread over every CU instead of a quarter of them
__global__ __launch_bounds__(64) void k_solve12_narrow(const float4* __restrict__ inv, float4* __restrict__ rc,
                                                      float4* __restrict__ zc, Solve12 q,
                                                      const int* __restrict__ done) {
    if (done && *done) return;
    solve12_wave(inv, rc, zc, q, blockIdx.x);
}

// Z = Inv R of level-1/2 block w (levels 1, then 2), one wave
__device__ __forceinline__ void solve12_wave(const float4* __restrict__ inv, float4* __restrict__ rc,
                                             float4* __restrict__ zc, const Solve12& q, int w) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    [[maybe_unused]] const int pw = blockIdx.x * 4 + (threadIdx.x >> 6);
    MAS_STAMP(1, pw, 0);
    int blk, lvBegin, cnt;
    if (w < q.nb1) {
        blk = q.b1 + w; lvBegin = q.lv1Begin; cnt = q.n1;
    } else {
        blk = q.b2 + (w - q.nb1); lvBegin = q.lv2Begin; cnt = q.n2;
    }
    const int node = blk * 32 + n;
    const bool own = lane < 32 && node - lvBegin < cnt;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (own) {
        const float4 v = rc[node - q.begin1];
        ax = v.x; ay = v.y; az = v.z;
    }
    ax = __shfl(ax, n);  // half 1 takes node n's residual from lane n
    ay = __shfl(ay, n);
    az = __shfl(az, n);
    MAS_STAMP(1, pw, 1);
    const float3 out = block_solve(g, tl, make_float3(ax, ay, az), lane);
    MAS_STAMP(1, pw, 2);
    if (lane < 32) zc[node - q.begin1] = make_float4(out.x, out.y, out.z, 0.f);
}

// Level-3 nodes alone (the per-level form and the sharded apply): R1 gathered
// through d.idx from d.src.
__global__ __launch_bounds__(kApplyThreads) void k_coarse_deep(const float4* __restrict__ inv, DeepArgs d,
                                                              float4* __restrict__ rc, float4* __restrict__ zc,
                                                              int begin1, const int* __restrict__ done) {
    if (done && *done) return;
    deep_node<true>(inv, d.lv3Begin + blockIdx.x, d, rc, zc, begin1);
}

int deep_nodes(const mas_context* h) {  // level-3 node ids incl. padding (L >= 4)
    return h->L >= 4 ? (h->L >= 5 ? h->levelSize[9] : h->totalClusters) - h->levelSize[7] : 0;
}

DeepArgs deep_args(mas_context* h, const float4* src, const int* idx) {
    DeepArgs d{};
    d.idx = idx;
    d.src = src;
    d.lv3Begin = h->L >= 4 ? h->levelSize[7] : h->totalClusters;
    d.stride = h->deepStride;
    d.cnt = P<int>(h->deepCnt);
    return d;
}

// every level-3 node (L >= 4); src/idx: R1 and the list entries' positions
// in it (null: Rc and deepIdx)
void launch_coarse_deep(mas_context* h, const float4* src, const int* idx, hipStream_t s) {
    if (h->L < 4) return;
    const DeepArgs d = deep_args(h, src ? src : P<float4>(h->Rc), idx ? idx : P<int>(h->deepIdx));
    k_coarse_deep<<<deep_nodes(h), kApplyThreads, 0, s>>>(P<float4>(h->inv), d, P<float4>(h->Rc), P<float4>(h->Zc),
                                                          h->levelSize[3], h->applyDone);
}

// L >= 3: k_restrict12, then k_solve123 (level-3 nodes + levels 1 and 2).
void launch_coarse_twopass(mas_context* h, const float4* r, hipStream_t s) {
    const int begin1 = h->levelSize[3];
    const int n1 = h->levelSize[2];
    const int nb1 = ceil32(n1) / 32;
    // the occupancy forms once a launch holds several rounds of waves (A/B: env MAS_COARSE_OCC)
    const bool occ = h->coarseOcc > 0 || (h->coarseOcc < 0 && nb1 >= kCoarseOccBlocks);
    // single-wave workgroups when there is no level-3 chain (L = 3): the few
    // hundred coarse waves then spread over every CU (256k: pre-fine 12.7 ->
    // 11.3 us; at 1M the restriction alone this way measured no gain)
    const bool narrow = h->coarseNarrow > 0 || (h->coarseNarrow < 0 && h->L == 3);
    const dim3 rg(cdiv(nb1, kRestrictWaves)), rb(64 * kRestrictWaves);
    const bool grouped = h->groupedR3 && h->L >= 4;
    const int* deepPos = grouped ? nullptr : P<int>(h->deepPos);  // grouped: no level-3 lists to fill
    if (narrow && !occ)
        k_restrict12<false, 1><<<nb1, 64, 0, s>>>(n1, begin1, h->L, P<int>(h->l1src), P<int>(h->goingNext),
                                                  P<int2>(h->members), r, P<float4>(h->Rc), deepPos,
                                                  P<float4>(h->deepR1), h->applyDone);
    else if (occ)
        k_restrict12<true><<<rg, rb, 0, s>>>(n1, begin1, h->L, P<int>(h->l1src), P<int>(h->goingNext),
                                             P<int2>(h->members), r, P<float4>(h->Rc), deepPos,
                                             P<float4>(h->deepR1), h->applyDone);
    else
        k_restrict12<false><<<rg, rb, 0, s>>>(n1, begin1, h->L, P<int>(h->l1src), P<int>(h->goingNext),
                                              P<int2>(h->members), r, P<float4>(h->Rc), deepPos,
                                              P<float4>(h->deepR1), h->applyDone);
    Solve12 q{};
    q.begin1 = begin1;
    q.lv1Begin = begin1;
    q.n1 = n1;
    q.b1 = begin1 / 32;
    q.nb1 = ceil32(n1) / 32;
    q.lv2Begin = h->levelSize[5];
    q.n2 = h->levelSize[4];
    q.b2 = q.lv2Begin / 32;
    q.nb2 = ceil32(q.n2) / 32;
    if (grouped) {
        Solve3 q3{};
        q3.n3 = h->levelSize[6];
        q3.lv3Begin = h->levelSize[7];
        q3.lv2Begin = q.lv2Begin;
        q3.b3 = q3.lv3Begin / 32;
        q3.nb3 = ceil32(q3.n3) / 32;
        const int grid = std::max(q3.nb3, cdiv(q3.nb3 + q.nb1 + q.nb2, kApplyThreads / 64));
        k_solve123g<<<grid, kApplyThreads, 0, s>>>(P<float4>(h->inv), P<int2>(h->members), P<float4>(h->Rc),
                                                   P<float4>(h->Zc), q, q3, h->applyDone);
        return;
    }
    const DeepArgs d = deep_args(h, P<float4>(h->deepR1), nullptr);
    q.nDeepNodes = deep_nodes(h);
    const dim3 sg(q.nDeepNodes + cdiv(q.nb1 + q.nb2, kApplyThreads / 64));
    if (narrow && q.nDeepNodes == 0)
        k_solve12_narrow<<<q.nb1 + q.nb2, 64, 0, s>>>(P<float4>(h->inv), P<float4>(h->Rc), P<float4>(h->Zc), q,
                                                     h->applyDone);
    else if (occ)
        k_solve123<false><<<sg, kApplyThreads, 0, s>>>(P<float4>(h->inv), d, P<float4>(h->Rc), P<float4>(h->Zc), q,
                                                       h->applyDone);
    else if (h->coarseWide > 0)
        k_solve123<true, 512><<<q.nDeepNodes + cdiv(q.nb1 + q.nb2, 8), 512, 0, s>>>(
            P<float4>(h->inv), d, P<float4>(h->Rc), P<float4>(h->Zc), q, h->applyDone);
    else
        k_solve123<true><<<sg, kApplyThreads, 0, s>>>(P<float4>(h->inv), d, P<float4>(h->Rc), P<float4>(h->Zc), q,
                                                      h->applyDone);
}

// ---- Prepare: the level-3 descendant lists ----
// keys[i] = level-3 local id of level-1 node i's ancestor; a stable sort by
// key lists every level-3 node's level-1 descendants in ascending id order.
__global__ __launch_bounds__(256) void k_deep_keys(int n1, int begin1, int lv3Begin, const int* __restrict__ gn,
                                                   int* __restrict__ keys, int* __restrict__ vals) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n1) return;
    keys[i] = gn[gn[begin1 + i]] - lv3Begin;  // level 1 -> 2 -> 3
    vals[i] = i;
}

// off[k] = first sorted position with key >= k (k = 0 .. nDeep); the longest list
__global__ __launch_bounds__(256) void k_deep_off(int nDeep, int n, const int* __restrict__ sortedKeys,
                                                  int* __restrict__ off, int* __restrict__ maxLen) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k > nDeep) return;
    auto lower = [&](int key) {
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sortedKeys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int o = lower(k);
    off[k] = o;
    if (k < nDeep) atomicMax(maxLen, lower(k + 1) - o);
}

// sorted position p holds level-1 node i of node T = key: its list slot is
// T * stride + (p - off[T])
__global__ __launch_bounds__(256) void k_deep_pos(int n, int stride, const int* __restrict__ sortedKeys,
                                                  const int* __restrict__ sortedVals, const int* __restrict__ off,
                                                  int* __restrict__ idx, int* __restrict__ pos) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int T = sortedKeys[p], i = sortedVals[p];
    const int slot = T * stride + (p - off[T]);
    idx[slot] = i;
    pos[i] = slot;
}

__global__ __launch_bounds__(256) void k_map_idx(int n, const int* __restrict__ map, const int* __restrict__ in,
                                                 int* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i] >= 0 ? map[in[i]] : -1;
}

int build_deep_lists(mas_context* h, hipStream_t s) {
    h->deepStride = 0;
    if (h->L < 4) return MAS_OK;
    const int n1 = h->levelSize[2], begin1 = h->levelSize[3], lv3Begin = h->levelSize[7];
    const int nDeep = deep_nodes(h);
    int rc;
    if ((rc = ensure(h, h->deepKeys, (size_t)n1 * 4 * 2)) || (rc = ensure(h, h->deepVals, (size_t)n1 * 4 * 2)) ||
        (rc = ensure(h, h->deepPos, (size_t)n1 * 4)) || (rc = ensure(h, h->deepOff, (size_t)(nDeep + 2) * 4)) ||
        (rc = ensure(h, h->deepCnt, (size_t)(nDeep / 32) * 4)))
        return rc;
    int* keys = P<int>(h->deepKeys);
    int* keysS = keys + n1;
    int* vals = P<int>(h->deepVals);
    int* valsS = vals + n1;
    int* off = P<int>(h->deepOff);
    k_deep_keys<<<cdiv(n1, 256), 256, 0, s>>>(n1, begin1, lv3Begin, P<int>(h->goingNext), keys, vals);
    int bits = 1;
    while ((1 << bits) < nDeep) ++bits;
    if ((rc = sort_pairs_u32(h, reinterpret_cast<const unsigned*>(keys), reinterpret_cast<unsigned*>(keysS), vals,
                             valsS, n1, bits, s, "deep sort")) ||
        (rc = hip_check(h, hipMemsetAsync(off + nDeep + 1, 0, 4, s), "memset")))
        return rc;
    k_deep_off<<<cdiv(nDeep + 1, 256), 256, 0, s>>>(nDeep, n1, keysS, off, off + nDeep + 1);
    int maxLen = 0;
    if ((rc = read_back(h, s, {off + nDeep + 1}, &maxLen))) return rc;
    const int stride = std::max(32, (maxLen + 31) / 32 * 32);  // whole 8-float4 batches in the fold
    const size_t slots = (size_t)nDeep * stride;
    if ((rc = ensure(h, h->deepIdx, slots * 4)) || (rc = ensure(h, h->deepR1, slots * 16)) ||
        (rc = hip_check(h, hipMemsetAsync(h->deepIdx.p, 0xff, slots * 4, s), "memset deepIdx")) ||
        (rc = hip_check(h, hipMemsetAsync(h->deepR1.p, 0, slots * 16, s), "memset deepR1")) ||
        (rc = hip_check(h, hipMemsetAsync(h->deepCnt.p, 0, (size_t)(nDeep / 32) * 4, s), "memset deepCnt")))
        return rc;
    k_deep_pos<<<cdiv(n1, 256), 256, 0, s>>>(n1, stride, keysS, valsS, off, P<int>(h->deepIdx), P<int>(h->deepPos));
    h->deepStride = stride;
    return hip_check(h, hipGetLastError(), "deep lists");
}

// the sharded apply reads R1 from the gathered segments: deepIdx through pos1
int build_deep_shard_idx(mas_context* h, hipStream_t s) {
    if (h->L < 4) return MAS_OK;
    const int n = deep_nodes(h) * h->deepStride;
    int rc;
    if ((rc = ensure(h, h->deepIdxShard, (size_t)n * 4))) return rc;
    k_map_idx<<<cdiv(n, 256), 256, 0, s>>>(n, P<int>(h->shardPos1), P<int>(h->deepIdx), P<int>(h->deepIdxShard));
    return hip_check(h, hipGetLastError(), "deep shard idx");
}

}  // namespace mas

#ifdef MAS_PROBE
extern "C" int mas_probe_dump(unsigned long long* out, int n) {
    if (n > 2 * 4096 * 8) n = 2 * 4096 * 8;
    hipDeviceSynchronize();
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mas::g_probe), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
extern "C" int mas_probe_clear() {
    static unsigned long long zero[2 * 4096 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(mas::g_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
