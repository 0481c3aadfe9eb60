// k_apply.hip -- Preconditioning (.cpp:100-110, 1548-1719): the hot path.
//
// Per apply, on one stream: the coarse levels, then k_solve_fine.  For
// L >= 3 the coarse levels default to one launch (k_coarse1.hip; the
// two-launch form k_coarse.hip is taken while a graph is captured); the
// per-level form below is kept as coarseMode 0 (and is the L = 2 path).  All
// forms are bitwise equal.
//   k_coarse_l1         per level-1 block (one wave): R1 of its 32 nodes from
//                       r gathered through the Morton map, summed per parent
//                       in lane order from +0 exactly as the reference's owner
//                       loop (BuildResidualHierarchy .cpp:1558-1574); then
//                       Z1 = Inv_b R1 (SchwarzLocalXSym .cpp:1600-1696).
//   k_coarse_up         level 2: R2 from R1 the same way (the reference's
//                       level-1-id-order sum, .cpp:1581-1590), then Z2;
//                       levels >= 3: k_coarse_deep (k_coarse.hip).
//   k_solve_fine        every level-0 block fused with the gather r[s2o[v]]
//                       and the prolongation z[s2o[v]] = Z0 + Z1[a1] + Z2[a2]
//                       + Z3[a3] (CollectFinalZ .cpp:1698-1719, min(L,4)-1
//                       coarse levels, B-6).  This kernel streams 18 624 B of
//                       packed inverse per block and dominates the apply.
//
// Block solve (layout.h): one wave64 per 32-node block, lane 32h + n owns
// node n; the halves split the 3x3 node-pair blocks by rotation distance.
// The packed inverse arrives through 18 float4 loads per lane (1 KiB
// contiguous per wave-instruction) plus a 12-byte tail straight into
// registers; the symmetric mat-vec is 8 rotation steps of ds_bpermute
// shuffles (lane n multiplies G(n, n+s) with r_{n+s} and returns G^T r_n to
// lane n+s) and one cross-half add.  No LDS, no atomics, no barriers.
#include <vector>

#include "block_solve.h"

namespace mas {

static inline int grid_for_blocks(int blocks) { return cdiv(blocks, kApplyThreads / 64); }

// Fine blocks: gather r through the Morton map, solve, prolongate, scatter z.
// The packed inverses are read exactly once per apply (630 MB at 1M, more
// than the 256 MiB Infinity Cache), so they are loaded nontemporal: measured
// 98.8 vs 109.7 us per launch at 1M against default-policy loads (VAR = 0,
// env MAS_FINE_VARIANT=0 keeps that variant for A/B runs; VAR = 1: the
// nontemporal form without the XCD chunking of VAR = 4).
// RZ (the PCG driver's applies, k_pcg.hip): exit at once when *done is set,
// and emit this workgroup's r.z (fp64; a fixed xor butterfly per wave, then
// the waves in order) to rzPart[blockIdx.x], so the solver needs no separate
// pass over r and z.
// VAR 4 (MAS_FINE_VARIANT=4; 6, the default, in two-wave workgroups): nontemporal, and workgroups are
// dealt to the XCDs in contiguous chunks (workgroup g runs on XCD g % 8, so
// logical workgroup (g % 8) * (G / 8) + g / 8): Morton-adjacent blocks then
// share an XCD's L2 for the r lines they gather and the z lines they write.
// Interleaved in one process, bitwise equal (profiles/round4/fine_pmc/ab_*.json):
// 4M tet 382 -> 357 us per launch, 1M + contacts 98.5 -> 98.0 us.
__device__ __forceinline__ int xcd_chunked(int g, int G) {
    const int full = G & ~7;
    return g < full ? (g & 7) * (full >> 3) + (g >> 3) : g;
}

template <int NPROL, int VAR, bool RZ, int WPB = kApplyThreads / 64>
__device__ __forceinline__ void solve_fine_body(const float4* __restrict__ inv, int blk0, int nFineBlk, int nV,
                                                const float4* __restrict__ r, const int4* __restrict__ vmap,
                                                const float4* __restrict__ zc, int begin1, float4* __restrict__ z,
                                                double* __restrict__ rzPart) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int wg = (VAR == 4 || VAR == 8) ? xcd_chunked(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int blk = blk0 + wg * WPB + (threadIdx.x >> 6);
    const bool bvalid = blk < nFineBlk;
    const int v = blk * 32 + n;
    const bool vvalid = bvalid && v < nV;
    const int4 m = vmap[vvalid ? v : 0];
    float g[kRecord], tl[3];
    load_record<VAR != 0 && VAR != 8>(inv, bvalid ? blk : 0, lane, g, tl);
    const float4 rv = r[m.x];
    const float3 rr = vvalid ? make_float3(rv.x, rv.y, rv.z) : make_float3(0.f, 0.f, 0.f);
    float3 out = block_solve(g, tl, rr, lane);
    const bool writer = vvalid && lane < 32;
    if (writer) {
        if (NPROL >= 1) {
            const float4 a = zc[m.y - begin1];
            out.x = __fadd_rn(out.x, a.x); out.y = __fadd_rn(out.y, a.y); out.z = __fadd_rn(out.z, a.z);
        }
        if (NPROL >= 2) {
            const float4 a = zc[m.z - begin1];
            out.x = __fadd_rn(out.x, a.x); out.y = __fadd_rn(out.y, a.y); out.z = __fadd_rn(out.z, a.z);
        }
        if (NPROL >= 3) {
            const float4 a = zc[m.w - begin1];
            out.x = __fadd_rn(out.x, a.x); out.y = __fadd_rn(out.y, a.y); out.z = __fadd_rn(out.z, a.z);
        }
        z[m.x] = make_float4(out.x, out.y, out.z, 0.f);
    }
    if (RZ) {
        double a = writer ? (double)out.x * rr.x + (double)out.y * rr.y + (double)out.z * rr.z : 0.0;
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
        __shared__ double sw[WPB];
        if (lane == 0) sw[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int w = 0; w < WPB; ++w) t += sw[w];
            rzPart[blockIdx.x] = t;
        }
    }
}


// WPB blocks (waves) per workgroup: 2 by default (MAS_FINE_VARIANT=6) -- two-
// wave workgroups, XCD-chunked, measured interleaved against four-wave ones,
// bitwise equal (profiles/round4/ab/fine_wpb/): 1M + contacts 113.0 -> 112.0
// us per apply, 256k 32.03 -> 31.78, 4M tet 453.6 -> 451.3 (one-wave
// workgroups: better at 1M, worse at 256k and 4M).
template <int NPROL, int VAR, bool RZ, int WPB = kApplyThreads / 64>
__global__ __launch_bounds__(64 * WPB) void k_solve_fine(const float4* __restrict__ inv, int blk0, int nFineBlk,
                                                        int nV, const float4* __restrict__ r,
                                                        const int4* __restrict__ vmap,
                                                        const float4* __restrict__ zc, int begin1,
                                                        float4* __restrict__ z, const int* __restrict__ done,
                                                        double* __restrict__ rzPart) {
    if (RZ && *done) return;
    solve_fine_body<NPROL, VAR, RZ, WPB>(inv, blk0, nFineBlk, nV, r, vmap, zc, begin1, z, rzPart);
}

// A/B (MAS_FINE_VARIANT=7): the chunked form in one-wave workgroups.
template <int NPROL>
__global__ __launch_bounds__(64) void k_solve_fine1c(const float4* __restrict__ inv, int blk0, int nFineBlk, int nV,
                                                    const float4* __restrict__ r, const int4* __restrict__ vmap,
                                                    const float4* __restrict__ zc, int begin1, float4* __restrict__ z) {
    solve_fine_body<NPROL, 4, false, 1>(inv, blk0, nFineBlk, nV, r, vmap, zc, begin1, z, nullptr);
}

// A/B (MAS_FINE_VARIANT=3): one wave per workgroup.  Measured interleaved,
// 4M tet: 433.5 -> 394.6 us per launch on one box, 436.3 -> 472.0 us on
// another; 1M 104.2 -> 107.2 us; 256k unchanged -- not the default.
template <int NPROL>
__global__ __launch_bounds__(64) void k_solve_fine1(const float4* __restrict__ inv, int blk0, int nFineBlk, int nV,
                                                   const float4* __restrict__ r, const int4* __restrict__ vmap,
                                                   const float4* __restrict__ zc, int begin1, float4* __restrict__ z) {
    solve_fine_body<NPROL, 1, false, 1>(inv, blk0, nFineBlk, nV, r, vmap, zc, begin1, z, nullptr);
}

// Coarse levels, one wave per 32-node block; lane n (half 0) owns node
// P = 32 blk + n.  The children of P are exactly the lanes of one component
// of one child bank (the connected component the clustering merged into P,
// .cpp:590-625 / 917-954).  Every child value is gathered up front (one
// latency), then lane n adds its children in lane order from +0 -- the
// reference's accumulation order for level 1 (.cpp:1560-1572) and level 2
// (level-1 id order, .cpp:1581-1590).  Then Z_l = Inv_b R_l; R_l and Z_l are
// stored.
//
// Level 1 reads its children's original vertex ids from l1src (32 ids per
// level-1 node, -1 where the lane is not a child; built at Prepare), so the
// r gather is the second dependent load of the wave instead of the third
// (members -> s2o -> r).  Levels >= 2 read members = (child bank, mask).
__device__ __forceinline__ void coarse_finish(const float (&g)[kRecord], const float (&tl)[3], int lane, int n,
                                              int node, bool own, float ax, float ay, float az,
                                              float4* __restrict__ rc, float4* __restrict__ zc, int begin1) {
    // half 1 takes node n's residual from lane n
    ax = __shfl(ax, n);
    ay = __shfl(ay, n);
    az = __shfl(az, n);
    const float3 out = block_solve(g, tl, make_float3(ax, ay, az), lane);
    if (lane < 32) {
        rc[node - begin1] = make_float4(ax, ay, az, 0.f);
        zc[node - begin1] = make_float4(out.x, out.y, out.z, 0.f);
    }
    (void)own;
}

__device__ __forceinline__ void coarse_block_l1(const float4* __restrict__ inv, int blk, int blkBegin, int count,
                                                const int* __restrict__ l1src, const float4* __restrict__ r,
                                                float4* __restrict__ rc, float4* __restrict__ zc, int begin1,
                                                int lane) {
    const int n = lane & 31;
    const int node = blk * 32 + n;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    const bool own = lane < 32 && (node - blkBegin * 32) < count;
    int src[32];
    const int4* s4 = reinterpret_cast<const int4*>(l1src + (size_t)(node - blkBegin * 32) * 32);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int4 t = own ? s4[q] : make_int4(-1, -1, -1, -1);
        src[4 * q + 0] = t.x;
        src[4 * q + 1] = t.y;
        src[4 * q + 2] = t.z;
        src[4 * q + 3] = t.w;
    }
    float vx[32], vy[32], vz[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (src[j] >= 0) v = r[src[j]];
        vx[j] = v.x;
        vy[j] = v.y;
        vz[j] = v.z;
    }
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if (src[j] >= 0) {
            ax = __fadd_rn(ax, vx[j]);
            ay = __fadd_rn(ay, vy[j]);
            az = __fadd_rn(az, vz[j]);
        }
    }
    coarse_finish(g, tl, lane, n, node, own, ax, ay, az, rc, zc, begin1);
}

__device__ __forceinline__ void coarse_block_up(const float4* __restrict__ inv, int blk, int blkBegin, int count,
                                                const int2* __restrict__ members, int childBegin,
                                                float4* __restrict__ rc, float4* __restrict__ zc, int begin1,
                                                int lane) {
    const int n = lane & 31;
    const int node = blk * 32 + n;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    const bool own = lane < 32 && (node - blkBegin * 32) < count;
    const int2 mb = own ? members[node - begin1] : make_int2(0, 0);
    const unsigned msk = (unsigned)mb.y;
    const int base = childBegin + mb.x * 32 - begin1;
    float vx[32], vy[32], vz[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((msk >> j) & 1u) v = rc[base + j];
        vx[j] = v.x;
        vy[j] = v.y;
        vz[j] = v.z;
    }
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if ((msk >> j) & 1u) {
            ax = __fadd_rn(ax, vx[j]);
            ay = __fadd_rn(ay, vy[j]);
            az = __fadd_rn(az, vz[j]);
        }
    }
    coarse_finish(g, tl, lane, n, node, own, ax, ay, az, rc, zc, begin1);
}

__global__ __launch_bounds__(kApplyThreads) void k_coarse_l1(const float4* __restrict__ inv, int blkBegin, int nb,
                                                            int count, const int* __restrict__ l1src,
                                                            const float4* __restrict__ r, float4* __restrict__ rc,
                                                            float4* __restrict__ zc, int begin1,
                                                            const int* __restrict__ done) {
    if (done && *done) return;
    const int w = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= nb) return;  // wave-uniform
    coarse_block_l1(inv, blkBegin + w, blkBegin, count, l1src, r, rc, zc, begin1, threadIdx.x & 63);
}

__global__ __launch_bounds__(kApplyThreads) void k_coarse_up(const float4* __restrict__ inv, int blkBegin, int nb,
                                                            int count, const int2* __restrict__ members,
                                                            int childBegin, float4* __restrict__ rc,
                                                            float4* __restrict__ zc, int begin1,
                                                            const int* __restrict__ done) {
    if (done && *done) return;
    const int w = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= nb) return;  // wave-uniform
    coarse_block_up(inv, blkBegin + w, blkBegin, count, members, childBegin, rc, zc, begin1, threadIdx.x & 63);
}

// Prepare-time: members[P] = (bank, closure mask) of the component that
// became coarse node P; written by the component's lowest lane.
__global__ __launch_bounds__(256) void k_members(int nChild, int childBegin, const unsigned* __restrict__ masks,
                                                 const int* __restrict__ gn, int begin1, int2* __restrict__ members) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nChild) return;
    const unsigned m = masks[c];
    const unsigned lane = c & 31;
    if (__popc(m & ((1u << lane) - 1u)) != 0) return;
    members[gn[childBegin + c] - begin1] = make_int2(c >> 5, (int)m);
}


template <int NPROL>
static void launch_fine_n(int var, int g, hipStream_t s, const float4* inv, int blk0, int blkEnd, int nV,
                          const float4* r, const int4* vmap, const float4* zc, int begin1, float4* z,
                          const int* done, double* rzPart, int rzWpb = 2) {
    if (rzPart) {  // the PCG driver's applies (fine_grid(h) workgroups: one r.z partial each)
        if (var == 6 && rzWpb == 8)
            k_solve_fine<NPROL, 4, true, 8><<<cdiv(blkEnd - blk0, 8), 512, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                                 begin1, z, done, rzPart);
        else if (var == 6 && rzWpb == 4)
            k_solve_fine<NPROL, 4, true, 4><<<cdiv(blkEnd - blk0, 4), 256, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                                 begin1, z, done, rzPart);
        else if (var == 8)
            k_solve_fine<NPROL, 8, true, 4><<<cdiv(blkEnd - blk0, 4), 256, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                                 begin1, z, done, rzPart);
        else if (var == 6)
            k_solve_fine<NPROL, 4, true, 2><<<cdiv(blkEnd - blk0, 2), 128, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                                 begin1, z, done, rzPart);
        else if (var == 0)
            k_solve_fine<NPROL, 0, true><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                       done, rzPart);
        else if (var >= 4)  // 4, 5, 7: four-wave workgroups
            k_solve_fine<NPROL, 4, true><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                       done, rzPart);
        else
            k_solve_fine<NPROL, 1, true><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                       done, rzPart);
    } else if (var == 3) {
        k_solve_fine1<NPROL><<<blkEnd - blk0, 64, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z);
    } else if (var == 4) {
        k_solve_fine<NPROL, 4, false><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                    nullptr, nullptr);
    } else if (var == 6) {
        k_solve_fine<NPROL, 4, false, 2><<<cdiv(blkEnd - blk0, 2), 128, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                               begin1, z, nullptr, nullptr);
    } else if (var == 8) {  // the default form with default-policy inverse loads (fine_var)
        k_solve_fine<NPROL, 8, false, 2><<<cdiv(blkEnd - blk0, 2), 128, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc,
                                                                               begin1, z, nullptr, nullptr);
    } else if (var == 7) {
        k_solve_fine1c<NPROL><<<blkEnd - blk0, 64, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z);
    } else if (var == 0) {
        k_solve_fine<NPROL, 0, false><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                    nullptr, nullptr);
    } else {
        k_solve_fine<NPROL, 1, false><<<g, kApplyThreads, 0, s>>>(inv, blk0, blkEnd, nV, r, vmap, zc, begin1, z,
                                                                    nullptr, nullptr);
    }
}

// The inverse loads' cache policy for a launch over nb level-0 blocks.  The
// default form (6) loads them nontemporal: at 1M they are 630 MB, read once
// per apply, more than the 256 MiB Infinity Cache keeps.  Where they and an
// apply's vectors fit in 192 MiB (256k: 158 MB; a world-8 rank of 1M: 76 MB),
// default-policy loads (8) let the Infinity Cache keep them from one apply to
// the next: 256k 31.35 -> 30.51 us per apply, PCG 0.0753 -> 0.0729
// ms/iteration; 1M 110.9 -> 125.1 us (profiles/round5/ab/fine_inv_policy/).
// Bitwise equal.  MAS_INV_RESIDENT=0/1 forces either.
static int fine_var(const mas_context* h, int nb) {
    if (h->fineVariant != 6) return h->fineVariant;
    const size_t bytes = (size_t)nb * (kBlockFloats * 4 + 32 * 48);
    const bool resident = h->invResident >= 0 ? h->invResident != 0 : bytes <= ((size_t)192 << 20);
    return resident ? 8 : 6;
}

// level-0 blocks [blk0, blkEnd) with prolongation of min(L,4)-1 coarse levels
// (rzPart: the PCG hooks, see solve_fine_body)
void launch_fine(mas_context* h, int blk0, int blkEnd, const float4* r, float4* z, hipStream_t s,
                 const int* done, double* rzPart) {
    const int L = h->L;
    const int g = cdiv(blkEnd - blk0, kApplyThreads / 64);
    if (g <= 0) return;
    const float4* inv = P<float4>(h->inv);
    const int4* vmap = P<int4>(h->vmap);
    const float4* zc = P<float4>(h->Zc);
    const int begin1 = h->levelSize[3], nV = h->nV, var = fine_var(h, blkEnd - blk0);
    const int w = h->rzWpb;
    auto go = [&](int v, int b0, int b1) {
        const int gg = cdiv(b1 - b0, kApplyThreads / 64);
        switch (L < 4 ? L - 1 : 3) {
            case 0: launch_fine_n<0>(v, gg, s, inv, b0, b1, nV, r, vmap, zc, begin1, z, done, rzPart, w); break;
            case 1: launch_fine_n<1>(v, gg, s, inv, b0, b1, nV, r, vmap, zc, begin1, z, done, rzPart, w); break;
            case 2: launch_fine_n<2>(v, gg, s, inv, b0, b1, nV, r, vmap, zc, begin1, z, done, rzPart, w); break;
            default: launch_fine_n<3>(v, gg, s, inv, b0, b1, nV, r, vmap, zc, begin1, z, done, rzPart, w); break;
        }
    };
    // A/B (env MAS_RESIDENT_SPLIT = K): the first K blocks' inverses with
    // default-policy loads (kept in the Infinity Cache between applies if the
    // nontemporal stream of the rest does not evict them), the rest
    // nontemporal, as two launches
    if (!rzPart && var == 6 && h->residentSplit > 0 && blkEnd - blk0 > h->residentSplit) {
        go(8, blk0, blk0 + h->residentSplit);
        go(6, blk0 + h->residentSplit, blkEnd);
        return;
    }
    go(var, blk0, blkEnd);
}

// workgroups of one fine launch of the PCG's applies (= its r.z partials)
int fine_grid(const mas_context* h) {
    const int var = fine_var(h, h->nFineBlk);
    return cdiv(h->nFineBlk, var == 6 ? h->rzWpb : var == 8 ? 4 : kApplyThreads / 64);
}

// coarse levels lFirst..L-1: level 1 from the vertices (k_coarse_l1), level
// 2 from R1 (k_coarse_up), levels >= 3 in one k_coarse_deep launch (R folded
// from R1 in the reference's order, k_coarse.hip).  (Levels >= 2 in
// one workgroup separated by barriers measured 99 us at 1M: a 1024-thread
// workgroup caps the block solve at 128 VGPRs and it spills; fewer waves
// serialise the blocks.)
void launch_coarse_levels(mas_context* h, int lFirst, const float4* d_r, hipStream_t s) {
    const float4* inv = P<float4>(h->inv);
    float4* rc = P<float4>(h->Rc);
    float4* zc = P<float4>(h->Zc);
    const int begin1 = h->levelSize[3];
    // grouped level 3 (the default): R3 from R2 like level 2 from R1; else the reference's fold over R1
    const int lTop = h->groupedR3 ? 4 : 3;
    for (int l = lFirst; l < h->L && l < lTop; ++l) {
        const int cnt = h->levelSize[2 * l], beg = h->levelSize[2 * l + 1];
        const int nb = ceil32(cnt) / 32;
        if (l == 1)
            k_coarse_l1<<<grid_for_blocks(nb), kApplyThreads, 0, s>>>(inv, beg / 32, nb, cnt, P<int>(h->l1src), d_r,
                                                                      rc, zc, begin1, h->applyDone);
        else
            k_coarse_up<<<grid_for_blocks(nb), kApplyThreads, 0, s>>>(inv, beg / 32, nb, cnt, P<int2>(h->members),
                                                                      h->levelSize[2 * (l - 1) + 1], rc, zc, begin1,
                                                                      h->applyDone);
    }
    if (h->L >= 4 && !h->groupedR3) launch_coarse_deep(h, nullptr, nullptr, s);
}

// z[s2o[v]] += Z1[a1]; += Z2[a2]; += Z3[a3] for v in [v0, v1) -- the
// reference's CollectFinalZ order (.cpp:1706-1717) applied to z = Z0.
template <int NPROL>
__global__ __launch_bounds__(256) void k_prolong(int v0, int v1, const int4* __restrict__ vmap,
                                                 const float4* __restrict__ zc, int begin1, float4* __restrict__ z) {
    const int v = v0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= v1) return;
    const int4 m = vmap[v];
    float4 o = z[m.x];
    if (NPROL >= 1) {
        const float4 a = zc[m.y - begin1];
        o.x = __fadd_rn(o.x, a.x); o.y = __fadd_rn(o.y, a.y); o.z = __fadd_rn(o.z, a.z);
    }
    if (NPROL >= 2) {
        const float4 a = zc[m.z - begin1];
        o.x = __fadd_rn(o.x, a.x); o.y = __fadd_rn(o.y, a.y); o.z = __fadd_rn(o.z, a.z);
    }
    if (NPROL >= 3) {
        const float4 a = zc[m.w - begin1];
        o.x = __fadd_rn(o.x, a.x); o.y = __fadd_rn(o.y, a.y); o.z = __fadd_rn(o.z, a.z);
    }
    z[m.x] = o;
}

void launch_prolong(mas_context* h, int v0, int v1, float4* z, hipStream_t s) {
    const int nprol = h->L < 4 ? h->L - 1 : 3;
    const int g = cdiv(v1 - v0, 256);
    if (g <= 0 || nprol == 0) return;
    const int4* vmap = P<int4>(h->vmap);
    const float4* zc = P<float4>(h->Zc);
    const int b1 = h->levelSize[3];
    if (nprol == 1) k_prolong<1><<<g, 256, 0, s>>>(v0, v1, vmap, zc, b1, z);
    else if (nprol == 2) k_prolong<2><<<g, 256, 0, s>>>(v0, v1, vmap, zc, b1, z);
    else k_prolong<3><<<g, 256, 0, s>>>(v0, v1, vmap, zc, b1, z);
}

// Fine blocks without prolongation (z = Z0) for [blk0, blkEnd).
void launch_fine_z0(mas_context* h, int blk0, int blkEnd, const float4* r, float4* z, hipStream_t s) {
    const int g = cdiv(blkEnd - blk0, kApplyThreads / 64);
    if (g <= 0) return;
    launch_fine_n<0>(fine_var(h, blkEnd - blk0), g, s, P<float4>(h->inv), blk0, blkEnd, h->nV, r, P<int4>(h->vmap),
                     P<float4>(h->Zc), h->levelSize[3], z, nullptr, nullptr);
}

// the coarse form an apply uses: the env / config choice, else the one-launch
// tagged form at L = 3 (256k: 34.3 -> 32.3 us per apply) and at L >= 4 with
// the grouped level 3.
// With the grouped level 3 (the default) the one-launch form wins at L >= 4
// too (1M + contacts: pre-fine 17.9 -> 14.7 us, 4M tet 50.1 -> 47.5 us,
// profiles/round4/apply/); with the reference's 1 024-add level-3 fold it
// measured from 2 us faster to 6 us slower at 1M (round 3), so that mode
// keeps the two-launch form at L >= 4.
int coarse_mode(const mas_context* h) {
    if (h->coarseMode >= 0) return h->coarseMode;
    return h->L == 3 || (h->L >= 4 && h->groupedR3) ? 3 : 2;
}

// (A fused form -- the coarse levels and the level-0 blocks in one launch,
// the fine waves reading tagged coarse Z -- was measured slower at every size
// and removed: DESIGN.md section 4 "Fused apply".)

// the coarse levels of an apply (run_apply), in the form it selects
void launch_coarse_apply(mas_context* h, const float4* d_r, hipStream_t s) {
    const int mode = coarse_mode(h);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool capturing = h->L > 2 && mode == 3 &&
                           (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone);
    if (h->L > 2 && mode == 3 && !capturing && coarse1_supported(h))
        launch_coarse_one(h, d_r, s);
    else if (h->L > 2 && mode >= 2) launch_coarse_twopass(h, d_r, s);
    else if (h->L > 1) launch_coarse_levels(h, 1, d_r, s);
}

int run_apply(mas_context* h, float4* d_z, const float4* d_r, hipStream_t s) {
    if (h->L >= 4 && !h->deepOff.p) return fail(h, MAS_ERR_STATE, "apply: deep-level lists not built");
    if (h->fineBlk0 != 0 || h->fineBlk1 != h->nFineBlk)
        return fail(h, MAS_ERR_STATE, "apply: the handle was prepared for one shard (mas_set_prepare_shard); "
                                      "use the sharded apply of that shard");
    hipEvent_t* ev = nullptr;
    if (h->profiling && h->profRecorded < kProfRing) ev = &h->prof[4 * h->profRecorded++];
    if (ev) hipEventRecord(ev[0], s);
    // coarse levels (mas_internal.h coarseMode); every form bitwise equal.  The
    // one-launch form's tags carry a host-side epoch, which a graph capture
    // would freeze: a capturing stream gets the two-launch form.
    launch_coarse_apply(h, d_r, s);
    if (ev) hipEventRecord(ev[1], s);
    launch_fine(h, 0, h->nFineBlk, d_r, d_z, s, h->applyDone, h->applyRzPart);
    if (ev) hipEventRecord(ev[2], s);
    if (ev) hipEventRecord(ev[3], s);
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "apply kernels");
}

// l1src[P][j] = original id of lane j of P's bank if that lane is a child of
// level-1 node P, else -1 (P = level-1 local id; padding nodes all -1).
__global__ __launch_bounds__(256) void k_l1src(int n1Pad, int n1, const int2* __restrict__ members,
                                               const int* __restrict__ s2o, int* __restrict__ l1src) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n1Pad * 32) return;
    const int P = t >> 5, j = t & 31;
    int id = -1;
    if (P < n1) {
        const int2 mb = members[P];
        if (((unsigned)mb.y >> j) & 1u) id = s2o[mb.x * 32 + j];
    }
    l1src[t] = id;
}

int build_l1src(mas_context* h, hipStream_t s) {
    if (h->L < 2) return MAS_OK;
    const int n1 = h->levelSize[2], n1Pad = ceil32(n1);
    int rc = ensure(h, h->l1src, (size_t)n1Pad * 32 * 4);
    if (rc) return rc;
    k_l1src<<<cdiv((long long)n1Pad * 32, 256), 256, 0, s>>>(n1Pad, n1, P<int2>(h->members), P<int>(h->s2o),
                                                             P<int>(h->l1src));
    if ((rc = hip_check(h, hipGetLastError(), "l1src"))) return rc;
    if ((rc = build_deep_lists(h, s))) return rc;  // level 3 (L >= 4)
    return build_coarse1_tables(h, s);
}

// Apply-side tables, built once per Prepare (and by mas_load_blob from the
// restored maps): members[] for every coarse node, l1src for level 1, the
// deep-level descendant lists.
int prepare_apply_tables(mas_context* h, hipStream_t s) {
    const int nV = h->nV, L = h->L;
    const int begin1 = h->levelSize[3];
    const int nCoarse = h->totalClusters - begin1;
    int rc;
    if ((rc = ensure(h, h->members, (size_t)(nCoarse > 0 ? nCoarse : 1) * 8))) return rc;
    if ((rc = hip_check(h, hipMemsetAsync(h->members.p, 0, (size_t)(nCoarse > 0 ? nCoarse : 1) * 8, s), "memset")))
        return rc;
    const int* gn = P<int>(h->goingNext);
    for (int l = 1; l < L; ++l) {
        const int nChild = l == 1 ? nV : h->levelSize[2 * (l - 1)];
        const int childBegin = l == 1 ? 0 : h->levelSize[2 * (l - 1) + 1];
        const unsigned* masks = l == 1 ? P<unsigned>(h->fineMask) : P<unsigned>(h->coarseMask) + (childBegin - begin1);
        k_members<<<cdiv(nChild, 256), 256, 0, s>>>(nChild, childBegin, masks, gn, begin1, P<int2>(h->members));
    }
    if ((rc = hip_check(h, hipGetLastError(), "apply tables"))) return rc;
    return build_l1src(h, s);
}

}  // namespace mas
