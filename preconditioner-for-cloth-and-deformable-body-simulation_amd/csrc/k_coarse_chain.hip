// k_coarse_chain.hip -- the whole coarse hierarchy of one Preconditioning
// (.cpp:1548-1696 for levels >= 1) in ONE launch.
//
// The per-level form (k_apply.hip, launch_coarse_levels) runs one launch per
// coarse level: at 1M the level-2 and level-3 launches solve 32 and 1 blocks
// and cost ~6 us each, mostly launch and dependent-load latency.  Here one
// grid of level-1 waves climbs the hierarchy by last arrival:
//
//   * one wave per level-1 block: R1 gathered from r through l1src, Z1 =
//     Inv R1 (same operations and order as k_coarse_l1);
//   * a wave that finishes a block adds 1 to the arrival counter of each parent
//     block at the next level; the wave whose add returns need-1 (it came
//     last) solves that parent block right away (R_l summed from R_{l-1} as in
//     k_coarse_up), and so on up to the top level.  No wave ever waits.
//
// R and Z of every coarse node are therefore bitwise equal to the per-level
// form; the level-0 kernel (k_solve_fine) follows as the next launch.
//
// Hand-offs inside the launch (MI355X: per-XCD L2s are not coherent, a CU's L1
// is never refreshed by another CU's stores) use the write-through form of
// cdna_hip_programming.md §6 Guideline 16 / MI355X_MICROARCH.md "Valid forms",
// table row 1: Rc/Zc are stored with 16-byte `sc1` buffer stores, every
// storing wave drains (`s_waitcnt vmcnt(0)`) before its agent-scope counter
// add, and every load of Rc in a parent solve is an `sc1` buffer load issued
// after the add returned.  Each wave signals for its own stores only.  Static
// tables (inverses, members, l1src, parent ranges, need) are plain loads.
// Counters reset themselves: the last arrival stores 0 (no other add to that
// counter happens in this launch), so nothing is re-initialised per call.
//
// Status: correct (bitwise equal, tests/test_gpu_chain.py) but NOT the
// default: at 1M + contacts the chain kernel takes 24.4 us against 10.7 +
// 2 x 6.0 = 22.7 us for the per-level launches (rocprofv3, same box), even
// with every static operand of the climb prefetched.  A level step is bound by
// the single-wave block solve (1.25 us, scripts/dev/solve_latency.hip), the
// sc1 gather and the drained write-through stores, not by launch boundaries,
// which the per-level launches already hide behind each other.  Opt in with
// MAS_COARSE_CHAIN=1.
//
// Also measured and dropped: the chain and the level-0 stream
// in ONE launch.  Beside the 630 MB inverse stream each of the chain's
// dependent round trips queues behind ~55 MB of in-flight loads (chain done
// 70-180 us into the launch instead of ~25 us), so most level-0 blocks finish
// first and need a second pass; level-0 waves polling a "coarse done" flag
// slow the chain further (fused launch 118-256 us vs 125 us for the whole
// per-level apply).
#include "block_solve.h"

namespace mas {

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t rs, int i, float x, float y, float z) {
    const v4u u = {__float_as_uint(x), __float_as_uint(y), __float_as_uint(z), 0u};
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, i * 16, 0, 16 /* sc1 */);
}
__device__ __forceinline__ float4 ld_sc1(__amdgpu_buffer_rsrc_t rs, int i) {
    const v4u u = __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, 16 /* sc1 */);
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), 0.f);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// a[l] for a wave-uniform l without dynamic indexing (which would copy the
// kernel-argument struct to scratch)
__device__ __forceinline__ int pick(const int (&a)[kMaxLevels + 1], int l) {
    int v = a[0];
#pragma unroll
    for (int k = 1; k <= kMaxLevels; ++k) v = l == k ? a[k] : v;
    return v;
}

// lane 0 adds 1 (agent scope); the value before the add, wave-uniform
__device__ __forceinline__ unsigned wave_arrive(unsigned* ptr, int lane) {
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(ptr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (unsigned)__builtin_amdgcn_readfirstlane((int)__shfl((int)old, 0));
}

}  // namespace

struct ChainParams {
    const float4* inv;
    const float4* r;
    float4* rc;           // coarse residuals, node id - begin1
    float4* zc;           // coarse solutions, node id - begin1
    unsigned ccBytes;     // bytes of rc / zc
    const int* l1src;     // 32 original child ids per level-1 node (-1: none)
    const int2* members;  // (child bank, component mask) per coarse node
    const int2* prange;   // per coarse block: parent blocks [x, y] at the next level
    const int* need;      // per coarse block of level >= 2: number of child banks
    unsigned* cnt;        // per coarse block: arrivals this apply (self-resetting)
    int nFineBlk, begin1, L, nb1;
    int lvBlk[kMaxLevels + 1];    // first global block of level l (1..L-1); lvBlk[L] = end
    int lvBegin[kMaxLevels + 1];  // first node id of level l
    int lvCnt[kMaxLevels + 1];    // nodes at level l
};

// R1 of level-1 block blk, node of lane n (lanes >= 32: zero): the children
// gathered through l1src and summed in lane order from +0 (as k_coarse_l1).
__device__ __forceinline__ float3 gather_l1(const ChainParams& p, int blk, int lane) {
    const int local = blk * 32 + (lane & 31) - p.lvBegin[1];
    const bool own = lane < 32 && local < p.lvCnt[1];
    const int4* s4 = reinterpret_cast<const int4*>(p.l1src + (size_t)local * 32);
    int src[32];
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
        const float4 v = p.r[src[j] >= 0 ? src[j] : 0];
        vx[j] = v.x;
        vy[j] = v.y;
        vz[j] = v.z;
    }
    float3 a = make_float3(0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if (src[j] >= 0) {
            a.x = __fadd_rn(a.x, vx[j]);
            a.y = __fadd_rn(a.y, vy[j]);
            a.z = __fadd_rn(a.z, vz[j]);
        }
    }
    return a;
}

// R_l of a level >= 2 node from its children R_{l-1} (handed-off bytes: sc1
// loads), in child-lane order from +0 (as k_coarse_up).  mb: the node's
// (child bank, mask), (0, 0) for padding lanes.
__device__ __forceinline__ float3 gather_up(const ChainParams& p, __amdgpu_buffer_rsrc_t rsR, int l, int2 mb) {
    const unsigned msk = (unsigned)mb.y;
    const int base = pick(p.lvBegin, l - 1) + mb.x * 32 - p.begin1;
    float vx[32], vy[32], vz[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const float4 v = ld_sc1(rsR, (msk >> j) & 1u ? base + j : 0);
        vx[j] = v.x;
        vy[j] = v.y;
        vz[j] = v.z;
    }
    float3 a = make_float3(0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if ((msk >> j) & 1u) {
            a.x = __fadd_rn(a.x, vx[j]);
            a.y = __fadd_rn(a.y, vy[j]);
            a.z = __fadd_rn(a.z, vz[j]);
        }
    }
    return a;
}

// (child bank, mask) of the level-l node owned by this lane, (0, 0) if none
__device__ __forceinline__ int2 member_of(const ChainParams& p, int blk, int l, int lane) {
    const int node = blk * 32 + (lane & 31);
    const bool own = lane < 32 && (node - pick(p.lvBegin, l)) < pick(p.lvCnt, l);
    return own ? p.members[node - p.begin1] : make_int2(0, 0);
}
__device__ __forceinline__ int2 parents_of(const ChainParams& p, int blk, int l) {
    return l < p.L - 1 ? p.prange[blk - p.nFineBlk] : make_int2(0, -1);
}

// One wave per level-1 block, then up the hierarchy by last arrival.
//
// Latency: everything static the climb needs is loaded BEFORE the block it
// follows is finished -- the first parent's inverse record, its members row
// and its parent range, and the need counts -- so a last arrival goes straight
// from its counter add to the sc1 gather of its children.  (The drain before
// the add also waits for these loads; they were issued with the gather and are
// done by then.)  One wave per SIMD (1 024 waves at 1M), so the second record
// costs no occupancy.  A block can complete two parents (its bank's components
// straddle a 32-node boundary); the second waits on a small stack and loads
// its data on demand.
__global__ __launch_bounds__(kApplyThreads, 1) void k_coarse_chain(ChainParams p) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int w = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= p.nb1) return;  // wave-uniform
    const __amdgpu_buffer_rsrc_t rsR = rsrc(p.rc, p.ccBytes), rsZ = rsrc(p.zc, p.ccBytes);
    int cur = p.lvBlk[1] + w, lvl = 1;
    float g[kRecord], tl[3];
    load_record<true>(p.inv, cur, lane, g, tl);
    int2 pr = parents_of(p, cur, lvl);
    float3 a = gather_l1(p, cur, lane);
    int s0 = -1, s1 = -1, s2 = -1, s3 = -1;  // pending second parents (blk | lvl << 28)
    for (;;) {
        // static data of the first parent, issued before this block's solve
        const bool up = lvl < p.L - 1;
        float gp[kRecord], tlp[3];
        int2 mbp = make_int2(0, 0), prp = make_int2(0, -1);
        int need0 = 0, need1 = 0;
        if (up) {
            load_record<true>(p.inv, pr.x, lane, gp, tlp);
            mbp = member_of(p, pr.x, lvl + 1, lane);
            prp = parents_of(p, pr.x, lvl + 1);
            need0 = p.need[pr.x - p.nFineBlk];
            need1 = p.need[pr.y - p.nFineBlk];
        }
        // solve this block, publish R and Z (write-through), drain
        a.x = __shfl(a.x, n);
        a.y = __shfl(a.y, n);
        a.z = __shfl(a.z, n);
        const float3 out = block_solve(g, tl, a, lane);
        const int node = cur * 32 + n;
        if (lane < 32) {
            st_sc1(rsR, node - p.begin1, a.x, a.y, a.z);
            st_sc1(rsZ, node - p.begin1, out.x, out.y, out.z);
        }
        drain();
        // arrive at the parents; continue with the first one completed
        int next = -1;
        if (up) {
            for (int q = pr.x; q <= pr.y; ++q) {
                const int c = q - p.nFineBlk;
                if (wave_arrive(p.cnt + c, lane) == (unsigned)(q == pr.x ? need0 : need1) - 1u) {
                    if (lane == 0) __hip_atomic_store(p.cnt + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (q == pr.x) next = q;
                    else { s3 = s2; s2 = s1; s1 = s0; s0 = q | ((lvl + 1) << 28); }
                }
            }
        }
        int2 mb;
        if (next >= 0) {
            cur = next;
            ++lvl;
#pragma unroll
            for (int k = 0; k < kRecord; ++k) g[k] = gp[k];
            tl[0] = tlp[0]; tl[1] = tlp[1]; tl[2] = tlp[2];
            mb = mbp;
            pr = prp;
        } else if (s0 >= 0) {
            cur = s0 & 0x0FFFFFFF;
            lvl = s0 >> 28;
            s0 = s1; s1 = s2; s2 = s3; s3 = -1;
            load_record<true>(p.inv, cur, lane, g, tl);
            mb = member_of(p, cur, lvl, lane);
            pr = parents_of(p, cur, lvl);
        } else {
            break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the sc1 loads below the add
        a = gather_up(p, rsR, lvl, mb);
    }
}

// ---- Prepare-time tables -------------------------------------------------

__global__ __launch_bounds__(256) void k_chain_init(int nCoarseBlk, int2* __restrict__ prange, int* __restrict__ need,
                                                    unsigned* __restrict__ cnt) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= nCoarseBlk) return;
    prange[c] = make_int2(0x7FFFFFFF, -1);
    need[c] = 0;
    cnt[c] = 0u;
}

// parents of the child banks of level l (nodes [begin, begin + count)); the
// components of one bank get consecutive ids (k_assign_ids), so a bank's
// parents are the contiguous block range [min, max]
__global__ __launch_bounds__(256) void k_chain_prange(int begin, int count, int begin1, int childBlk0, int nFineBlk,
                                                      const int2* __restrict__ members, int2* __restrict__ prange) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const int node = begin + i;
    const int c = childBlk0 + members[node - begin1].x - nFineBlk;
    atomicMin(&prange[c].x, node / 32);
    atomicMax(&prange[c].y, node / 32);
}

// need[parent] = number of child banks arriving at it
__global__ __launch_bounds__(256) void k_chain_need(int blk0, int nb, int nFineBlk, const int2* __restrict__ prange,
                                                    int* __restrict__ need) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nb) return;
    const int2 pr = prange[blk0 + i - nFineBlk];
    for (int q = pr.x; q <= pr.y; ++q) atomicAdd(&need[q - nFineBlk], 1);
}

// Built from members[] after every Prepare and blob load (build_l1src).
int build_chain_tables(mas_context* h, hipStream_t s) {
    if (h->L < 2) return MAS_OK;
    const int nCoarseBlk = h->nBlk - h->nFineBlk;
    int rc;
    if ((rc = ensure(h, h->chainPrange, (size_t)nCoarseBlk * 8)) || (rc = ensure(h, h->chainNeed, (size_t)nCoarseBlk * 4)) ||
        (rc = ensure(h, h->chainCnt, (size_t)nCoarseBlk * 4)))
        return rc;
    int2* pr = P<int2>(h->chainPrange);
    int* need = P<int>(h->chainNeed);
    k_chain_init<<<cdiv(nCoarseBlk, 256), 256, 0, s>>>(nCoarseBlk, pr, need, P<unsigned>(h->chainCnt));
    const int begin1 = h->levelSize[3];
    for (int l = 2; l < h->L; ++l) {
        const int cnt = h->levelSize[2 * l], beg = h->levelSize[2 * l + 1];
        const int childBlk0 = h->levelSize[2 * (l - 1) + 1] / 32;
        k_chain_prange<<<cdiv(cnt, 256), 256, 0, s>>>(beg, cnt, begin1, childBlk0, h->nFineBlk, P<int2>(h->members), pr);
    }
    for (int l = 1; l + 1 < h->L; ++l) {
        const int nb = ceil32(h->levelSize[2 * l]) / 32, blk0 = h->levelSize[2 * l + 1] / 32;
        k_chain_need<<<cdiv(nb, 256), 256, 0, s>>>(blk0, nb, h->nFineBlk, pr, need);
    }
    return hip_check(h, hipGetLastError(), "chain tables");
}

// All coarse levels of one apply, one launch (L >= 2).
void launch_coarse_chain(mas_context* h, const float4* r, hipStream_t s) {
    ChainParams p{};
    p.inv = P<float4>(h->inv);
    p.r = r;
    p.rc = P<float4>(h->Rc);
    p.zc = P<float4>(h->Zc);
    p.begin1 = h->levelSize[3];
    p.ccBytes = (unsigned)((size_t)(h->totalClusters - p.begin1) * 16);
    p.l1src = P<int>(h->l1src);
    p.members = P<int2>(h->members);
    p.prange = P<int2>(h->chainPrange);
    p.need = P<int>(h->chainNeed);
    p.cnt = P<unsigned>(h->chainCnt);
    p.nFineBlk = h->nFineBlk;
    p.L = h->L;
    for (int l = 1; l < h->L; ++l) {
        p.lvBegin[l] = h->levelSize[2 * l + 1];
        p.lvCnt[l] = h->levelSize[2 * l];
        p.lvBlk[l] = p.lvBegin[l] / 32;
    }
    p.lvBlk[h->L] = h->totalClusters / 32;
    p.nb1 = p.lvBlk[2] - p.lvBlk[1];  // lvBlk[2] is the end when L == 2
    k_coarse_chain<<<cdiv(p.nb1, kApplyThreads / 64), kApplyThreads, 0, s>>>(p);
}

}  // namespace mas
