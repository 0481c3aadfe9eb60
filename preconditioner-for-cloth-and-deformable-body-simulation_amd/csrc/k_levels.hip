// k_levels.hip -- contact stencils and the aggregation hierarchy on the GPU
// (PrepareCollisionStencils .cpp:304-413, ReorderRealtime .cpp:415-1162).
//
// The reference emulates 32-lane warps on the CPU; here one 32-lane group of
// a wave64 is one "bank" (two banks per wave).  Bank-local state (connection
// masks for the bit-BFS) lives in LDS; cross-bank ids come from a device-wide
// exclusive scan (hipcub) -- the reference's block-prefix loop has a bug above
// 33 792 nodes per level (B-5), the scan is correct and identical below it.
// Everything here is integer work and is bit-exact with the reference.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include <functional>

#include "mas_internal.h"

namespace mas {

// ---------------------------------------------------------------------------
// contact stencils
// ---------------------------------------------------------------------------

// flag[i]: 1 = valid record, 0 = skipped (negative id, .cpp:330,359,385),
// 2 = id out of range (reference UB; reported as MAS_ERR_ARG).
// flag[i] = 1 for a record that becomes a stencil, 0 otherwise (flag[total]
// = 0 closes the scan); a record naming an out-of-range edge/face/vertex sets
// *bad, which the host reads with the stencil count (one 8-byte copy, not the
// whole flag array: that copy and a host pass over it cost ~115 us at 100k).
__global__ __launch_bounds__(256) void k_stencil_flags(const unsigned char* __restrict__ raw, int efNum, int eeNum,
                                                       int total, int nV, int nE, int nF, int* __restrict__ flag,
                                                       int* __restrict__ bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > total) return;
    if (i == total) {
        flag[i] = 0;
        return;
    }
    const int* rec = reinterpret_cast<const int*>(raw + 48 * (size_t)i);
    int a = rec[0], b = rec[1];
    int f = 1;
    if (a < 0 || b < 0) f = 0;
    else if (i < efNum) f = (a < nE && b < nF) ? 1 : 2;
    else if (i < efNum + eeNum) f = (a < nE && b < nE) ? 1 : 2;
    else f = (a < nV && b < nF) ? 1 : 2;
    if (f == 2) atomicOr(bad, 1);
    flag[i] = f == 1;
}

__global__ __launch_bounds__(256) void k_stencil_build(const unsigned char* __restrict__ raw, int efNum, int eeNum,
                                                       int total, const int* __restrict__ flag,
                                                       const int* __restrict__ slot, const int4* __restrict__ edges,
                                                       const int4* __restrict__ faces, const int* __restrict__ o2s,
                                                       int fixVfBary, DevStencil* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total || flag[i] != 1) return;
    const unsigned char* p = raw + 48 * (size_t)i;
    const int* pi = reinterpret_cast<const int*>(p);
    const float* pf = reinterpret_cast<const float*>(p);
    DevStencil s;
    int vidx[5] = {0, 0, 0, 0, 0};
    s.stiff = pf[2];
    s.dir[0] = pf[8];
    s.dir[1] = pf[9];
    s.dir[2] = pf[10];
    if (i < efNum) {  // EfSet: bary Float3 @12; .cpp:326-354
        int4 e = edges[pi[0]], f = faces[pi[1]];
        float b0 = pf[3], b1 = pf[4], b2 = pf[5];
        s.n = 5;
        s.nFirst = 2;
        vidx[0] = e.x; vidx[1] = e.y; vidx[2] = f.x; vidx[3] = f.y; vidx[4] = f.z;
        s.w[0] = b0;
        s.w[1] = __fsub_rn(1.f, b0);
        s.w[2] = -b1;
        s.w[3] = -b2;
        s.w[4] = -__fsub_rn(__fsub_rn(1.f, b1), b2);
    } else if (i < efNum + eeNum) {  // EeSet: bary Float2 @16; .cpp:355-380 (B-3 fixed)
        int4 e0 = edges[pi[0]], e1 = edges[pi[1]];
        float b0 = pf[4], b1 = pf[5];
        s.n = 4;
        s.nFirst = 2;
        vidx[0] = e0.x; vidx[1] = e0.y; vidx[2] = e1.x; vidx[3] = e1.y;
        s.w[0] = b0;
        s.w[1] = __fsub_rn(1.f, b0);
        s.w[2] = -b1;
        s.w[3] = -__fsub_rn(1.f, b1);
        s.w[4] = 0.f;
    } else {  // VfSet: bary Float2 @16, B-2 reads the float @24; .cpp:381-405
        int4 f = faces[pi[1]];
        float b0 = pf[4], b1 = pf[5], b2 = pf[6];
        s.n = 4;
        s.nFirst = 3;
        vidx[0] = f.x; vidx[1] = f.y; vidx[2] = f.z; vidx[3] = pi[0];
        s.w[0] = -b0;
        s.w[1] = -b1;
        s.w[2] = fixVfBary ? -__fsub_rn(__fsub_rn(1.f, b0), b1) : -__fsub_rn(1.f, b2);
        s.w[3] = 1.f;
        s.w[4] = 0.f;
    }
    for (int k = 0; k < 5; ++k) s.idx[k] = (k < s.n) ? o2s[vidx[k]] : 0;  // MapCollisionStencilIndices
    out[slot[i]] = s;
}

// BuildCollisionConnection, .cpp:514-563 (pCoarse == nullptr at level 0)
__global__ __launch_bounds__(256) void k_collision_connect(const DevStencil* __restrict__ st, int n,
                                                           const int* __restrict__ pCoarse,
                                                           unsigned* __restrict__ connect) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DevStencil s = st[i];
    int idx[5];
    unsigned msk[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < 5; ++k) idx[k] = (k < s.n) ? (pCoarse ? pCoarse[s.idx[k]] : s.idx[k]) : 0;
    for (int a = 0; a < s.n; ++a)
        for (int b = a + 1; b < s.n; ++b) {
            unsigned my = (unsigned)idx[a], ot = (unsigned)idx[b];
            if (my == ot) continue;
            if ((my >> 5) == (ot >> 5) && a < s.nFirst && b >= s.nFirst) {
                msk[a] |= 1u << (ot & 31);
                msk[b] |= 1u << (my & 31);
            }
        }
    // coarse levels: many stencils set the same bits of the same few nodes;
    // skip the atomic when they are all set already (OR is idempotent, so a
    // stale read only costs a redundant atomic)
    for (int k = 0; k < s.n; ++k)
        if (msk[k] && (connect[idx[k]] & msk[k]) != msk[k]) atomicOr(&connect[idx[k]], msk[k]);
}

// ---------------------------------------------------------------------------
// aggregation hierarchy
// ---------------------------------------------------------------------------

// BuildConnectMaskL0, .cpp:447-511: same-bank neighbour bits, compact the rest.
__global__ __launch_bounds__(256) void k_connect_l0(int nV, int* __restrict__ numRem, int* __restrict__ rem,
                                                    unsigned* __restrict__ fineMask) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nV) return;
    int warp = v >> 5, num = numRem[v], nk = 0;
    unsigned msk = 1u << (v & 31);
    for (int k = 0; k < num; ++k) {
        int u = rem[(size_t)k * nV + v];
        if ((u >> 5) == warp) msk |= 1u << (u & 31);
        else rem[(size_t)(nk++) * nV + v] = u;
    }
    numRem[v] = nk;
    fineMask[v] = msk;
}

// BuildConnectMaskLx, .cpp:743-871.  Every member of a level-0 component maps
// to the same level-l node, so OR-ing each vertex's same-bank bits straight
// into nextMask[coarse] is the reference's per-component OR (see oracle).
// Consecutive vertices share their level-l node (32 per level-1 node, ~32^l
// per level-l node), so one atomicOr per lane put thousands of atomics on one
// word at the upper levels (85 us per level at 1M): the wave ORs its lanes'
// bits per distinct node first (usually one or two nodes per wave) and its
// lowest lane of each node issues the atomic, only when it would set a bit.
__global__ __launch_bounds__(256) void k_connect_lx(int nV, const int* __restrict__ cstPrev, int* __restrict__ numRem,
                                                    int* __restrict__ rem, unsigned* __restrict__ nextMask) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned cv = 0xffffffffu, msk = 0;
    if (v < nV) {
        cv = (unsigned)cstPrev[v];
        int kn = numRem[v], nk = 0;
        for (int k = 0; k < kn; ++k) {
            int u = rem[(size_t)k * nV + v];
            unsigned cu = (unsigned)cstPrev[u];
            if ((cv >> 5) == (cu >> 5)) msk |= 1u << (cu & 31);
            else rem[(size_t)(nk++) * nV + v] = u;
        }
        numRem[v] = nk;
    }
    const int lane = threadIdx.x & 63;
    for (unsigned long long todo = __ballot(msk != 0); todo;) {
        const int lead = __ffsll((long long)todo) - 1;
        const unsigned node = (unsigned)__shfl((int)cv, lead);
        unsigned part = (msk != 0 && cv == node) ? msk : 0u;
        for (int o = 32; o; o >>= 1) part |= (unsigned)__shfl_xor((int)part, o);
        todo &= ~__ballot(msk != 0 && cv == node);
        if (lane == lead && (nextMask[node] & part) != part) atomicOr(&nextMask[node], part);
    }
}

// Level sizes stay on the device while the levels are built (one host read
// after the last level): tot[l] = node count of level l >= 1 (written by
// k_assign_ids of level l - 1), level l starts at id begin_l = nv32 +
// sum_{1 <= j < l} ceil32(tot[j]).  Grids are sized for the level-0 count.
__device__ __forceinline__ int level_count(int n0, const int* tot, int level) { return level == 0 ? n0 : tot[level]; }
__device__ __forceinline__ int level_begin(const int* tot, int level, int nv32) {
    int b = nv32;
    for (int j = 1; j < level; ++j) b += (tot[j] + 31) / 32 * 32;
    return level == 0 ? 0 : b;
}

// PreparePrefixSumL0 (.cpp:565-628) / NextLevelCluster (.cpp:873-961):
// per-bank bit-BFS closure from each lane, leader = lowest lane of its mask,
// leaders counted per bank; save (levels >= 1 below the top): the closed masks
// also go to the level's slice of coarseMask (the apply's child lists).
__global__ __launch_bounds__(256) void k_bank_closure(int n0, const int* __restrict__ tot, int level, int nv32,
                                                      unsigned* __restrict__ masks, int* __restrict__ counts,
                                                      unsigned* __restrict__ save) {
    __shared__ unsigned cache[256];
    const int n = level_count(n0, tot, level);
    const int t = threadIdx.x, lane = t & 31, gbase = t & ~31;
    const int c = blockIdx.x * 256 + t;
    cache[t] = (1u << lane) | (c < n ? masks[c] : 0u);
    __syncthreads();
    bool leader = false;
    if (c < n) {
        unsigned m = cache[t], visited = 1u << lane;
        while (m != 0xFFFFFFFFu) {
            unsigned todo = visited ^ m;
            if (!todo) break;
            unsigned nxt = (unsigned)__ffs(todo) - 1u;
            visited |= 1u << nxt;
            m |= cache[gbase + nxt];
        }
        masks[c] = m;
        if (save) save[level_begin(tot, level, nv32) - nv32 + c] = m;
        leader = __popc(m & ((1u << lane) - 1u)) == 0;
    }
    unsigned long long b = __ballot(leader);
    if (lane == 0 && (c & ~31) < n) counts[c >> 5] = __popc((unsigned)(b >> (t & 32)));
}

// BuildLevel1 (.cpp:630-740) / PrefixSumLx (.cpp:963-1072): cluster id =
// bank prefix + rank of the lowest lane of the component among the leaders.
__global__ __launch_bounds__(256) void k_assign_ids(int n0, int level, int nv32, unsigned* __restrict__ masks,
                                                    const int* __restrict__ prefix, const int* __restrict__ counts,
                                                    int* __restrict__ cst0, int* __restrict__ goingNext,
                                                    int* __restrict__ levelTotal) {
    const int n = level_count(n0, levelTotal, level), begin = level_begin(levelTotal, level, nv32);
    const int nBanks = (n + 31) / 32;
    const int t = threadIdx.x, lane = t & 31;
    const int c = blockIdx.x * 256 + t;
    unsigned m = c < n ? masks[c] : 0u;
    bool leader = (c < n) && __popc(m & ((1u << lane) - 1u)) == 0;
    unsigned long long b = __ballot(leader);
    unsigned elected = (unsigned)(b >> (t & 32));
    if (c < n) {
        unsigned lead = (unsigned)__ffs(m) - 1u;
        int id = prefix[c >> 5] + __popc(elected & ((1u << lead) - 1u));
        if (level == 0) {
            cst0[c] = id;                       // m_CoarseSpaceTables[0][vid]
            goingNext[c] = id + nv32;           // m_goingNext[vid]
        } else {
            masks[c] = (unsigned)id;            // m_nextConnectMsk[vid] := local id
            goingNext[begin + c] = id + begin + ((n + 31) / 32) * 32;
        }
    }
    if (c == 0) levelTotal[level + 1] = nBanks ? prefix[nBanks - 1] + counts[nBanks - 1] : 0;
}

// ComputeNextLevel, .cpp:1074-1084
__global__ __launch_bounds__(256) void k_next_level(int nV, const int* __restrict__ cstPrev,
                                                    const unsigned* __restrict__ ids, int* __restrict__ cstCur) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < nV) cstCur[v] = (int)ids[cstPrev[v]];
}

// AggregationKernel, .cpp:1092-1162, plus the per-vertex apply record
// vmap[v] = {s2o[v], ancestor ids at levels 1..3}.
__global__ __launch_bounds__(256) void k_vertex_maps(int nV, int L, const int* __restrict__ s2o,
                                                     const int* __restrict__ goingNext, int4* __restrict__ coarseTables,
                                                     int4* __restrict__ vmap) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nV) return;
    int a[4] = {0, 0, 0, 0};
    int cur = v;
    for (int l = 0; l < L - 1 && l < 4; ++l) {
        cur = goingNext[cur];
        a[l] = cur;
    }
    coarseTables[v] = make_int4(a[0], a[1], a[2], a[3]);
    vmap[v] = make_int4(s2o[v], a[0], a[1], a[2]);
}

// ---------------------------------------------------------------------------
// incremental level maps: do the contact stencils change the mesh hierarchy?
// ---------------------------------------------------------------------------
//
// The level-(l+1) nodes are the connected components, inside each level-l
// bank, of the mesh edges plus the contact pairs mapped to level l
// (BuildCollisionConnection .cpp:514-563 ORs a stencil's first x second
// primitive pairs into the connect masks).  While levels 0..l-1 are unchanged
// (same ids as the contact-free hierarchy), the mesh edges at level l are the
// contact-free ones, so level l changes iff some pair maps to two different
// nodes of one bank that lie in different contact-free components -- the
// pair's bit is missing from the closed mask of its first node.  A pair that
// joins nodes of one component merges nothing and maps to one node above.
// flag[0] = the lowest level a pair changes (atomicMin; init >= L: none).
struct HierCheckArgs {
    const unsigned* fine;         // closed level-0 masks (contact-free)
    const unsigned* coarseMask;   // closed masks of levels >= 1 at (begin_l - nv32) + local id
    const int* cst;               // contact-free CoarseSpaceTables [L][nV]
    int maskBase[kMaxLevels];     // begin_l - nv32 (l >= 1)
    int L, nV;
};
__global__ __launch_bounds__(256) void k_hier_check(const DevStencil* __restrict__ st, int n, HierCheckArgs a,
                                                    int* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DevStencil s = st[i];
    // every vertex's node at every level first (independent loads), so the
    // walk below waits for one round trip instead of one per level
    // (static indices throughout: the arrays stay in registers)
    unsigned node[5][kMaxLevels];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        node[k][0] = (unsigned)s.idx[k];
#pragma unroll
        for (int l = 1; l < kMaxLevels; ++l)
            node[k][l] = k < s.n && l < a.L ? (unsigned)a.cst[(size_t)(l - 1) * a.nV + s.idx[k]] : 0u;
    }
    int dirty = a.L;
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
        for (int y = 1; y < 5; ++y) {
            if (!(y > x && x < s.nFirst && y >= s.nFirst && y < s.n)) continue;
#pragma unroll
            for (int l = 0; l < kMaxLevels; ++l) {
                if (l >= a.L || l >= dirty) break;
                const unsigned my = node[x][l], ot = node[y][l];
                if (my == ot) break;             // one node from here up
                if ((my >> 5) != (ot >> 5)) continue;  // not connected at this level
                const unsigned m = l ? a.coarseMask[a.maskBase[l] + my] : a.fine[my];
                if (!((m >> (ot & 31)) & 1u)) dirty = l;  // joins two components
                break;                           // same component: one node above
            }
        }
    if (dirty < a.L) atomicMin(flag, dirty);
}

// flag |= (a != b) over n ints: the CSR ranges the cached coarse records index
// off9 with, against this Prepare's
__global__ __launch_bounds__(256) void k_ranges_differ(const int* __restrict__ a, const int* __restrict__ b, int n,
                                                       int* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool d = i < n && a[i] != b[i];
    if (__ballot(d) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------

static int scan_counts(mas_context* h, const int* counts, int* prefix, int n, hipStream_t s) {
    if (h->sortImpl) return rs_exclusive_scan(h, counts, prefix, n, s, "exclusive scan");
    size_t tmp = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, counts, prefix, n, s);
    int rc = ensure(h, h->cubTemp, tmp);
    if (rc) return rc;
    return hip_check(h, hipcub::DeviceScan::ExclusiveSum(h->cubTemp.p, tmp, counts, prefix, n, s), "exclusive scan");
}


// Contact records and their count arrays may live on the host or on the
// device (e.g. straight from a GPU collision-detection pass):
// totals are read with one 4-byte copy of unified addressing, records are
// staged with hipMemcpyDefault.
static long long count_total(mas_context* h, const unsigned* c, int at) {
    if (!c) return 0;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, c) == hipSuccess && a.type == hipMemoryTypeDevice) {
        unsigned v = 0;
        if (hipMemcpy(&v, c + at, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        return v;
    }
    (void)hipGetLastError();  // a host pointer may leave "invalid value" behind
    return c[at];
}

int build_stencils(mas_context* h, const void* ef, const void* ee, const void* vf, const unsigned* efC,
                   const unsigned* eeC, const unsigned* vfC, hipStream_t s) {
    long long efNum = count_total(h, efC, h->nE), eeNum = count_total(h, eeC, h->nE),
              vfNum = count_total(h, vfC, h->nV);
    if (efNum < 0 || eeNum < 0 || vfNum < 0) return fail(h, MAS_ERR_HIP, "reading contact counts");
    long long total = efNum + eeNum + vfNum;
    const long long maxStencil = (long long)h->nV * 32;  // .cpp:187-188
    h->nStencil = h->nStencilEF = 0;
    if (total <= 0) return MAS_OK;
    if ((efNum && !ef) || (eeNum && !ee) || (vfNum && !vf)) return fail(h, MAS_ERR_ARG, "contact records missing");
    if ((efNum || eeNum) && !h->edges.p) return fail(h, MAS_ERR_ARG, "EF/EE contacts need m_edges");
    if ((efNum || vfNum) && !h->faces.p) return fail(h, MAS_ERR_ARG, "EF/VF contacts need m_faces");
    if (total > maxStencil) {
        // .cpp:312-316: the reference truncates and prints
        std::fprintf(stderr, "stencil size %lld exceed max stencils num  %lld\n", total, maxStencil);
        total = maxStencil;
        if (efNum > total) efNum = total;
        if (efNum + eeNum > total) eeNum = total - efNum;
        vfNum = total - efNum - eeNum;
    }
    int rc;
    if ((rc = ensure(h, h->rawContacts, (size_t)total * 48)) || (rc = ensure(h, h->stencilFlags, (size_t)(total + 1) * 4)) ||
        (rc = ensure(h, h->stencilSlots, (size_t)total * 4 + 16)) ||
        (rc = ensure(h, h->stencils, (size_t)total * sizeof(DevStencil))))
        return rc;
    unsigned char* raw = P<unsigned char>(h->rawContacts);
    if (efNum && (rc = hip_check(h, hipMemcpyAsync(raw, ef, efNum * 48, hipMemcpyDefault, s), "stage ef"))) return rc;
    if (eeNum && (rc = hip_check(h, hipMemcpyAsync(raw + efNum * 48, ee, eeNum * 48, hipMemcpyDefault, s), "stage ee")))
        return rc;
    if (vfNum && (rc = hip_check(h, hipMemcpyAsync(raw + (efNum + eeNum) * 48, vf, vfNum * 48, hipMemcpyDefault, s),
                                 "stage vf")))
        return rc;
    const int n = (int)total;
    int* slots = P<int>(h->stencilSlots);  // [0, n]: exclusive scan of the flags; [n + 1]: the bad-record word
    if ((rc = hip_check(h, hipMemsetAsync(slots + n + 1, 0, 4, s), "clear bad-record word"))) return rc;
    k_stencil_flags<<<cdiv(n + 1, 256), 256, 0, s>>>(raw, (int)efNum, (int)eeNum, n, h->nV, h->nE, h->nF,
                                                     P<int>(h->stencilFlags), slots + n + 1);
    // deterministic compaction == the reference's atomic slot counter at CPU_THREAD_NUM=1
    if ((rc = scan_counts(h, P<int>(h->stencilFlags), slots, n + 1, s))) return rc;
    int head[2] = {0, 0};  // stencil count, bad-record word
    if ((rc = read_back(h, s, {slots + n, slots + n + 1}, head))) return rc;
    if (head[1]) return fail(h, MAS_ERR_ARG, "contact record references an out-of-range edge/face/vertex");
    const int valid = head[0];
    k_stencil_build<<<cdiv(n, 256), 256, 0, s>>>(raw, (int)efNum, (int)eeNum, n, P<int>(h->stencilFlags),
                                                 P<int>(h->stencilSlots), P<int4>(h->edges), P<int4>(h->faces),
                                                 P<int>(h->o2s), h->cfg.fix_vf_bary, P<DevStencil>(h->stencils));
    h->nStencil = valid;
    h->nStencilEF = (int)std::min<long long>(valid, efNum);  // the EF stencils come first (5 vertices each)
    return hip_check(h, hipGetLastError(), "stencil kernels");
}

// ReorderRealtime, .cpp:415-445; contacts = false: the contact-free (mesh)
// hierarchy, the stencils ignored
static int build_levels(mas_context* h, hipStream_t s, const std::function<int()>& beforeRead, bool contacts) {
    const int nV = h->nV, L = h->L, nv32 = ceil32(nV);
    const int nB0 = nv32 / 32;
    const int nSt = contacts ? h->nStencil : 0;
    int rc;
    // .cpp:74-75: fresh copies of the ELL neighbour table (compacted level by level below)
    if ((rc = hip_check(h, hipMemcpyAsync(h->nbrRem.p, h->nbr.p, (size_t)h->maxNbr * nV * 4, hipMemcpyDeviceToDevice, s),
                        "copy nbr")) ||
        (rc = hip_check(h, hipMemcpyAsync(h->nbrNumRem.p, h->nbrNum.p, (size_t)nV * 4, hipMemcpyDeviceToDevice, s),
                        "copy nbrNum")))
        return rc;
    if ((rc = ensure(h, h->fineMask, (size_t)nv32 * 4)) || (rc = ensure(h, h->nextMask, (size_t)nv32 * 4)) ||
        (rc = ensure(h, h->bankCount, (size_t)(nB0 + 1) * 4)) || (rc = ensure(h, h->bankPrefix, (size_t)(nB0 + 1) * 4)) ||
        (rc = ensure(h, h->levelTotal, 16 * 4)) || (rc = ensure(h, h->cst, (size_t)L * nV * 4)) ||
        (rc = ensure(h, h->goingNext, (size_t)(L + 1) * nv32 * 4)) || (rc = ensure(h, h->vmap, (size_t)nV * 16)) ||
        (rc = ensure(h, h->coarseTables, (size_t)nV * 16)) ||
        (rc = ensure(h, h->coarseMask, (size_t)L * nv32 * 4)))
        return rc;
    std::fill(h->levelSize, h->levelSize + 18, 0);
    int* cst = P<int>(h->cst);
    int* gn = P<int>(h->goingNext);
    unsigned* fine = P<unsigned>(h->fineMask);
    unsigned* next = P<unsigned>(h->nextMask);
    int* cnt = P<int>(h->bankCount);
    int* pre = P<int>(h->bankPrefix);
    int* tot = P<int>(h->levelTotal);
    const DevStencil* st = P<DevStencil>(h->stencils);
    const int g = cdiv(nV, 256);
    if ((rc = hip_check(h, hipMemsetAsync(gn, 0, (size_t)(L + 1) * nv32 * 4, s), "memset goingNext"))) return rc;

    // level 0 -> 1
    k_connect_l0<<<g, 256, 0, s>>>(nV, P<int>(h->nbrNumRem), P<int>(h->nbrRem), fine);
    if (nSt) k_collision_connect<<<cdiv(nSt, 256), 256, 0, s>>>(st, nSt, nullptr, fine);
    k_bank_closure<<<cdiv(nV, 256), 256, 0, s>>>(nV, tot, 0, nv32, fine, cnt, nullptr);
    if ((rc = scan_counts(h, cnt, pre, nB0, s))) return rc;
    k_assign_ids<<<cdiv(nV, 256), 256, 0, s>>>(nV, 0, nv32, fine, pre, cnt, cst, gn, tot);

    // levels >= 1 (.cpp:427-440): sizes on the device, grids for <= nV nodes
    // (a level has at most as many nodes as vertices; banks past its count are
    // never read), no host round trip until the hierarchy is complete
    for (int level = 1; level < L; ++level) {
        const int* prev = cst + (size_t)(level - 1) * nV;
        if ((rc = hip_check(h, hipMemsetAsync(next, 0, (size_t)nv32 * 4, s), "memset nextMask"))) return rc;
        k_connect_lx<<<g, 256, 0, s>>>(nV, prev, P<int>(h->nbrNumRem), P<int>(h->nbrRem), next);
        if (nSt) k_collision_connect<<<cdiv(nSt, 256), 256, 0, s>>>(st, nSt, prev, next);
        // keeps the level-l component masks (the apply's child lists, and the
        // contact check's closed masks, k_hier_check) before k_assign_ids
        // overwrites them with ids
        k_bank_closure<<<cdiv(nV, 256), 256, 0, s>>>(0, tot, level, nv32, next, cnt, P<unsigned>(h->coarseMask));
        if ((rc = scan_counts(h, cnt, pre, nB0, s))) return rc;
        k_assign_ids<<<cdiv(nV, 256), 256, 0, s>>>(0, level, nv32, next, pre, cnt, nullptr, gn, tot);
        k_next_level<<<g, 256, 0, s>>>(nV, prev, next, cst + (size_t)level * nV);
    }
    int totals[kMaxLevels + 2] = {};
    // the host's other work (run_level0_early's launches) while the levels build
    if (beforeRead && (rc = beforeRead())) return rc;
    if ((rc = read_back(h, s, {tot, tot + 1, tot + 2, tot + 3, tot + 4, tot + 5}, totals))) return rc;
    h->levelSize[2] = totals[1];
    h->levelSize[3] = nv32;
    for (int level = 1; level < L; ++level) {
        h->levelSize[2 * (level + 1)] = totals[level + 1];
        h->levelSize[2 * (level + 1) + 1] = h->levelSize[2 * level + 1] + ceil32(totals[level]);
    }
    h->totalClusters = h->levelSize[2 * L + 1];  // TotalNodes, .cpp:1086-1090
    h->nBlk = h->totalClusters / 32;
    // (set by run_prepare before the early path forked; its worker reads it)
    k_vertex_maps<<<g, 256, 0, s>>>(nV, L, P<int>(h->s2o), gn, P<int4>(h->coarseTables), P<int4>(h->vmap));
    return hip_check(h, hipGetLastError(), "level kernels");
}

// the hierarchy maps of the live slot <-> the spare slot (mas_context)
static void swap_hier_slots(mas_context* h) {
    std::swap(h->cst, h->spCst);
    std::swap(h->goingNext, h->spGn);
    std::swap(h->vmap, h->spVmap);
    std::swap(h->coarseTables, h->spCoarseTables);
    std::swap(h->fineMask, h->spFine);
    std::swap(h->coarseMask, h->spCoarseMask);
}

// Incremental level maps: the contact-free hierarchy is built
// once per sort; a Prepare whose stencils do not change it (k_hier_check, one
// host read) reuses it as is, and everything derived from it alone (records,
// term lists, apply tables: hierId) is reused too; otherwise the levels are
// rebuilt with the contacts, the contact-free hierarchy kept in the spare
// slot.  Either way the maps equal a full rebuild's, bit for bit.
int run_levels(mas_context* h, hipStream_t s, const int* d_ranges, const std::function<int()>& beforeRead) {
    const int L = h->L, nV = h->nV, nv32 = ceil32(nV);
    int rc;
    h->rangesChanged = true;
    h->lastHierBuilt = true;  // until a reuse below says otherwise
    if (!h->hierCache) {  // A/B (MAS_HIER_CACHE=0): the full build every Prepare
        h->meshHierValid = h->liveIsMesh = false;
        h->hierId = ++h->hierCounter;
        h->lastHierDirty = -1;
        return build_levels(h, s, beforeRead, true);
    }
    bool hooked = false;
    auto hook = [&]() -> int {
        if (hooked || !beforeRead) return MAS_OK;
        hooked = true;
        return beforeRead();
    };
    bool justBuilt = false;
    if (!h->meshHierValid) {  // first Prepare after a sort: the contact-free hierarchy
        justBuilt = true;
        if ((rc = build_levels(h, s, hook, false))) return rc;
        std::copy(h->levelSize, h->levelSize + 18, h->meshLevelSize);
        h->meshHierValid = h->liveIsMesh = true;
        h->meshHierId = h->hierId = ++h->hierCounter;
        h->lastHierDirty = L;
        if (h->nStencil == 0) return hook();
    }
    // does this Prepare's contact set change it?  (and do the CSR ranges
    // differ from the ones the cached records index off9 with?)
    const bool live = h->liveIsMesh;
    const bool wantRanges = h->recHierId == h->meshHierId && h->recRanges.bytes >= (size_t)(nV + 1) * 4;
    int flags[2] = {L, 1};
    if (h->nStencil > 0 || wantRanges) {
        if ((rc = ensure(h, h->hierFlags, 16))) return rc;
        int* f = P<int>(h->hierFlags);
        if ((rc = hip_check(h, hipMemsetD32Async(f, L, 1, s), "hier flags")) ||
            (rc = hip_check(h, hipMemsetD32Async(f + 1, 0, 1, s), "hier flags")))
            return rc;
        if (h->nStencil > 0) {
            HierCheckArgs a{};
            a.fine = P<unsigned>(live ? h->fineMask : h->spFine);
            a.coarseMask = P<unsigned>(live ? h->coarseMask : h->spCoarseMask);
            a.cst = P<int>(live ? h->cst : h->spCst);
            for (int l = 1; l < L; ++l) a.maskBase[l] = h->meshLevelSize[2 * l + 1] - nv32;
            a.L = L;
            a.nV = nV;
            k_hier_check<<<cdiv(h->nStencil, 256), 256, 0, s>>>(P<DevStencil>(h->stencils), h->nStencil, a, f);
        }
        if (wantRanges)
            k_ranges_differ<<<cdiv(nV + 1, 256), 256, 0, s>>>(d_ranges, P<int>(h->recRanges), nV + 1, f + 1);
        if ((rc = hip_check(h, hipGetLastError(), "hierarchy check")) || (rc = hook()) ||
            (rc = read_back(h, s, {f, f + 1}, flags)))
            return rc;
    }
    if ((rc = hook())) return rc;
    h->rangesChanged = !wantRanges || flags[1] != 0;
    if (flags[0] >= L) {  // unchanged: the contact-free hierarchy is this Prepare's
        h->lastHierBuilt = justBuilt;  // swapping slots is not a build
        if (!h->liveIsMesh) swap_hier_slots(h);
        h->liveIsMesh = true;
        std::copy(h->meshLevelSize, h->meshLevelSize + 18, h->levelSize);
        h->totalClusters = h->levelSize[2 * L + 1];
        h->nBlk = h->totalClusters / 32;
        // nFineBlk: set by run_prepare before the early path forked (its worker reads it)
        h->hierId = h->meshHierId;
        h->lastHierDirty = L;
        return MAS_OK;
    }
    // level flags[0] changes: rebuild with the contacts, the contact-free maps kept in the spare slot
    if (h->liveIsMesh) swap_hier_slots(h);
    h->liveIsMesh = false;
    h->lastHierDirty = flags[0];
    h->hierId = ++h->hierCounter;
    return build_levels(h, s, {}, true);
}

}  // namespace mas
