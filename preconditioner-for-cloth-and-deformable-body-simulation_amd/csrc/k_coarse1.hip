// k_coarse1.hip -- every coarse level of one Preconditioning in ONE launch
// (BuildResidualHierarchy .cpp:1548-1598, SchwarzLocalXSym .cpp:1600-1696
// for levels 1..min(L-1, 3)); coarseMode 3.
//
// The two-launch form (k_coarse.hip) starts the level-3 fold only after the
// whole level-1 restriction, a kernel boundary and the dispatch of the second
// launch, and its level-1/2 solves wait for the same boundary.  Here one launch
// of single-wave workgroups holds four roles, producers first in the grid:
//
//   bank waves, one per level-1 bank (= level-1 block): R1 of its 32 nodes
//       from r (lane order from +0), R2 of the level-2 nodes whose children are
//       its components (level-1 id order from +0) -- the two-launch form's
//       sums, bit for bit; R1 is published at its place in its level-3
//       ancestor's descendant list, R2 at its level-2 node; then the bank's own
//       level-1 block is solved (Z1) from the R1 already in registers.
//   fold waves (L >= 4), one per level-3 node T: T's descendant list in
//       level-1 id order is polled chunk by chunk; the valid prefix is folded
//       left from +0 (the reference's R3, .cpp:1577-1590) while later banks are
//       still restricting; R3 is published.
//   level-2 solve waves, one per level-2 block: the block's inverse in flight
//       while its 32 R2 are polled, then Z2.
//   level-3 solve waves (L >= 4), one per level-3 block: the same for R3.
//
// Hand-offs carry their own validity: each of x, y, z travels in a 64-bit
// word (value bits | apply epoch << 32) written with an agent-scope atomic
// store and read with an agent-scope atomic load.  A 64-bit atomic is
// single-copy atomic, so a word whose tag is this apply's epoch holds this
// apply's value whatever order the words land in: no flag, no store drain, no
// arrival counter, and a consumer's loads can be in flight before the
// producer has finished.  (The first one-launch form published with drained
// write-through stores, per-bank flags and arrival counters: every hand-off
// paid a drain and two round trips, 26.7 vs 18.5 us before the fine kernel at
// 1M + contacts, profiles/round3/ab/coarse1_1M.json.)  On gfx942/gfx950 the
// agent-scope atomics are sc1 accesses performed at memory-side coherence
// (deep_fold.h header), so no stale L2 line is consulted.
//
// The epoch is a per-handle apply counter passed by value (tags are zeroed at
// Prepare and on wrap-around); a stream being captured into a graph would
// freeze it, so run_apply selects the two-launch form while capturing.
// Consumers sit after their producers in the grid, so every producer a
// resident consumer waits for has been dispatched; every wait is bounded.
#include "block_solve.h"
#include "deep_fold.h"

namespace mas {

// Diagnostic stamps (probe build only): lane 0 of a wave writes the 100 MHz
// wall clock into g_probe1[kind][slot][k] (kind 0: level-3 fold waves by node,
// kind 1: bank waves by bank, kind 2: solve waves by block); mas_probe1_dump
// reads them back (scripts/dev/probe_coarse1.py).
#ifdef MAS_PROBE
__device__ unsigned long long g_probe1[3 * 8192 * 8];
#define C1_STAMP(kind, slot, k)                                                                          \
    do {                                                                                                 \
        unsigned long long t_;                                                                           \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        if ((threadIdx.x & 63) == 0 && (slot) < 8192) g_probe1[((kind) * 8192 + (slot)) * 8 + (k)] = t_; \
    } while (0)
#else
#define C1_STAMP(kind, slot, k) \
    do {                        \
    } while (0)
#endif

constexpr int kFoldStep = 512;     // list entries polled per fold step (8 per lane)

// x, y, z of one hand-off, one tagged 64-bit word each (TagWord)
struct Tag3 {
    unsigned long long w[3];
};

__device__ __forceinline__ void st_tag(Tag3* p, float x, float y, float z, unsigned e) {
    const unsigned long long hi = (unsigned long long)e << 32;
    __hip_atomic_store(&p->w[0], hi | __float_as_uint(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p->w[1], hi | __float_as_uint(y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p->w[2], hi | __float_as_uint(z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ld_tag(const Tag3* p, unsigned long long (&v)[3]) {
    v[0] = __hip_atomic_load(&p->w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v[1] = __hip_atomic_load(&p->w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v[2] = __hip_atomic_load(&p->w[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tag_ok(const unsigned long long (&v)[3], unsigned e) {
    return (unsigned)(v[0] >> 32) == e && (unsigned)(v[1] >> 32) == e && (unsigned)(v[2] >> 32) == e;
}
__device__ __forceinline__ float tag_val(unsigned long long w) { return __uint_as_float((unsigned)w); }

struct Coarse1Args {
    const float4* inv;
    const float4* r;
    const int* l1src;     // 32 original vertex ids (or -1) per level-1 node
    const int4* l1info;   // per level-1 node: (parent - begin1, the parent's child mask, list slot, 0)
    float4* rc;           // R per coarse node (node id - begin1), for mas_get_coarse_residual
    float4* zc;           // Z per coarse node
    Tag3* tR1;            // level-3 list slot T * stride + i -> R1 of the i-th descendant
    Tag3* tR2;            // level-2 local id -> R2
    Tag3* tR3;            // level-3 local id -> R3
    int n1, begin1, L;
    int n2, lv2Begin, nb2;
    int n3, lv3Begin, nb3, stride;
    const int* deepOff;   // list start per level-3 node, + 1
    unsigned epoch;       // this apply's tag
    int nb1;
    int pollDelay;        // fold / solve waves: s_sleep(64) rounds before the first poll (A/B)
    int chunk;            // bank waves XCD-chunked (as k_apply.hip xcd_chunked): Morton-adjacent banks share an L2
    const int* done;      // PCG: exit at once when set
    int pollLimit;        // polls before a wait gives up (kPollLimit; < 0: give up at once, a test knob)
    int* timeouts;        // waits that gave up: this apply's z is incomplete (mas_stats.wait_timeouts)
    int* giveupHost;      // pinned host word: the epoch of an apply whose wait gave up (the next call reports it)
    const int2* members;  // grouped level 3: per coarse node (child bank, child mask); null: the reference's fold
};

// A bounded wait gave up: count it on the device (mas_stats.wait_timeouts) and
// name this apply in the handle's pinned host word with a system-scope vector
// store, which the next host call reads without synchronising (mas_capi.hip
// pending_giveup).
__device__ __forceinline__ void gave_up(const Coarse1Args& a) {
    atomicAdd(a.timeouts, 1);
    __hip_atomic_store(a.giveupHost, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

union C1Shared {
    struct {
        float svs[3][32][33];  // [component][node][child]
        float4 red[32];
    } bank;
    __attribute__((aligned(16))) float stg[3][kFoldStep];  // fold: R1 of one step, component-major
};

// ---------------------------------------------------------------------------
// level-1 bank B: R1, R2, their publication, then Z1
// ---------------------------------------------------------------------------
__device__ __forceinline__ void bank_wave(const Coarse1Args& a, int B, C1Shared& sh) {
    const int lane = threadIdx.x & 63, j = lane & 31;
    const int c0 = B * 32;
    C1_STAMP(1, B, 0);
    const int* s = a.l1src + (size_t)c0 * 32;  // l1src covers ceil32(n1) nodes
    int src[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) src[q] = s[64 * q + lane];
    const int c = c0 + j;
    const bool own = lane < 32 && c < a.n1;
    const int4 info = own ? a.l1info[c] : make_int4(0, 0, -1, 0);
    // every gather issued unconditionally (a non-child lane reads r[0] and
    // drops it): a conditional load made the compiler wait for the first
    // gather before issuing the rest, one more round trip on the chain
    float4 val[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) val[q] = a.r[src[q] >= 0 ? src[q] : 0];
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (src[q] < 0) val[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        sh.bank.svs[0][2 * q + (lane >> 5)][j] = val[q].x;
        sh.bank.svs[1][2 * q + (lane >> 5)][j] = val[q].y;
        sh.bank.svs[2][2 * q + (lane >> 5)][j] = val[q].z;
    }
    __builtin_amdgcn_wave_barrier();
    C1_STAMP(1, B, 1);
    float ax = 0.f, ay = 0.f, az = 0.f;  // R1, lane order from +0 (non-children are +0.0)
    if (own) {
#pragma unroll
        for (int k0 = 0; k0 < 32; k0 += 8) {
            float vx[8], vy[8], vz[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                vx[k] = sh.bank.svs[0][j][k0 + k];
                vy[k] = sh.bank.svs[1][j][k0 + k];
                vz[k] = sh.bank.svs[2][j][k0 + k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                ax = __fadd_rn(ax, vx[k]);
                ay = __fadd_rn(ay, vy[k]);
                az = __fadd_rn(az, vz[k]);
            }
        }
    }
    if (a.L >= 4 && !a.members && own && info.z >= 0)  // the reference-order level-3 fold's input
        st_tag(a.tR1 + info.z, ax, ay, az, a.epoch);
    if (lane < 32) sh.bank.red[j] = make_float4(ax, ay, az, 0.f);
    __builtin_amdgcn_wave_barrier();
    // R2 of the level-2 nodes whose children are this bank's components (their lowest lane)
    const unsigned pmsk = (unsigned)info.y;
    if (own && (unsigned)(__ffs(pmsk) - 1) == (unsigned)j) {
        float bx = 0.f, by = 0.f, bz = 0.f;
#pragma unroll
        for (int k0 = 0; k0 < 32; k0 += 8) {
            float4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = sh.bank.red[k0 + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool in = (pmsk >> (k0 + k)) & 1u;
                bx = __fadd_rn(bx, in ? v[k].x : 0.f);
                by = __fadd_rn(by, in ? v[k].y : 0.f);
                bz = __fadd_rn(bz, in ? v[k].z : 0.f);
            }
        }
        st_tag(a.tR2 + info.x - (a.lv2Begin - a.begin1), bx, by, bz, a.epoch);
        a.rc[info.x] = make_float4(bx, by, bz, 0.f);
    }
    if (own) a.rc[c] = make_float4(ax, ay, az, 0.f);
    C1_STAMP(1, B, 2);
    // Z1 of the bank's block from the R1 in registers (inverse loaded after the
    // publications, so the restriction's gathers do not queue behind it)
    float g[kRecord], tl[3];
    load_record<true>(a.inv, a.begin1 / 32 + B, lane, g, tl);
    const float3 out = block_solve(g, tl, make_float3(__shfl(ax, j), __shfl(ay, j), __shfl(az, j)), lane);
    if (lane < 32) a.zc[c] = make_float4(out.x, out.y, out.z, 0.f);
    C1_STAMP(1, B, 3);
}

// ---------------------------------------------------------------------------
// level-3 node T: fold R1 in level-1 id order as its banks publish
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fold_wave(const Coarse1Args& a, int T, C1Shared& sh) {
    const int lane = threadIdx.x & 63;
    C1_STAMP(0, T, 0);
    const int len = a.deepOff[T + 1] - a.deepOff[T];
    const Tag3* list = a.tR1 + (size_t)T * a.stride;
    constexpr int kQ = kFoldStep / 64;
    unsigned long long v[kQ][3];
    auto poll = [&](int e) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = e + 64 * q + lane;
            if (i < len) ld_tag(list + i, v[q]);
        }
    };
    __builtin_amdgcn_s_setprio(3);  // the fold is the launch's longest chain
    float acc = 0.f;  // lanes 0..2: x, y, z
    int e = 0, idle = 0;
    for (int d = 0; d < a.pollDelay; ++d) __builtin_amdgcn_s_sleep(64);  // nothing is published yet
    if (len > 0) poll(0);
    while (e < len) {
        // the valid prefix of this step's entries (list order = 64 q + lane)
        const int n = min(kFoldStep, len - e);
        int bad = kFoldStep;
#pragma unroll
        for (int q = kQ - 1; q >= 0; --q)
            if (64 * q + lane < n && !tag_ok(v[q], a.epoch)) bad = 64 * q + lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bad = min(bad, __shfl_xor(bad, o));
        const int p = min(bad, n);
        if (p == 0) {
            if (a.pollLimit < 0 || ++idle > a.pollLimit) {  // never hang: the fold stays incomplete, and says so
                if (lane == 0) gave_up(a);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            poll(e);
            continue;
        }
        if (e == 0) C1_STAMP(0, T, 1);
        // stage the prefix component-major, +0.0 up to whole 32-entry batches
        const int p32 = (p + 31) & ~31;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = 64 * q + lane;
            if (i < p32) {
                const bool in = i < p;
                sh.stg[0][i] = in ? tag_val(v[q][0]) : 0.f;
                sh.stg[1][i] = in ? tag_val(v[q][1]) : 0.f;
                sh.stg[2][i] = in ? tag_val(v[q][2]) : 0.f;
            }
        }
        e += p;
        if (e < len) poll(e);  // the next step's loads in flight during the fold
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 3) acc = fold_row(reinterpret_cast<const float4*>(sh.stg[lane]), p32 / 4, acc);
        __builtin_amdgcn_wave_barrier();
    }
    C1_STAMP(0, T, 2);
    const float ax = __shfl(acc, 0), ay = __shfl(acc, 1), az = __shfl(acc, 2);
    if (lane == 0) {
        st_tag(a.tR3 + T, ax, ay, az, a.epoch);
        a.rc[a.lv3Begin + T - a.begin1] = make_float4(ax, ay, az, 0.f);
    }
    C1_STAMP(0, T, 3);
}

// grouped level 3 (mas_config.reference_restriction = 0): node T's R3 is its
// children's R2 -- the lanes of one component of one level-2 bank -- folded
// in lane (= level-2 id) order from +0, as k_solve123g; lane j polls child
// j's tagged R2 until every child's has this apply's tag
__device__ __forceinline__ void fold_wave_grouped(const Coarse1Args& a, int T) {
    const int lane = threadIdx.x & 63, j = lane & 31;
    const int2 mb = a.members[a.lv3Begin + T - a.begin1];  // (level-2 bank, children)
    const bool child = lane < 32 && (((unsigned)mb.y >> j) & 1u);
    C1_STAMP(0, T, 0);
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    bool ok = !child;
    for (int d = 0; d < a.pollDelay; ++d) __builtin_amdgcn_s_sleep(64);
    for (int polls = 0; polls <= a.pollLimit; ++polls) {
        if (!ok) {
            ld_tag(a.tR2 + mb.x * 32 + j, v);
            ok = tag_ok(v, a.epoch);
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (!__all(ok) && lane == 0) gave_up(a);  // R3 from stale R2: counted
    C1_STAMP(0, T, 1);
    const float x = child ? tag_val(v[0]) : 0.f, y = child ? tag_val(v[1]) : 0.f, z = child ? tag_val(v[2]) : 0.f;
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        ax = __fadd_rn(ax, __shfl(x, k));
        ay = __fadd_rn(ay, __shfl(y, k));
        az = __fadd_rn(az, __shfl(z, k));
    }
    C1_STAMP(0, T, 2);
    if (lane == 0) {
        st_tag(a.tR3 + T, ax, ay, az, a.epoch);
        a.rc[a.lv3Begin + T - a.begin1] = make_float4(ax, ay, az, 0.f);
    }
    C1_STAMP(0, T, 3);
}

// ---------------------------------------------------------------------------
// level-2 / level-3 block: poll its 32 R, then Z = Inv R
// ---------------------------------------------------------------------------
__device__ __forceinline__ void solve_wave(const Coarse1Args& a, int blk, int lvBegin, int cnt, const Tag3* tR,
                                           int slot) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    C1_STAMP(2, slot, 0);
    float g[kRecord], tl[3];
    load_record<true>(a.inv, blk, lane, g, tl);  // in flight during the polls
    const int loc = blk * 32 + n - lvBegin;
    const bool real = lane < 32 && loc < cnt;
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    bool ok = !real;
    for (int d = 0; d < a.pollDelay; ++d) __builtin_amdgcn_s_sleep(64);
    for (int polls = 0; polls <= a.pollLimit; ++polls) {
        if (!ok) {
            ld_tag(tR + loc, v);
            ok = tag_ok(v, a.epoch);
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (!__all(ok) && lane == 0) gave_up(a);  // solved from stale R: counted
    C1_STAMP(2, slot, 1);
    // half 1 takes node n's residual from lane n (padding nodes: +0)
    const float rx = __shfl(tag_val(v[0]), n), ry = __shfl(tag_val(v[1]), n), rz = __shfl(tag_val(v[2]), n);
    const float3 out = block_solve(g, tl, make_float3(rx, ry, rz), lane);
    if (lane < 32) a.zc[blk * 32 + n - a.begin1] = make_float4(out.x, out.y, out.z, 0.f);
    C1_STAMP(2, slot, 2);
}

// grid (single-wave workgroups): [0, nb1) banks, then n3 fold waves, then nb2
// level-2 and nb3 level-3 solve waves
__global__ __launch_bounds__(64) void k_coarse1(Coarse1Args a) {
    if (a.done && *a.done) return;
    __shared__ C1Shared sh;
    int w = blockIdx.x;  // workgroup-uniform roles
    if (w < a.nb1) {  // the first nb1 workgroups: workgroup w runs on XCD w % 8
        const int full = a.nb1 & ~7;
        return bank_wave(a, a.chunk && w < full ? (w & 7) * (full >> 3) + (w >> 3) : w, sh);
    }
    w -= a.nb1;
    if (w < a.n3) return a.members ? fold_wave_grouped(a, w) : fold_wave(a, w, sh);
    w -= a.n3;
    if (w < a.nb2) return solve_wave(a, a.lv2Begin / 32 + w, a.lv2Begin, a.n2, a.tR2, w);
    w -= a.nb2;
    if (w < a.nb3) solve_wave(a, a.lv3Begin / 32 + w, a.lv3Begin, a.n3, a.tR3, a.nb2 + w);
}

// per level-1 node: its parent (local to begin1), the parent's child mask, its level-3 list slot
__global__ __launch_bounds__(256) void k_l1info(int n1, int begin1, const int* __restrict__ gn,
                                                const int2* __restrict__ members, const int* __restrict__ deepPos,
                                                int4* __restrict__ info) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= n1) return;
    const int p = gn[begin1 + c] - begin1;
    info[c] = make_int4(p, members[p].y, deepPos ? deepPos[c] : -1, 0);
}

// tagged hand-off slots: level-3 lists, then level-2 nodes, then level-3 nodes
static size_t coarse1_tags(const mas_context* h) {
    const int n2 = h->levelSize[4];
    const size_t nList = h->L >= 4 ? (size_t)deep_nodes(h) * h->deepStride : 0;
    const size_t n3 = h->L >= 4 ? (size_t)ceil32(h->levelSize[6]) : 0;
    return nList + ceil32(n2) + n3;
}

int build_coarse1_tables(mas_context* h, hipStream_t s) {
    h->coarse1Epoch = 0;
    if (h->L < 3) return MAS_OK;
    const int n1 = h->levelSize[2], begin1 = h->levelSize[3];
    const size_t bytes = coarse1_tags(h) * sizeof(Tag3);
    int rc;
    if ((rc = ensure(h, h->c1Tags, bytes)) ||
        (rc = hip_check(h, hipMemsetAsync(h->c1Tags.p, 0, bytes, s), "memset coarse1 tags")) ||
        (rc = ensure(h, h->l1info, (size_t)ceil32(n1) * 16)))
        return rc;
    k_l1info<<<cdiv(n1, 256), 256, 0, s>>>(n1, begin1, P<int>(h->goingNext), P<int2>(h->members),
                                          h->L >= 4 ? P<int>(h->deepPos) : nullptr, P<int4>(h->l1info));
    return hip_check(h, hipGetLastError(), "coarse1 tables");
}

bool coarse1_supported(const mas_context* h) { return h->L >= 3 && h->c1Tags.p != nullptr; }

void launch_coarse_one(mas_context* h, const float4* r, hipStream_t s) {
    if (++h->coarse1Epoch == 0) {  // wrap-around: no tag from 2^32 applies ago may match
        hipMemsetAsync(h->c1Tags.p, 0, coarse1_tags(h) * sizeof(Tag3), s);
        h->coarse1Epoch = 1;
    }
    Coarse1Args a{};
    a.inv = P<float4>(h->inv);
    a.r = r;
    a.l1src = P<int>(h->l1src);
    a.l1info = P<int4>(h->l1info);
    a.rc = P<float4>(h->Rc);
    a.zc = P<float4>(h->Zc);
    a.n1 = h->levelSize[2];
    a.begin1 = h->levelSize[3];
    a.L = h->L;
    a.n2 = h->levelSize[4];
    a.lv2Begin = h->levelSize[5];
    a.nb2 = ceil32(a.n2) / 32;
    a.nb1 = ceil32(a.n1) / 32;
    const bool deep = h->L >= 4;
    a.n3 = deep ? h->levelSize[6] : 0;
    a.lv3Begin = deep ? h->levelSize[7] : h->totalClusters;
    a.nb3 = ceil32(a.n3) / 32;
    a.stride = h->deepStride;
    a.deepOff = P<int>(h->deepOff);
    Tag3* t = P<Tag3>(h->c1Tags);
    const size_t nList = deep ? (size_t)deep_nodes(h) * h->deepStride : 0;
    a.tR1 = t;
    a.tR2 = t + nList;
    a.tR3 = a.tR2 + ceil32(a.n2);
    a.epoch = h->coarse1Epoch;
    a.pollDelay = h->c1PollDelay;
    a.chunk = h->c1Chunk;
    a.done = h->applyDone;
    a.pollLimit = h->c1PollLimit;
    a.members = h->groupedR3 && deep ? P<int2>(h->members) : nullptr;
    a.timeouts = P<int>(h->devStatus) + 2;
    a.giveupHost = h->c1Host;
    h->c1Launched = true;
    k_coarse1<<<a.nb1 + a.n3 + a.nb2 + a.nb3, 64, 0, s>>>(a);
    // (no event here: a marker between k_coarse1 and the fine kernel held the
    // fine kernel back ~5 us per apply -- the trace's coarse -> fine gap went
    // from ~0 to 6.7 us; mas_get_stats reads the counter on its own stream)
}


}  // namespace mas

#ifdef MAS_PROBE
extern "C" int mas_probe1_dump(unsigned long long* out, int n) {
    if (n > 3 * 8192 * 8) n = 3 * 8192 * 8;
    hipDeviceSynchronize();
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mas::g_probe1), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
extern "C" int mas_probe1_clear() {
    static unsigned long long zero[3 * 8192 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(mas::g_probe1), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
