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

// workgroup g of G runs on XCD g % 8: the logical index that gives each XCD a
// contiguous range (as k_apply.hip xcd_chunked)
__device__ __forceinline__ int xcd_chunk_of(int g, int G) {
    const int full = G & ~7;
    return g < full ? (g & 7) * (full >> 3) + (g >> 3) : g;
}

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

int build_fused_tables(mas_context* h, hipStream_t s);

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
    if ((rc = hip_check(h, hipGetLastError(), "coarse1 tables"))) return rc;
    return build_fused_tables(h, s);
}

bool coarse1_supported(const mas_context* h) { return h->L >= 3 && h->c1Tags.p != nullptr; }

void launch_coarse_one(mas_context* h, const float4* r, hipStream_t s) {
    if (++h->coarse1Epoch == 0) {  // wrap-around: no tag from 2^32 applies ago may match
        hipMemsetAsync(h->c1Tags.p, 0, coarse1_tags(h) * sizeof(Tag3), s);
        if (h->tZ.p) hipMemsetAsync(h->tZ.p, 0, h->tZ.bytes, s);  // the fused form's tags share the epoch
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
    // mas_get_stats waits for this event (the latest one-launch apply, on
    // whatever stream it ran), not for the whole device; run_apply never
    // launches this form on a capturing stream
    hipEventRecord(h->evC1, s);
}


// ===========================================================================
// Fused apply (coarseMode 4): the coarse levels AND the level-0 blocks in ONE
// launch of two-wave workgroups, so no kernel boundary (and its drain and
// refill) sits between the coarse chain and the fine pass.
//
//   coarse waves (first in the grid, so dispatched first): the roles of
//       k_coarse1 (bank / grouped fold / level-2 / level-3 solve waves) without
//       LDS; every coarse Z is also published as a tagged word (tZ, as the R
//       hand-offs), and every Z-producing wave counts itself in `solved`
//       after its stores have drained.
//   hold workgroups (holdWG, the chip's resident slots by default): one wave
//       polls `solved` until this apply's coarse waves are all counted, then
//       the workgroup exits.  Workgroups are dispatched in grid order as slots
//       free up, so no fine workgroup after them starts while the chain runs:
//       under the full fine load every hop of the chain queues behind ~50 MB
//       of inverse loads (measured: the chain then outlasts the fine pass).
//   fine waves, one per level-0 block: gather r, solve, read the tagged
//       Z1..Z3 of the 32 vertices' ancestors (published by then; a wave that
//       started beside the chain -- earlyWG, an A/B knob, or a slot the holds
//       missed -- polls, bounded), add them in CollectFinalZ order
//       (.cpp:1706-1717) and store z: bitwise the unfused apply's z.
//
// (A first form let early fine waves store Z0 and defer the coarse terms to a
// list drained by later waves: every wave then paid same-address atomics on
// the list counters, ~17 ms per apply at 1M; measured and removed, DESIGN.md
// section 4 "Fused apply".)
// ===========================================================================
struct FusedArgs {
    Coarse1Args c;
    const int4* vmap;
    float4* z;
    Tag3* tZ;                      // coarse node (id - begin1) -> tagged Z
    int nV, nFineBlk, nprol;
    int bankWG;                    // workgroups of bank waves
    int coarseWG;                  // workgroups before the fine ones (a multiple of 8)
    int earlyWG;                   // fine workgroups right after the coarse ones (they may wait)
    int holdWG;                    // hold workgroups after them: wait for the coarse Z, then exit
    unsigned long long* solved;    // coarse Z-producing waves finished, since the tables were built
    unsigned long long target;     // *solved once this apply's coarse waves are all done
};

// a Z-producing coarse wave is done: its tagged stores drained, then counted
// (the hold workgroups wait for the count; the tags themselves stay the
// fine waves' test)
__device__ __forceinline__ void count_solved(const FusedArgs& f) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_fetch_add(f.solved, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// R1 / R2 / Z1 of level-1 bank B without LDS (bitwise the same sums as
// bank_wave): lane 32 h + j gathers children 16 h .. 16 h + 15 of node j, so
// lane j folds its own 16 in lane order from +0 and then lane j + 32's 16,
// one shuffle each.
__device__ __forceinline__ void bank_wave_fused(const FusedArgs& f, int B) {
    const Coarse1Args& a = f.c;
    const int lane = threadIdx.x & 63, j = lane & 31, hh = lane >> 5;
    const int c0 = B * 32;
    const int c = c0 + j;
    // l1src covers ceil32(n1) nodes (-1 padded)
    const int4* s4 = reinterpret_cast<const int4*>(a.l1src + (size_t)c * 32 + 16 * hh);
    int src[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int4 t = s4[q];
        src[4 * q + 0] = t.x;
        src[4 * q + 1] = t.y;
        src[4 * q + 2] = t.z;
        src[4 * q + 3] = t.w;
    }
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
    float ax = 0.f, ay = 0.f, az = 0.f;  // R1, lane order from +0 (non-children are +0.0)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        ax = __fadd_rn(ax, val[q].x);
        ay = __fadd_rn(ay, val[q].y);
        az = __fadd_rn(az, val[q].z);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        ax = __fadd_rn(ax, __shfl_xor(val[q].x, 32));
        ay = __fadd_rn(ay, __shfl_xor(val[q].y, 32));
        az = __fadd_rn(az, __shfl_xor(val[q].z, 32));
    }
    if (!own) ax = ay = az = 0.f;
    // R2 of the level-2 nodes whose children are this bank's components (their lowest lane)
    const unsigned pmsk = (unsigned)info.y;
    const bool lead = own && (unsigned)(__ffs(pmsk) - 1) == (unsigned)j;
    float bx = 0.f, by = 0.f, bz = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const float vx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ax), k));
        const float vy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ay), k));
        const float vz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(az), k));
        const bool in = (pmsk >> k) & 1u;
        bx = __fadd_rn(bx, in ? vx : 0.f);
        by = __fadd_rn(by, in ? vy : 0.f);
        bz = __fadd_rn(bz, in ? vz : 0.f);
    }
    if (lead) {
        st_tag(a.tR2 + info.x - (a.lv2Begin - a.begin1), bx, by, bz, a.epoch);
        a.rc[info.x] = make_float4(bx, by, bz, 0.f);
    }
    if (own) a.rc[c] = make_float4(ax, ay, az, 0.f);
    float g[kRecord], tl[3];
    load_record<true>(a.inv, a.begin1 / 32 + B, lane, g, tl);
    const float3 out = block_solve(g, tl, make_float3(__shfl(ax, j), __shfl(ay, j), __shfl(az, j)), lane);
    if (lane < 32) {
        a.zc[c] = make_float4(out.x, out.y, out.z, 0.f);
        st_tag(f.tZ + c, out.x, out.y, out.z, a.epoch);
    }
    count_solved(f);
}

// level-2 / level-3 block (solve_wave) that also publishes its Z tagged
__device__ __forceinline__ void solve_wave_fused(const FusedArgs& f, int blk, int lvBegin, int cnt, const Tag3* tR) {
    const Coarse1Args& a = f.c;
    const int lane = threadIdx.x & 63, n = lane & 31;
    float g[kRecord], tl[3];
    load_record<true>(a.inv, blk, lane, g, tl);
    const int loc = blk * 32 + n - lvBegin;
    const bool real = lane < 32 && loc < cnt;
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    bool ok = !real;
    for (int polls = 0; polls <= a.pollLimit; ++polls) {
        if (!ok) {
            ld_tag(tR + loc, v);
            ok = tag_ok(v, a.epoch);
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (!__all(ok) && lane == 0) gave_up(a);
    const float rx = __shfl(tag_val(v[0]), n), ry = __shfl(tag_val(v[1]), n), rz = __shfl(tag_val(v[2]), n);
    const float3 out = block_solve(g, tl, make_float3(rx, ry, rz), lane);
    if (lane < 32) {
        const int node = blk * 32 + n - a.begin1;
        a.zc[node] = make_float4(out.x, out.y, out.z, 0.f);
        st_tag(f.tZ + node, out.x, out.y, out.z, a.epoch);
    }
    count_solved(f);
}

// Z1..Z_nprol of vertex map m, tagged; true when all carry this epoch
__device__ __forceinline__ bool coarse_z(const FusedArgs& f, int4 m, unsigned long long (&t)[3][3]) {
    const int b1 = f.c.begin1;
    const int anc[3] = {m.y, m.z, m.w};
    bool ok = true;
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        if (l < f.nprol) {
            ld_tag(f.tZ + anc[l] - b1, t[l]);
            ok = ok && tag_ok(t[l], f.c.epoch);
        }
    }
    return ok;
}

__device__ __forceinline__ float3 add_coarse(const FusedArgs& f, float3 o, const unsigned long long (&t)[3][3]) {
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        if (l < f.nprol) {
            o.x = __fadd_rn(o.x, tag_val(t[l][0]));
            o.y = __fadd_rn(o.y, tag_val(t[l][1]));
            o.z = __fadd_rn(o.z, tag_val(t[l][2]));
        }
    }
    return o;
}

__device__ __forceinline__ void fine_wave_fused(const FusedArgs& f, int blk) {
    const Coarse1Args& a = f.c;
    const int lane = threadIdx.x & 63, n = lane & 31;
    const bool bvalid = blk < f.nFineBlk;
    const int v = blk * 32 + n;
    const bool vvalid = bvalid && v < f.nV;
    const int4 m = f.vmap[vvalid ? v : 0];
    float g[kRecord], tl[3];
    load_record<true>(a.inv, bvalid ? blk : 0, lane, g, tl);
    const float4 rv = a.r[m.x];
    const float3 rr = vvalid ? make_float3(rv.x, rv.y, rv.z) : make_float3(0.f, 0.f, 0.f);
    const float3 z0 = block_solve(g, tl, rr, lane);
    const bool writer = vvalid && lane < 32;
    // the coarse Z of this block's vertices: published already unless this
    // wave started beside the coarse chain (an early workgroup, or a slot the
    // hold workgroups did not cover); then it waits, bounded
    unsigned long long t[3][3] = {};
    bool ok = !writer || coarse_z(f, m, t);
    for (int polls = 0; polls <= a.pollLimit; ++polls) {
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(2);
        if (!ok) ok = coarse_z(f, m, t);
    }
    if (!__all(ok) && lane == 0) gave_up(a);
    if (writer) {
        const float3 o = add_coarse(f, z0, t);
        f.z[m.x] = make_float4(o.x, o.y, o.z, 0.f);
    }
}

// grid of two-wave workgroups: [0, bankWG) bank waves (XCD-chunked), then
// the fold / level-2 / level-3 solve waves, idle waves up to coarseWG (a
// multiple of 8, so the fine workgroups keep the XCD chunking); then earlyWG
// fine workgroups (they run beside the coarse chain and may defer), holdWG
// hold workgroups, and the remaining fine workgroups (XCD-chunked like
// k_solve_fine over the early + remaining ones).  Workgroups are dispatched in
// grid order as slots free up, so while the hold workgroups wait for the
// coarse chain no later fine workgroup takes a slot: the chain runs under the
// early fine waves' load only (under the full fine load every hop queues
// behind ~50 MB of inverse loads and the chain outlasts the fine pass).
__global__ __launch_bounds__(128) void k_apply_fused(FusedArgs f) {
    const Coarse1Args& a = f.c;
    if (a.done && *a.done) return;
    const int h = threadIdx.x >> 6;
    const int g = blockIdx.x;
    if (g < f.bankWG) {
        const int B = 2 * (a.chunk ? xcd_chunk_of(g, f.bankWG) : g) + h;
        if (B < a.nb1) bank_wave_fused(f, B);
        return;
    }
    if (g < f.coarseWG) {
        int w = 2 * (g - f.bankWG) + h;
        if (w < a.n3) return fold_wave_grouped(a, w);
        w -= a.n3;
        if (w < a.nb2) return solve_wave_fused(f, a.lv2Begin / 32 + w, a.lv2Begin, a.n2, a.tR2);
        w -= a.nb2;
        if (w < a.nb3) solve_wave_fused(f, a.lv3Begin / 32 + w, a.lv3Begin, a.n3, a.tR3);
        return;
    }
    int fg = g - f.coarseWG;
    if (fg >= f.earlyWG) {
        if (fg < f.earlyWG + f.holdWG) {  // hold: one wave polls, then the workgroup exits
            if (h == 0) {
                bool ok = false;
                for (int polls = 0; polls <= a.pollLimit && !ok; ++polls) {
                    ok = __hip_atomic_load(f.solved, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= f.target;
                    if (!ok) __builtin_amdgcn_s_sleep(32);  // ~1 us: a thousand pollers of one word
                }
                if (!ok && (threadIdx.x & 63) == 0) gave_up(a);
            }
            return;
        }
        fg -= f.holdWG;
    }
    const int G = gridDim.x - f.coarseWG - f.holdWG;
    fine_wave_fused(f, 2 * xcd_chunk_of(fg, G) + h);
}

bool fused_supported(const mas_context* h) {
    return coarse1_supported(h) && (h->L == 3 || h->groupedR3) && h->tZ.p != nullptr;
}

void launch_apply_fused(mas_context* h, const float4* r, float4* z, hipStream_t s) {
    if (++h->coarse1Epoch == 0) {
        hipMemsetAsync(h->c1Tags.p, 0, coarse1_tags(h) * sizeof(Tag3), s);
        hipMemsetAsync(h->tZ.p, 0, h->tZ.bytes, s);
        hipMemsetAsync(h->fuseDef.p, 0, h->fuseDef.bytes, s);
        h->coarse1Epoch = 1;
        h->fuseApplies = 0;
    }
    FusedArgs f{};
    Coarse1Args& a = f.c;
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
    a.chunk = h->c1Chunk;
    a.done = h->applyDone;
    a.pollLimit = h->c1PollLimit;
    a.members = deep ? P<int2>(h->members) : nullptr;
    a.timeouts = P<int>(h->devStatus) + 2;
    a.giveupHost = h->c1Host;
    f.vmap = P<int4>(h->vmap);
    f.z = z;
    f.tZ = P<Tag3>(h->tZ);
    f.nV = h->nV;
    f.nFineBlk = h->nFineBlk;
    f.nprol = h->L < 4 ? h->L - 1 : 3;
    f.bankWG = cdiv(a.nb1, 2);
    const int other = a.n3 + a.nb2 + a.nb3;
    f.coarseWG = (f.bankWG + cdiv(other, 2) + 7) & ~7;
    const int fineWG = cdiv(h->nFineBlk, 2);
    // early fine workgroups and hold workgroups, multiples of 8 (XCD chunking)
    f.earlyWG = std::min(fineWG, h->fuseEarly >= 0 ? h->fuseEarly : 0) & ~7;
    f.holdWG = h->fuseHold >= 0 ? h->fuseHold : h->fuseSlots;
    f.holdWG = (f.holdWG + 7) & ~7;
    f.solved = P<unsigned long long>(h->fuseDef);
    f.target = (unsigned long long)(++h->fuseApplies) * (unsigned long long)(a.nb1 + a.nb2 + a.nb3);
    h->c1Launched = true;
    k_apply_fused<<<f.coarseWG + f.holdWG + fineWG, 128, 0, s>>>(f);
    hipEventRecord(h->evC1, s);
}

// tagged coarse Z (one Tag3 per coarse node) and the 64-bit count of
// Z-producing coarse waves done (reset with the epoch)
int build_fused_tables(mas_context* h, hipStream_t s) {
    if (h->L < 3) return MAS_OK;
    const size_t nCoarse = (size_t)(h->totalClusters - h->levelSize[3]);
    const size_t zb = (nCoarse > 0 ? nCoarse : 1) * sizeof(Tag3);
    const size_t db = 64;
    h->fuseApplies = 0;
    if (h->fuseSlots == 0) {  // resident workgroups of k_apply_fused on the whole chip
        int perCU = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, k_apply_fused, 128, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess)
            return fail(h, MAS_ERR_HIP, "k_apply_fused occupancy");
        h->fuseSlots = perCU * cus;
    }
    int rc;
    if ((rc = ensure(h, h->tZ, zb)) || (rc = ensure(h, h->fuseDef, db)) ||
        (rc = hip_check(h, hipMemsetAsync(h->tZ.p, 0, h->tZ.bytes, s), "memset tZ")) ||
        (rc = hip_check(h, hipMemsetAsync(h->fuseDef.p, 0, h->fuseDef.bytes, s), "memset solved count")))
        return rc;
    return MAS_OK;
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
