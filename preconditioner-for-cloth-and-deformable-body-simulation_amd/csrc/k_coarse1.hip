// k_coarse1.hip -- every coarse level of one Preconditioning in ONE launch
// (BuildResidualHierarchy .cpp:1548-1598, SchwarzLocalXSym .cpp:1600-1696
// for levels 1..min(L-1, 3)); coarseMode 3.
//
// The two-launch form (k_coarse.hip) starts the level-3 fold only after the
// whole level-1 restriction, a kernel boundary and the workgroup dispatch of
// the second launch.  Here one launch holds
//
//   bank waves (first in the grid), one per level-1 bank (= level-1 block):
//       R1 of its 32 nodes from r (lane order from +0), R2 of the level-2
//       nodes whose children are its components (level-1 id order from +0) --
//       the two-launch form's sums, bit for bit; R1 is also published at its
//       place in its level-3 ancestor's descendant list and R2 at its node,
//       write-through, then the bank's completion flag (= this apply's epoch);
//       one arrival per level-2 block it contributed to (expected counts from
//       Prepare, k_l2_expect); the level-2 block's last contributor solves it;
//       then the bank's own level-1 block (its inverse is loaded only after
//       the publication, off the chain's path).
//   fold waves (L >= 4, last in the grid), one per level-3 node T: they poll
//       the completion flags of T's banks in order and fold every R1 whose
//       bank is done, left from +0 in level-1 id order (the reference's R3,
//       .cpp:1577-1590), while later banks are still restricting; the next
//       poll is in flight during each fold step.  R3 is published and the
//       block's last arriving node solves the level-3 block.
//
// Hand-offs (flags, R1, R2, R3): write-through (sc1) stores, drained, then the
// flag / a relaxed agent-scope arrival count; the consumer reads with sc1
// loads (deep_fold.h header).  The epoch lives in device memory (the last
// fold wave advances it), so a captured graph of this launch replays
// correctly.  Bank waves never wait; fold waves wait only for bank waves,
// which precede them in the grid; every poll loop is bounded.
//
// Every R and Z is the two-launch form's value bit for bit;
// tests/test_gpu_chain.py compares the forms over many back-to-back applies.
#include "block_solve.h"
#include "deep_fold.h"

namespace mas {

// Diagnostic stamps (probe build only): lane 0 of a wave writes the 100 MHz
// wall clock into g_probe1[kind][slot][k] (kind 0: level-3 fold waves by node,
// kind 1: bank waves by bank); mas_probe1_dump reads them back.
#ifdef MAS_PROBE
__device__ unsigned long long g_probe1[2 * 8192 * 8];
#define C1_STAMP(kind, slot, k)                                                                          \
    do {                                                                                                 \
        unsigned long long t_;                                                                           \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        if ((threadIdx.x & 63) == 0 && (slot) < 8192) g_probe1[((kind) * 8192 + (slot)) * 8 + (k)] = t_; \
    } while (0)
#define C1_DBG(kind, slot, k, val) \
    do { if ((threadIdx.x & 63) == 0 && (slot) < 8192) g_probe1[((kind) * 8192 + (slot)) * 8 + (k)] = (unsigned long long)(val); } while (0)
#else
#define C1_DBG(kind, slot, k, val) \
    do {                           \
    } while (0)
#define C1_STAMP(kind, slot, k) \
    do {                        \
    } while (0)
#endif

constexpr int kFoldIds = 2048;   // list entries a fold wave stages (longer lists: MAS_ERR_CAPACITY at Prepare)
constexpr int kFoldStep = 512;   // entries loaded per fold step (8 per lane)
constexpr int kCntStride = 32;   // arrival counters 128 B apart (one cache line each)
constexpr int kPollLimit = 1 << 22;  // bounded waits (a few ms): never hang the device

struct Coarse1Args {
    const float4* inv;
    const float4* r;
    const int* l1src;     // 32 original vertex ids (or -1) per level-1 node
    const int4* l1info;   // per level-1 node: (parent - begin1, the parent's child mask, list slot, 0)
    float4* rc;           // R per coarse node (index: node id - begin1)
    float4* zc;           // Z per coarse node
    int n1, begin1, L;
    int n2, lv2Begin;     // level 2
    int* cnt2;            // per level-2 block (kCntStride apart): arrivals of contributing level-1 banks
    const int* exp2;      // per level-2 block: the number of contributing banks
    // level 3 (L >= 4)
    int nDeep, lv3Begin, stride;
    const int* deepOff;   // list start per level-3 node (sorted level-1 ids), + 1
    const int* deepIdx;   // list slot T * stride + i -> level-1 id
    float4* deepR1;       // list slot -> R1 (published by the banks)
    int* bankFlag;        // per level-1 bank: the epoch of its last publication
    int* epoch;           // [0] = the epoch of the previous apply, [kCntStride] = fold waves done
    int* cnt3;            // per level-3 block: node arrivals
    const int* done;      // PCG: exit at once when set
};

__device__ __forceinline__ void st_wt_int(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_wt_int(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int WAVES>
union C1Shared {
    struct {
        float svs[WAVES][3][32][33];  // [wave][component][node][child]
        float4 red[WAVES][32];
    } bank;
    struct {
        int ids[WAVES][kFoldIds];                          // the node's level-1 descendants, ascending
        __attribute__((aligned(16))) float stg[WAVES][3][kFoldStep];  // R1 of one step, component-major
    } fold;
};

// ---------------------------------------------------------------------------
// level-1 bank: R1, R2 and the publications; L2 / L1 solves
// ---------------------------------------------------------------------------
template <int WAVES>
__device__ __forceinline__ void bank_wave(const Coarse1Args& a, int B, C1Shared<WAVES>& sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane & 31;
    const int c0 = B * 32;
    if (c0 >= a.n1) return;  // wave-uniform; no workgroup barriers in this role
    C1_STAMP(1, B, 0);
    const int* s = a.l1src + (size_t)c0 * 32;
    int src[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) src[q] = s[64 * q + lane];
    const int c = c0 + j;
    const bool own = lane < 32 && c < a.n1;
    const bool hasL2 = a.L >= 3, hasL3 = a.L >= 4;
    const int4 info = own && hasL2 ? a.l1info[c] : make_int4(0, 0, -1, 0);
    float g[kRecord], tl[3];
    const int parent = info.x;
    const unsigned pmsk = (unsigned)info.y;
    const int E1 = hasL3 ? a.epoch[0] + 1 : 0;  // this apply's epoch
    // the level-2 blocks this bank contributes to: its parents are consecutive
    // ids, the smallest at lane 0 (always a component's lowest lane); their
    // expected arrival counts are loaded with the gathers
    int b2lo = 0, b2hi = 0, expc = 0;
    if (hasL2) {
        int pmax = own ? parent : -1;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) pmax = max(pmax, __shfl_xor(pmax, o));
        b2lo = (__shfl(parent, 0) + a.begin1) >> 5;
        b2hi = (__shfl(pmax, 0) + a.begin1) >> 5;
        if (lane < 2 && b2lo + lane <= b2hi) expc = a.exp2[b2lo + lane - a.lv2Begin / 32];
    }
    float4 val[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) val[q] = src[q] >= 0 ? a.r[src[q]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        sh.bank.svs[w][0][2 * q + (lane >> 5)][j] = val[q].x;
        sh.bank.svs[w][1][2 * q + (lane >> 5)][j] = val[q].y;
        sh.bank.svs[w][2][2 * q + (lane >> 5)][j] = val[q].z;
    }
    __builtin_amdgcn_wave_barrier();
    C1_STAMP(1, B, 1);
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (own) {
#pragma unroll
        for (int k0 = 0; k0 < 32; k0 += 8) {
            float vx[8], vy[8], vz[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                vx[k] = sh.bank.svs[w][0][j][k0 + k];
                vy[k] = sh.bank.svs[w][1][j][k0 + k];
                vz[k] = sh.bank.svs[w][2][j][k0 + k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                ax = __fadd_rn(ax, vx[k]);
                ay = __fadd_rn(ay, vy[k]);
                az = __fadd_rn(az, vz[k]);
            }
        }
    }
    const float4 R1 = make_float4(ax, ay, az, 0.f);
    if (hasL3 && own && info.z >= 0) st_wt(a.deepR1 + info.z, R1);  // its place in its level-3 ancestor's list
    if (lane < 32) sh.bank.red[w][j] = R1;
    __builtin_amdgcn_wave_barrier();
    // R2 of the level-2 nodes whose children are this bank's components (lowest lane writes)
    const bool r2w = own && hasL2 && (unsigned)(__ffs(pmsk) - 1) == (unsigned)j;
    if (r2w) {
        float bx = 0.f, by = 0.f, bz = 0.f;
#pragma unroll
        for (int k0 = 0; k0 < 32; k0 += 8) {
            float4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = sh.bank.red[w][k0 + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool in = (pmsk >> (k0 + k)) & 1u;
                bx = __fadd_rn(bx, in ? v[k].x : 0.f);
                by = __fadd_rn(by, in ? v[k].y : 0.f);
                bz = __fadd_rn(bz, in ? v[k].z : 0.f);
            }
        }
        st_wt(a.rc + parent, make_float4(bx, by, bz, 0.f));
    }
    if (own) a.rc[c] = R1;  // R1 itself (read after the launch only)
    int arrivedLast = 0;  // bit 0: first level-2 block, bit 1: second
    if (hasL2) {
        C1_STAMP(1, B, 2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the R1 / R2 publications have landed
        C1_STAMP(1, B, 3);
        if (hasL3 && lane == 0) st_wt_int(a.bankFlag + B, E1);
        int flag = 0;
        if (lane < 2 && b2lo + lane <= b2hi) {
            const int old = __hip_atomic_fetch_add(a.cnt2 + (b2lo + lane - a.lv2Begin / 32) * kCntStride, 1,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag = (old + 1 == expc) ? (1 << lane) : 0;
        }
        arrivedLast = __shfl(flag, 0) | __shfl(flag, 1);
        C1_STAMP(1, B, 4);
    }
    float g2[kRecord], tl2[3];
    // level-2 blocks completed by this bank first (they are on the longest
    // path at L = 3): R2 from the published values
    for (int e = 0; e < 2; ++e) {
        if (!((arrivedLast >> e) & 1)) continue;
        const int b2 = b2lo + e;
        if (lane == 0) a.cnt2[(b2 - a.lv2Begin / 32) * kCntStride] = 0;  // for the next apply
        load_record<true>(a.inv, b2, lane, g2, tl2);
        const int nd = b2 * 32 + j;
        float4 R = make_float4(0.f, 0.f, 0.f, 0.f);
        if (nd - a.lv2Begin < a.n2) R = ld_wt(a.rc + nd - a.begin1);
        const float3 out = block_solve(g2, tl2, make_float3(R.x, R.y, R.z), lane);
        if (lane < 32) a.zc[nd - a.begin1] = make_float4(out.x, out.y, out.z, 0.f);
        C1_STAMP(1, B, 6);
    }
    // Z1 of this bank's block; its inverse is loaded only now, so the
    // restriction's gathers (the chain) do not queue behind 18.6 KB per wave
    load_record<true>(a.inv, a.begin1 / 32 + B, lane, g, tl);
    {
        const float rx = __shfl(ax, j), ry = __shfl(ay, j), rz = __shfl(az, j);
        const float3 out = block_solve(g, tl, make_float3(rx, ry, rz), lane);
        if (lane < 32) a.zc[c] = make_float4(out.x, out.y, out.z, 0.f);
    }
    C1_STAMP(1, B, 5);
}

// ---------------------------------------------------------------------------
// level-3 node T: fold R1 in level-1 id order as its banks complete
// ---------------------------------------------------------------------------
template <int WAVES>
__device__ __forceinline__ void fold_wave(const Coarse1Args& a, int T, C1Shared<WAVES>& sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (T >= a.nDeep) return;  // wave-uniform
    const int node = a.lv3Begin + T, blk = node >> 5;
    C1_STAMP(0, T, 0);
    const int E1 = a.epoch[0] + 1;
    const int beg = a.deepOff[T];
    const int len = a.deepOff[T + 1] - beg;  // 0 for a padding node (<= kFoldIds: checked at Prepare)
    const size_t base = (size_t)T * a.stride;
    int* ids = sh.fold.ids[w];
    for (int i = lane; i < len; i += 64) ids[i] = a.deepIdx[base + i];
    // the level-3 block's inverse, in flight during the fold (needed if this node arrives last)
    float g[kRecord], tl[3];
    load_record<true>(a.inv, blk, lane, g, tl);
    __builtin_amdgcn_wave_barrier();
    float acc = 0.f;
    if (len > 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int B0 = ids[0] >> 5, nb = (ids[len - 1] >> 5) - B0 + 1;
        int ready = 0;  // banks B0 .. B0 + ready - 1 have published
        int e = 0;      // list entries folded
        int polls = 0;
        while (e < len) {
            // poll the pending banks (64 per load round while whole rounds are
            // ready), extend the ready prefix
            if (ready < nb) {
                int grow = 0;
                for (int w0 = ready; w0 < nb && grow == w0 - ready; w0 += 64) {
                    const int bk = w0 + lane;
                    const bool ok = bk >= nb || ld_wt_int(a.bankFlag + B0 + bk) == E1;
                    const unsigned long long nr = ~__ballot(ok);
                    grow += nr ? (int)__builtin_ctzll(nr) : 64;
                }
                ready += min(grow, nb - ready);
            }
            // entries whose bank is done: a prefix of the ascending list
            int E = e;
            const int lim = ready >= nb ? 0x7fffffff : (B0 + ready) << 5;  // first level-1 id not yet published
            while (E < len && E - e < kFoldStep) {
                const int i = E + lane;
                const bool in = i < len && ids[i] < lim;
                const unsigned long long m = __ballot(in);
                const int cnt = (int)__popcll(m);
                E += cnt;
                if (cnt < 64) break;
            }
            E = min(E, e + kFoldStep);
            if (E == e) {  // nothing new yet
                if (++polls > kPollLimit) break;  // never hang: leave the fold incomplete
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            // load them (sc1), stage component-major, fold lanes 0..2 in list order
            float4 v[kFoldStep / 64];
#pragma unroll
            for (int q = 0; q < kFoldStep / 64; ++q) {
                const int i = e + 64 * q + lane;
                v[q] = i < E ? ld_wt(a.deepR1 + base + i) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int q = 0; q < kFoldStep / 64; ++q) {
                sh.fold.stg[w][0][64 * q + lane] = v[q].x;
                sh.fold.stg[w][1][64 * q + lane] = v[q].y;
                sh.fold.stg[w][2][64 * q + lane] = v[q].z;
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane < 3) {
                // whole 32-entry batches (the staged tail past E is +0: exact),
                // the next batch's reads in flight behind the current batch's adds
                const float4* row = reinterpret_cast<const float4*>(sh.fold.stg[w][lane]);
                const int n4 = ((E - e + 31) & ~31) / 4;
                float4 cur[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) cur[q] = row[q];
                for (int k0 = 0; k0 < n4; k0 += 8) {
                    const int kn = k0 + 8 < n4 ? k0 + 8 : k0;
                    float4 nxt[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) nxt[q] = row[kn + q];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        acc = __fadd_rn(acc, cur[q].x);
                        acc = __fadd_rn(acc, cur[q].y);
                        acc = __fadd_rn(acc, cur[q].z);
                        acc = __fadd_rn(acc, cur[q].w);
                    }
#pragma unroll
                    for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
                }
            }
            __builtin_amdgcn_wave_barrier();
            e = E;
        }
        C1_DBG(0, T, 5, len);
        C1_DBG(0, T, 6, nb | (ready << 16));
        C1_DBG(0, T, 7, e | ((unsigned long long)polls << 20) | ((unsigned long long)E1 << 40));
    }
    C1_STAMP(0, T, 2);
    const float ax = __shfl(acc, 0), ay = __shfl(acc, 1), az = __shfl(acc, 2);
    int last = 0, lastFold = 0;
    if (lane == 0) {
        st_wt(a.rc + node - a.begin1, make_float4(ax, ay, az, 0.f));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(a.cnt3 + (blk - a.lv3Begin / 32), 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        last = old == 31;
        // the last fold wave of the launch advances the epoch for the next apply
        const int f = __hip_atomic_fetch_add(a.epoch + kCntStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lastFold = f == a.nDeep - 1;
        if (lastFold) {
            a.epoch[kCntStride] = 0;
            a.epoch[0] = E1;
        }
    }
    last = __shfl(last, 0);
    C1_STAMP(0, T, 3);
    if (!last) return;
    if (lane == 0) a.cnt3[blk - a.lv3Begin / 32] = 0;  // for the next apply (visible after this kernel)
    const int n = lane & 31;
    const float4 R = ld_wt(a.rc + blk * 32 + n - a.begin1);
    const float3 out = block_solve(g, tl, make_float3(R.x, R.y, R.z), lane);
    if (lane < 32) a.zc[blk * 32 + n - a.begin1] = make_float4(out.x, out.y, out.z, 0.f);
    C1_STAMP(0, T, 4);
}

// grid: [0, nBankWG) bank workgroups, then the fold workgroups (WAVES level-3 nodes each)
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_coarse1(Coarse1Args a, int nBankWG) {
    if (a.done && *a.done) return;
    __shared__ C1Shared<WAVES> sh;
    if ((int)blockIdx.x < nBankWG)  // workgroup-uniform
        bank_wave<WAVES>(a, blockIdx.x * WAVES + (threadIdx.x >> 6), sh);
    else
        fold_wave<WAVES>(a, (blockIdx.x - nBankWG) * WAVES + (threadIdx.x >> 6), sh);
}

// ---- Prepare: per level-2 block, the number of level-1 banks contributing R2 ----
__global__ __launch_bounds__(256) void k_l2_expect(int n1, int begin1, int lv2Begin, const int* __restrict__ gn,
                                                   int* __restrict__ exp2) {
    const int B = blockIdx.x * 256 + threadIdx.x;
    const int c0 = B * 32;
    if (c0 >= n1) return;
    int pmin = 1 << 30, pmax = -1;
    for (int k = 0; k < 32 && c0 + k < n1; ++k) {
        const int p = gn[begin1 + c0 + k];
        pmin = min(pmin, p);
        pmax = max(pmax, p);
    }
    atomicAdd(exp2 + (pmin >> 5) - lv2Begin / 32, 1);
    if ((pmax >> 5) != (pmin >> 5)) atomicAdd(exp2 + (pmax >> 5) - lv2Begin / 32, 1);
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

int build_coarse1_tables(mas_context* h, hipStream_t s) {
    if (h->L < 3) return MAS_OK;
    const int n1 = h->levelSize[2], begin1 = h->levelSize[3], n2 = h->levelSize[4], lv2Begin = h->levelSize[5];
    const int nb2 = ceil32(n2) / 32, nb1 = ceil32(n1) / 32;
    const size_t words = (size_t)nb2 * (kCntStride + 1) + 2 * kCntStride + nb1;
    int rc;
    if ((rc = ensure(h, h->l2Cnt, words * 4)) ||
        (rc = hip_check(h, hipMemsetAsync(h->l2Cnt.p, 0, words * 4, s), "memset coarse1 counters")) ||
        (rc = ensure(h, h->l1info, (size_t)ceil32(n1) * 16)))
        return rc;
    k_l2_expect<<<cdiv(nb1, 256), 256, 0, s>>>(n1, begin1, lv2Begin, P<int>(h->goingNext),
                                               P<int>(h->l2Cnt) + (size_t)nb2 * kCntStride);
    k_l1info<<<cdiv(n1, 256), 256, 0, s>>>(n1, begin1, P<int>(h->goingNext), P<int2>(h->members),
                                          h->L >= 4 ? P<int>(h->deepPos) : nullptr, P<int4>(h->l1info));
    return hip_check(h, hipGetLastError(), "coarse1 tables");
}

// the one-launch form needs every level-3 list to fit a fold wave's LDS
bool coarse1_supported(const mas_context* h) { return h->L == 3 || (h->L >= 4 && h->deepStride <= kFoldIds); }

void launch_coarse_one(mas_context* h, const float4* r, hipStream_t s) {
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
    const int nb2 = ceil32(a.n2) / 32, nb1 = ceil32(a.n1) / 32;
    int* words = P<int>(h->l2Cnt);
    a.cnt2 = words;
    a.exp2 = words + (size_t)nb2 * kCntStride;
    a.epoch = words + (size_t)nb2 * (kCntStride + 1);
    a.bankFlag = a.epoch + 2 * kCntStride;
    a.nDeep = deep_nodes(h);
    a.lv3Begin = h->L >= 4 ? h->levelSize[7] : h->totalClusters;
    a.stride = h->deepStride;
    a.deepOff = P<int>(h->deepOff);
    a.deepIdx = P<int>(h->deepIdx);
    a.deepR1 = P<float4>(h->deepR1);
    a.cnt3 = P<int>(h->deepCnt);
    a.done = h->applyDone;
    if (a.nDeep == 0) {  // L = 3: single-wave workgroups spread the bank waves over every CU
        k_coarse1<1><<<nb1, 64, 0, s>>>(a, nb1);
    } else {
        const int nBankWG = cdiv(nb1, 4);
        k_coarse1<4><<<nBankWG + cdiv(a.nDeep, 4), 256, 0, s>>>(a, nBankWG);
    }
}

}  // namespace mas

#ifdef MAS_PROBE
extern "C" int mas_probe1_dump(unsigned long long* out, int n) {
    if (n > 2 * 8192 * 8) n = 2 * 8192 * 8;
    hipDeviceSynchronize();
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mas::g_probe1), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
extern "C" int mas_probe1_clear() {
    static unsigned long long zero[2 * 8192 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(mas::g_probe1), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
