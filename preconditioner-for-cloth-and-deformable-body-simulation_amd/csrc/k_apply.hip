// k_apply.hip -- Preconditioning (.cpp:100-110, 1548-1719): the hot path.
//
//   k_restrict_l0   R1 = level-1 sums of r gathered through the Morton map
//                   (BuildResidualHierarchy .cpp:1558-1574); sums run in lane
//                   order from +0, exactly as the reference's owner loop.
//   k_restrict_lx   R_{l+1} from R_l for l >= 1 (deterministic per-bank sums;
//                   .cpp:1577-1591 sums level-1 values straight into every
//                   ancestor -- same value up to fp association).
//   k_solve<COARSE> Z_b = Inv_b R_b for every coarse block (SchwarzLocalXSym
//                   .cpp:1600-1696).
//   k_solve<FINE>   the same for every level-0 block, fused with the gather
//                   r[s2o[v]] and the prolongation
//                   z[s2o[v]] = Z0 + Z1[a1] + Z2[a2] + Z3[a3] (CollectFinalZ
//                   .cpp:1698-1719, min(L,4)-1 coarse levels, B-6).
//
// Block solve mapping (layout.h): a wave64 solves two blocks, one per 32-lane
// half; lane n owns node n.  The 18 624-byte packed inverse is streamed by 36
// float4 loads + one 12-byte tail load per lane (2 x 512 contiguous bytes per
// wave-instruction) straight into registers; the symmetric mat-vec then needs
// only ds_bpermute rotations: for s = 1..15 lane n multiplies G(n, n+s) with
// r_{n+s} and sends G^T r_n to lane n+s.  No LDS, no atomics, no barriers.
// The kernel is bound by HBM bandwidth (~1 flop/byte).
#include "layout.h"
#include "mas_internal.h"

namespace mas {

constexpr int kApplyThreads = 256;  // 4 waves = 4 blocks per workgroup

__device__ __forceinline__ float rd_lane(float x, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

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

__device__ __forceinline__ void load_record(const float4* __restrict__ inv, int blk, int lane, float (&g)[kRecord],
                                            float (&tl)[3]) {
    const float4* b = inv + (size_t)blk * kBlockF4 + lane;
#pragma unroll
    for (int q = 0; q < kRecord / 4; ++q) {
        const float4 x = b[q * 64];
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

// Fine blocks: gather r through the Morton map, solve, prolongate, scatter z.
template <int NPROL>
__global__ __launch_bounds__(kApplyThreads) void k_solve_fine(const float4* __restrict__ inv, int nFineBlk, int nV,
                                                             const float4* __restrict__ r,
                                                             const int4* __restrict__ vmap,
                                                             const float4* __restrict__ zc, int begin1,
                                                             float4* __restrict__ z) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int blk = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    const bool bvalid = blk < nFineBlk;
    const int v = blk * 32 + n;
    const bool vvalid = bvalid && v < nV;
    const int4 m = vmap[vvalid ? v : 0];
    float g[kRecord], tl[3];
    load_record(inv, bvalid ? blk : 0, lane, g, tl);
    const float4 rv = r[m.x];
    const float3 rr = vvalid ? make_float3(rv.x, rv.y, rv.z) : make_float3(0.f, 0.f, 0.f);
    float3 out = block_solve(g, tl, rr, lane);
    if (!vvalid || lane >= 32) return;
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

// Coarse blocks [blk0, blk0 + nb): Zc = Inv Rc (node-indexed from begin1).
__global__ __launch_bounds__(kApplyThreads) void k_solve_coarse(const float4* __restrict__ inv, int blk0, int nb,
                                                               const float4* __restrict__ rc, int begin1,
                                                               float4* __restrict__ zc) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int rel = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    const bool valid = rel < nb;
    const int blk = blk0 + (valid ? rel : 0);
    const int node = blk * 32 + n - begin1;
    float g[kRecord], tl[3];
    load_record(inv, blk, lane, g, tl);
    const float4 rv = rc[node];
    const float3 out = block_solve(g, tl, make_float3(rv.x, rv.y, rv.z), lane);
    if (valid && lane < 32) zc[node] = make_float4(out.x, out.y, out.z, 0.f);
}

// Segmented sum of a 32-lane bank by parent id, in lane order from +0 (the
// reference's owner loop, .cpp:1560-1572): each bank stages (value, parent)
// in LDS, every lane walks the 32 entries with broadcast ds_read_b128 and adds
// the ones with its parent; the lowest lane of each parent stores the sum.
__device__ __forceinline__ void bank_sum_store(float3 val, int p, bool valid, float4* __restrict__ rc, int begin1) {
    __shared__ float4 buf[kApplyThreads];
    const int t = threadIdx.x, n = t & 31, base = t & ~31;
    buf[t] = make_float4(val.x, val.y, val.z, __int_as_float(p));
    __syncthreads();
    float ax = 0.f, ay = 0.f, az = 0.f;
    bool leader = true;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) {
        const float4 e = buf[base + j];
        if (__float_as_int(e.w) == p) {
            ax = __fadd_rn(ax, e.x);
            ay = __fadd_rn(ay, e.y);
            az = __fadd_rn(az, e.z);
            leader = leader && (j >= n);
        }
    }
    if (valid && leader) rc[p - begin1] = make_float4(ax, ay, az, 0.f);
}

__global__ __launch_bounds__(kApplyThreads) void k_restrict_l0(int nV, int nBanks, const float4* __restrict__ r,
                                                              const int4* __restrict__ vmap, float4* __restrict__ rc,
                                                              int begin1) {
    const int bank = blockIdx.x * (kApplyThreads / 32) + (threadIdx.x >> 5);
    const int v = bank * 32 + (threadIdx.x & 31);
    const bool valid = bank < nBanks && v < nV;
    const int4 m = vmap[valid ? v : 0];
    const float4 rv = r[m.x];
    const float3 val = valid ? make_float3(rv.x, rv.y, rv.z) : make_float3(0.f, 0.f, 0.f);
    bank_sum_store(val, valid ? m.y : -1, valid, rc, begin1);
}

__global__ __launch_bounds__(kApplyThreads) void k_restrict_lx(int begin, int count, const int* __restrict__ gn,
                                                              float4* __restrict__ rc, int begin1) {
    const int local = blockIdx.x * kApplyThreads + threadIdx.x;
    const bool valid = local < count;
    const int node = begin + (valid ? local : 0);
    const float4 rv = rc[node - begin1];
    const float3 val = valid ? make_float3(rv.x, rv.y, rv.z) : make_float3(0.f, 0.f, 0.f);
    bank_sum_store(val, valid ? gn[node] : -1, valid, rc, begin1);
}

static inline int grid_for_banks(int banks) { return cdiv(banks, kApplyThreads / 32); }
static inline int grid_for_blocks(int blocks) { return cdiv(blocks, kApplyThreads / 64); }

int run_apply(mas_context* h, float4* d_z, const float4* d_r, hipStream_t s) {
    const int L = h->L, nV = h->nV;
    const int begin1 = h->levelSize[3];
    const int4* vmap = P<int4>(h->vmap);
    const float4* inv = P<float4>(h->inv);
    float4* rc = P<float4>(h->Rc);
    float4* zc = P<float4>(h->Zc);
    hipEvent_t* ev = nullptr;
    if (h->profiling && h->profRecorded < kProfRing) ev = &h->prof[4 * h->profRecorded++];
    if (ev) hipEventRecord(ev[0], s);
    if (L > 1) {
        k_restrict_l0<<<grid_for_banks(h->nFineBlk), kApplyThreads, 0, s>>>(nV, h->nFineBlk, d_r, vmap, rc, begin1);
        for (int l = 1; l + 1 < L; ++l) {
            const int cnt = h->levelSize[2 * l], beg = h->levelSize[2 * l + 1];
            k_restrict_lx<<<cdiv(cnt, kApplyThreads), kApplyThreads, 0, s>>>(beg, cnt, P<int>(h->goingNext), rc,
                                                                                   begin1);
        }
    }
    if (ev) hipEventRecord(ev[1], s);
    if (L > 1) {
        const int nc = h->nBlk - h->nFineBlk;
        k_solve_coarse<<<grid_for_blocks(nc), kApplyThreads, 0, s>>>(inv, h->nFineBlk, nc, rc, begin1, zc);
    }
    if (ev) hipEventRecord(ev[2], s);
    const int g = grid_for_blocks(h->nFineBlk);
    switch (L < 4 ? L - 1 : 3) {
        case 0: k_solve_fine<0><<<g, kApplyThreads, 0, s>>>(inv, h->nFineBlk, nV, d_r, vmap, zc, begin1, d_z); break;
        case 1: k_solve_fine<1><<<g, kApplyThreads, 0, s>>>(inv, h->nFineBlk, nV, d_r, vmap, zc, begin1, d_z); break;
        case 2: k_solve_fine<2><<<g, kApplyThreads, 0, s>>>(inv, h->nFineBlk, nV, d_r, vmap, zc, begin1, d_z); break;
        default: k_solve_fine<3><<<g, kApplyThreads, 0, s>>>(inv, h->nFineBlk, nV, d_r, vmap, zc, begin1, d_z); break;
    }
    if (ev) hipEventRecord(ev[3], s);
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "apply kernels");
}

// ---------------------------------------------------------------------------
// Prepare orchestration: stencils -> levels -> assembly -> factor
// ---------------------------------------------------------------------------

int run_prepare(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, const void* ef,
                const void* ee, const void* vf, const unsigned* efC, const unsigned* eeC, const unsigned* vfC,
                hipStream_t s) {
    int rc;
    h->prepared = false;
    hipEventRecord(h->ev[2], s);
    // .cpp:74-75: fresh copies of the ELL neighbour table
    if ((rc = hip_check(h, hipMemcpyAsync(h->nbrRem.p, h->nbr.p, (size_t)h->maxNbr * h->nV * 4, hipMemcpyDeviceToDevice, s),
                        "copy nbr")) ||
        (rc = hip_check(h, hipMemcpyAsync(h->nbrNumRem.p, h->nbrNum.p, (size_t)h->nV * 4, hipMemcpyDeviceToDevice, s),
                        "copy nbrNum")))
        return rc;
    if ((rc = build_stencils(h, ef, ee, vf, efC, eeC, vfC, s))) return rc;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    if ((rc = run_levels(h, s))) return rc;
    hipEventRecord(e0, s);
    if ((rc = run_assemble(h, d_diag9, d_off9, d_ranges, s))) return rc;
    hipEventRecord(e1, s);
    if ((rc = run_factor(h, s))) return rc;
    const int nCoarseNodes = h->totalClusters - h->levelSize[3];
    if ((rc = ensure(h, h->Rc, (size_t)(nCoarseNodes > 0 ? nCoarseNodes : 1) * 16)) ||
        (rc = ensure(h, h->Zc, (size_t)(nCoarseNodes > 0 ? nCoarseNodes : 1) * 16)))
        return rc;
    if (nCoarseNodes > 0 && (rc = hip_check(h, hipMemsetAsync(h->Rc.p, 0, (size_t)nCoarseNodes * 16, s), "memset Rc")))
        return rc;
    hipEventRecord(h->ev[3], s);
    if ((rc = hip_check(h, hipStreamSynchronize(s), "prepare sync"))) return rc;
    float a = 0, b = 0, c = 0, t = 0;
    hipEventElapsedTime(&t, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&a, h->ev[2], e0);
    hipEventElapsedTime(&b, e0, e1);
    hipEventElapsedTime(&c, e1, h->ev[3]);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    h->stats.prepare_ms = t;
    h->stats.prepare_levels_ms = a;
    h->stats.prepare_assemble_ms = b;
    h->stats.prepare_factor_ms = c;
    h->prepared = true;
    return MAS_OK;
}

}  // namespace mas
