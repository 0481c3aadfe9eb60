// k_allocate.hip -- AllocatePrecoditioner on the GPU (.cpp:38-65, 193-285).
//
//   k_aabb_partial / k_aabb_final  ComputeTotalAABB  (.cpp:193-211; SeAabbSimd.h:76-79)
//   k_morton                       FillSortingData   (.cpp:219-235; SeMorton.h:75-101)
//   onesweep radix sort (stable)   DoingSort         (.cpp:238-243; ties by index, B-9)
//   k_inverse_map                  ComputeInverseMapper (.cpp:245-255)
//   k_ell_map                      MapHessianTable   (.cpp:258-285)
//
// All of it is integer/byte work or exact min/max: bit-exact with the reference.
// The Morton normalisation keeps the reference's IEEE division and its
// ternary Clamp (NaN -> 2^21-1 on a degenerate axis, B-8); the build uses no
// fast-math so the compiler may not turn the selects into v_max/v_min.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "mas_internal.h"
#include "radix.h"

namespace mas {

constexpr int kAabbBlock = 256;
constexpr int kAabbGrid = 1024;

__device__ __forceinline__ float sel_min(float a, float b) { return a < b ? a : b; }  // _mm_min_ps
__device__ __forceinline__ float sel_max(float a, float b) { return a > b ? a : b; }  // _mm_max_ps

__global__ __launch_bounds__(kAabbBlock) void k_aabb_partial(const float4* __restrict__ pos, int n,
                                                             float4* __restrict__ part) {
    __shared__ float sm[6][kAabbBlock];
    float lo0 = FLT_MAX, lo1 = FLT_MAX, lo2 = FLT_MAX, hi0 = -FLT_MAX, hi1 = -FLT_MAX, hi2 = -FLT_MAX;
    for (int i = blockIdx.x * kAabbBlock + threadIdx.x; i < n; i += gridDim.x * kAabbBlock) {
        float4 p = pos[i];
        lo0 = sel_min(lo0, p.x); lo1 = sel_min(lo1, p.y); lo2 = sel_min(lo2, p.z);
        hi0 = sel_max(hi0, p.x); hi1 = sel_max(hi1, p.y); hi2 = sel_max(hi2, p.z);
    }
    int t = threadIdx.x;
    sm[0][t] = lo0; sm[1][t] = lo1; sm[2][t] = lo2; sm[3][t] = hi0; sm[4][t] = hi1; sm[5][t] = hi2;
    __syncthreads();
    for (int s = kAabbBlock / 2; s > 0; s >>= 1) {
        if (t < s) {
            for (int c = 0; c < 3; ++c) sm[c][t] = sel_min(sm[c][t], sm[c][t + s]);
            for (int c = 3; c < 6; ++c) sm[c][t] = sel_max(sm[c][t], sm[c][t + s]);
        }
        __syncthreads();
    }
    if (t == 0) {
        part[2 * blockIdx.x] = make_float4(sm[0][0], sm[1][0], sm[2][0], 0.f);
        part[2 * blockIdx.x + 1] = make_float4(sm[3][0], sm[4][0], sm[5][0], 0.f);
    }
}

__global__ __launch_bounds__(kAabbBlock) void k_aabb_final(float4* __restrict__ part, int nPart) {
    __shared__ float sm[6][kAabbBlock];
    float lo0 = FLT_MAX, lo1 = FLT_MAX, lo2 = FLT_MAX, hi0 = -FLT_MAX, hi1 = -FLT_MAX, hi2 = -FLT_MAX;
    for (int i = threadIdx.x; i < nPart; i += kAabbBlock) {
        float4 a = part[2 * i], b = part[2 * i + 1];
        lo0 = sel_min(lo0, a.x); lo1 = sel_min(lo1, a.y); lo2 = sel_min(lo2, a.z);
        hi0 = sel_max(hi0, b.x); hi1 = sel_max(hi1, b.y); hi2 = sel_max(hi2, b.z);
    }
    int t = threadIdx.x;
    sm[0][t] = lo0; sm[1][t] = lo1; sm[2][t] = lo2; sm[3][t] = hi0; sm[4][t] = hi1; sm[5][t] = hi2;
    __syncthreads();
    for (int s = kAabbBlock / 2; s > 0; s >>= 1) {
        if (t < s) {
            for (int c = 0; c < 3; ++c) sm[c][t] = sel_min(sm[c][t], sm[c][t + s]);
            for (int c = 3; c < 6; ++c) sm[c][t] = sel_max(sm[c][t], sm[c][t + s]);
        }
        __syncthreads();
    }
    // result lives in part[2*nPart], part[2*nPart+1]
    if (t == 0) {
        part[2 * nPart] = make_float4(sm[0][0], sm[1][0], sm[2][0], 0.f);
        part[2 * nPart + 1] = make_float4(sm[3][0], sm[4][0], sm[5][0], 0.f);
    }
}

// SeMorton64::ExpandBits, SeMorton.h:94-101
__device__ __forceinline__ uint64_t expand_bits(uint64_t b) {
    b = (b | (b << 32)) & 0xFFFF00000000FFFFull;
    b = (b | (b << 16)) & 0x00FF0000FF0000FFull;
    b = (b | (b << 8)) & 0xF00F00F00F00F00Full;
    b = (b | (b << 4)) & 0x30C30C30C30C30C3ull;
    return (b | (b << 2)) & 0x9249249249249249ull;
}

// Math::Clamp(a, lo, hi) = Min(Max(lo, a), hi) with SE_MIN/SE_MAX ternaries
// (SeMath.h:100-103, SePreDefine.h:37-38): a NaN input yields hi.
__device__ __forceinline__ float ref_clamp(float a, float lo, float hi) {
    float m = (lo > a) ? lo : a;
    return (m < hi) ? m : hi;
}

__global__ __launch_bounds__(256) void k_morton(const float4* __restrict__ pos, const float4* __restrict__ box,
                                                int n, uint64_t* __restrict__ code, int* __restrict__ iota) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    float4 lo = box[0], hi = box[1];
    float4 p = pos[v];
    // (p - Lower) / Extent(), per component IEEE sub/div (.cpp:225)
    float tx = __fdiv_rn(__fsub_rn(p.x, lo.x), __fsub_rn(hi.x, lo.x));
    float ty = __fdiv_rn(__fsub_rn(p.y, lo.y), __fsub_rn(hi.y, lo.y));
    float tz = __fdiv_rn(__fsub_rn(p.z, lo.z), __fsub_rn(hi.z, lo.z));
    // SeMorton64::Encode, SeMorton.h:75-86
    tx = ref_clamp(__fmul_rn(tx, 2097152.0f), 0.0f, 2097151.0f);
    ty = ref_clamp(__fmul_rn(ty, 2097152.0f), 0.0f, 2097151.0f);
    tz = ref_clamp(__fmul_rn(tz, 2097152.0f), 0.0f, 2097151.0f);
    uint64_t xx = expand_bits((uint64_t)tx), yy = expand_bits((uint64_t)ty), zz = expand_bits((uint64_t)tz);
    code[v] = (xx << 2) + (yy << 1) + zz;
    iota[v] = v;
}

__global__ __launch_bounds__(256) void k_inverse_map(const int* __restrict__ s2o, int n, int* __restrict__ o2s) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) o2s[s2o[v]] = v;
}

// MapHessianTable: ELL table [k][vid] in sorted ids, slot 0 = self.
__global__ __launch_bounds__(256) void k_ell_map(const int* __restrict__ s2o, const int* __restrict__ o2s,
                                                 const int* __restrict__ starts, const int* __restrict__ idx, int n,
                                                 int* __restrict__ nbrNum, int* __restrict__ nbr) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    int o = s2o[v];
    int b = starts[o], deg = starts[o + 1] - b;
    nbrNum[v] = deg + 1;
    nbr[v] = v;
    for (int k = 1; k <= deg; ++k) nbr[(size_t)k * n + v] = o2s[idx[b + k - 1]];
}

int run_allocate(mas_context* h, const float* pos4, const int* starts, const int* idx, const int* edges4,
                 const int* faces4) {
    const int nV = h->nV;
    hipStream_t s = h->stream;
    int rc;
    // Host-side size bookkeeping (the reference computes these in DoAlllocation, .cpp:137-191).
    if (!h->allocated) {
        int sz = ceil32(nV), total = sz, nl = 1;  // ComputeLevelNums, .cpp:112-135
        while (sz > 32) {
            sz /= 32;
            nl++;
            sz = ceil32(sz);
            total += sz;
        }
        (void)total;
        h->natL = nl;
        h->L = (h->cfg.max_levels > 0 && h->cfg.max_levels < nl) ? h->cfg.max_levels : nl;
        if (h->L > kMaxLevels) return fail(h, MAS_ERR_LEVELS, "more than 5 levels (reference B-6); set max_levels");
    }
    const int nnz = starts[nV];
    if (nnz < 0) return fail(h, MAS_ERR_ARG, "negative CSR size");
    int maxDeg = 0;
    for (int v = 0; v < nV; ++v) {
        int d = starts[v + 1] - starts[v];
        if (d < 0) return fail(h, MAS_ERR_ARG, "CSR starts not monotone");
        maxDeg = std::max(maxDeg, d);
    }
    for (int k = 0; k < nnz; ++k)
        if (idx[k] < 0 || idx[k] >= nV) return fail(h, MAS_ERR_ARG, "CSR neighbour id out of range");
    if (h->allocated && maxDeg + 1 > h->maxNbr)
        return fail(h, MAS_ERR_STATE, "valence grew after the first Allocate");
    // B-1: the reference re-sorts only on its first call (m_frameIndex % 17).
    const int period = h->cfg.resort_period;
    const bool sortNow = !h->allocated || (period > 0 && h->allocCalls % period == 0);
    h->allocCalls++;
    h->nnz = nnz;
    if (!h->allocated) h->maxNbr = maxDeg + 1;

    if ((rc = ensure(h, h->pos, (size_t)nV * 16)) || (rc = ensure(h, h->starts, (size_t)(nV + 1) * 4)) ||
        (rc = ensure(h, h->idx, (size_t)nnz * 4)))
        return rc;
    if ((rc = hip_check(h, hipMemcpyAsync(h->pos.p, pos4, (size_t)nV * 16, hipMemcpyHostToDevice, s), "H2D pos")) ||
        (rc = hip_check(h, hipMemcpyAsync(h->starts.p, starts, (size_t)(nV + 1) * 4, hipMemcpyHostToDevice, s),
                        "H2D starts")) ||
        (rc = hip_check(h, hipMemcpyAsync(h->idx.p, idx, (size_t)nnz * 4, hipMemcpyHostToDevice, s), "H2D idx")))
        return rc;
    if (edges4 && h->nE > 0) {
        if ((rc = ensure(h, h->edges, (size_t)h->nE * 16))) return rc;
        if ((rc = hip_check(h, hipMemcpyAsync(h->edges.p, edges4, (size_t)h->nE * 16, hipMemcpyHostToDevice, s),
                            "H2D edges")))
            return rc;
    }
    if (faces4 && h->nF > 0) {
        if ((rc = ensure(h, h->faces, (size_t)h->nF * 16))) return rc;
        if ((rc = hip_check(h, hipMemcpyAsync(h->faces.p, faces4, (size_t)h->nF * 16, hipMemcpyHostToDevice, s),
                            "H2D faces")))
            return rc;
    }
    if (!sortNow) {
        h->allocated = true;
        return hip_check(h, hipStreamSynchronize(s), "allocate sync");
    }
    // a new vertex order: the cached contact-free hierarchy (and all derived from it) is stale
    h->meshHierValid = h->liveIsMesh = false;
    hipEventRecord(h->ev[0], s);
    if ((rc = ensure(h, h->aabbPartial, (size_t)(2 * kAabbGrid + 2) * 16)) ||
        (rc = ensure(h, h->morton, (size_t)nV * 8)) || (rc = ensure(h, h->mortonSorted, (size_t)nV * 8)) ||
        (rc = ensure(h, h->iota, (size_t)nV * 4)) || (rc = ensure(h, h->s2o, (size_t)nV * 4)) ||
        (rc = ensure(h, h->o2s, (size_t)nV * 4)) || (rc = ensure(h, h->nbrNum, (size_t)nV * 4)) ||
        (rc = ensure(h, h->nbr, (size_t)h->maxNbr * nV * 4)) || (rc = ensure(h, h->nbrNumRem, (size_t)nV * 4)) ||
        (rc = ensure(h, h->nbrRem, (size_t)h->maxNbr * nV * 4)))
        return rc;
    const int nPart = std::min(kAabbGrid, cdiv(nV, kAabbBlock));
    k_aabb_partial<<<nPart, kAabbBlock, 0, s>>>(P<float4>(h->pos), nV, P<float4>(h->aabbPartial));
    k_aabb_final<<<1, kAabbBlock, 0, s>>>(P<float4>(h->aabbPartial), nPart);
    const float4* box = P<float4>(h->aabbPartial) + 2 * nPart;
    k_morton<<<cdiv(nV, 256), 256, 0, s>>>(P<float4>(h->pos), box, nV, P<uint64_t>(h->morton), P<int>(h->iota));
    if ((rc = sort_pairs(h, P<uint64_t>(h->morton), P<uint64_t>(h->mortonSorted), P<int>(h->iota), P<int>(h->s2o), nV,
                         64, s, "radix sort")))
        return rc;
    k_inverse_map<<<cdiv(nV, 256), 256, 0, s>>>(P<int>(h->s2o), nV, P<int>(h->o2s));
    if ((rc = hip_check(h, hipMemsetAsync(h->nbr.p, 0, (size_t)h->maxNbr * nV * 4, s), "memset nbr"))) return rc;
    k_ell_map<<<cdiv(nV, 256), 256, 0, s>>>(P<int>(h->s2o), P<int>(h->o2s), P<int>(h->starts), P<int>(h->idx), nV,
                                            P<int>(h->nbrNum), P<int>(h->nbr));
    hipEventRecord(h->ev[1], s);
    if ((rc = hip_check(h, hipGetLastError(), "allocate kernels"))) return rc;
    if ((rc = hip_check(h, hipStreamSynchronize(s), "allocate sync"))) return rc;
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    h->stats.allocate_ms = ms;
    h->allocated = true;
    h->prepared = false;
    return MAS_OK;
}

}  // namespace mas
