// k_pcg.hip -- GPU-resident preconditioned conjugate gradients, the caller of
// the MAS apply ("A GPU-resident PCG driver ... CSR 3x3-block
// SpMV (HBM-bound), dot products and axpy in HIP, with a mas_pcg_solve
// C-ABI").  The reference ships no solver; its preconditioner is called from
// a PCG loop (Preconditioning per iteration, SeSchwarzPreconditioner.h:63),
// so this is the loop a simulator would run around it, kept on the device:
//
//   r = b - A x, z = M r, p = z, rz = r.z
//   repeat: Ap = A p; alpha = rz / p.Ap; x += alpha p; r -= alpha Ap;
//           if |r| <= tol |b|: r = b - A x (residual replacement), stop when
//           the TRUE |r| <= tol |b|;
//           z = M r; beta = r.z / rz; p = z + beta p
//
// Residual replacement: the fp32 recursion r -= alpha Ap drifts from b - A x
// (at 1M the recursive residual reached 8.8e-6 while the true one was 5.7e-5),
// so whenever the recursive test passes, r is recomputed from x and the solve
// stops only if the true residual passes too; otherwise it continues from the
// replaced r.  `converged` always refers to the returned x's own residual.
// The solution accumulates in fp64 (x64, 24 B per vertex) and every true
// residual is evaluated with fp64 products and sums: an fp32 x updated in
// place stalls at ~1.1e-5 on the 100x100 grid (alpha p rounds away against
// x), and an fp32 evaluation of b - A x carries ~1e-5 of cancellation error,
// while the exact solution rounded to fp32 has 5.9e-6 (fp64 evaluation) --
// tol = 1e-5 sits right above that floor.  The stop test is taken on the fp32
// vector the caller receives, round(x64).
//
// A is the Prepare input in the caller's vertex order: diag9[nV] and
// off9[nnz] (3x3 column-major, SeMatrix.h:650-682) with the neighbour CSR
// (ranges == nbr_starts, nbr_idx from Allocate).  Vectors are float4[nV]
// (SeVec3fSimd).  Vector arithmetic is fp32; every dot product accumulates in
// fp64 over a fixed grid of workgroups; the kernel that consumes a dot
// product sums the per-workgroup partials itself, in the same fixed order in
// every workgroup (no single-workgroup "finish" launches), so a solve is
// run-to-run deterministic.  The scalars (rz, |r|^2, the stop flag) live in
// device memory: the host enqueues iterations in chunks and reads the done
// flag once per chunk, one chunk behind (pinned read-back words, so the queue
// never drains); every kernel of a finished solve exits at its first
// instruction.
//
// SpMV: G lanes per row (G = 8 for the cloth valence, 16/32 above), lane j
// takes the row's neighbours j, j+G, ...: the 36-byte blocks of consecutive
// rows are contiguous in the CSR, so one wave-instruction reads ~64
// consecutive blocks; the G partial products are combined by a fixed xor
// butterfly; each wave works on 4 row groups at a time so their dependent
// load chains overlap.  Per iteration: spmv, update_xr, true (residual
// replacement, exits at once unless the recursive test passed), the apply (or
// copy) -- whose fine kernel also emits the r.z partials -- and update_p,
// which takes the stop decision (iteration count, done flag) and forms p.
// Every kernel, the apply's included, exits at its first instruction once the
// solve is done, so the chunks enqueued past convergence cost launches only.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "mas_internal.h"

namespace mas {

#ifndef MAS_PCG_THREADS
#define MAS_PCG_THREADS 512
#endif
constexpr int kPcgThreads = MAS_PCG_THREADS;
#ifndef MAS_SPMV_NT
#define MAS_SPMV_NT 1
#endif
#ifndef MAS_PCG_BLOCKS
#define MAS_PCG_BLOCKS 1024
#endif
constexpr int kPcgBlocks = MAS_PCG_BLOCKS;  // fixed grid: partial sums in a fixed order

struct PcgState {
    double rz[2];  // r.z of the current / next iteration (slot it & 1)
    double rr, bb, alpha, tol2, rrTrue;
    int done, iters, maxIters, firstPass, replacements, pad;
};

// partial-sum slots; RRX: r.r of the fp32-rounded x64 (the returned vector's residual)
enum { kPartPAp = 0, kPartRR = 1, kPartRZ = 2, kPartBB = 3, kPartRRX = 4, kParts = 5 };

__device__ __forceinline__ float3 mat3_mul(const float* __restrict__ src, float4 x) {
    // column-major 3x3: y_i = sum_j m[3 j + i] x_j.  The 36-byte block is
    // 4-byte aligned: a memcpy lets the compiler use two dwordx4 + one dword
    // loads (unaligned-access mode) instead of nine dword loads.
    float m[9];
    __builtin_memcpy(m, src, 36);
    return make_float3(__fadd_rn(__fadd_rn(__fmul_rn(m[0], x.x), __fmul_rn(m[3], x.y)), __fmul_rn(m[6], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[1], x.x), __fmul_rn(m[4], x.y)), __fmul_rn(m[7], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[2], x.x), __fmul_rn(m[5], x.y)), __fmul_rn(m[8], x.z)));
}

// mat3_mul of the transposed block: y_i = sum_j m[3 i + j] x_j, in mat3_mul's
// order (for a = m^T, mat3_mul(a, x) reads a[i], a[3 + i], a[6 + i] = m[3 i],
// m[3 i + 1], m[3 i + 2])
__device__ __forceinline__ float3 mat3_mul_t(const float (&m)[9], float4 x) {
    return make_float3(__fadd_rn(__fadd_rn(__fmul_rn(m[0], x.x), __fmul_rn(m[1], x.y)), __fmul_rn(m[2], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[3], x.x), __fmul_rn(m[4], x.y)), __fmul_rn(m[5], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[6], x.x), __fmul_rn(m[7], x.y)), __fmul_rn(m[8], x.z)));
}

__device__ __forceinline__ void add3(float3& a, float3 b) {
    a.x = __fadd_rn(a.x, b.x);
    a.y = __fadd_rn(a.y, b.y);
    a.z = __fadd_rn(a.z, b.z);
}

// (A x)[v] for R rows per G-lane group at once (rows base + r * 64/G + lane/G):
// every first-neighbour load of the R rows is issued before any is consumed
// (the chain starts -> idx -> x is three dependent loads; a grid-stride loop
// over single rows was latency-bound at 100 us for 1M rows).  Lane j takes
// neighbours j, j+G, ... in CSR order, lane 0 adds the diagonal first; then a
// fixed xor butterfly over the group.  The full sums are returned in every
// lane of the group.
template <int G, int R>
__device__ __forceinline__ void spmv_rows(int base, int nV, int lane, const int* __restrict__ starts,
                                          const int* __restrict__ idx, const float* __restrict__ diag,
                                          const float* __restrict__ off, const float4* __restrict__ x,
                                          int (&v)[R], float3 (&acc)[R]) {
    const int sub = lane % G;
    int e[R], e1[R], nb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v[r] = base + r * (64 / G) + lane / G;
        const bool valid = v[r] < nV;
        e[r] = valid ? starts[v[r]] + sub : 0;
        e1[r] = valid ? starts[v[r] + 1] : 0;
    }
    float m[R][9];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool has = e[r] < e1[r];
        nb[r] = has ? idx[e[r]] : 0;
        __builtin_memcpy(m[r], off + 9 * (size_t)(has ? e[r] : 0), 36);
    }
    float4 xn[R], xd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        xn[r] = x[nb[r]];
        xd[r] = x[v[r] < nV ? v[r] : 0];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc[r] = make_float3(0.f, 0.f, 0.f);
        if (sub == 0 && v[r] < nV) acc[r] = mat3_mul(diag + 9 * (size_t)v[r], xd[r]);
        if (e[r] < e1[r]) add3(acc[r], mat3_mul(m[r], xn[r]));
        for (int ee = e[r] + G; ee < e1[r]; ee += G) add3(acc[r], mat3_mul(off + 9 * (size_t)ee, x[idx[ee]]));
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            acc[r].x = __fadd_rn(acc[r].x, __shfl_xor(acc[r].x, o));
            acc[r].y = __fadd_rn(acc[r].y, __shfl_xor(acc[r].y, o));
            acc[r].z = __fadd_rn(acc[r].z, __shfl_xor(acc[r].z, o));
        }
    }
}
constexpr int kSpmvRows = 1;  // row groups per wave and pass

// The SpMV's CSR blocks in wave-slot ELL form, built once per solve: a group
// of 64/G consecutive rows is one wave-row of 64 slots (slot = row-in-group *
// G + j, j = the row's j-th CSR entry, j < G), stored component-major:
// ellOff[group * 576 + q * 64 + slot] = off9[9 e + q], ellIdx[group * 64 +
// slot] = idx[e] (-1: no entry).  Each of a lane's nine off loads is then one
// 256-byte coalesced wave access instead of a 36-byte-strided sweep (the CSR
// form's 64 lanes x 36 B span 18 cache lines per instruction), and the idx
// load no longer waits for starts.  Entries j >= G (rows longer than G) stay
// in the CSR arrays.  Same entries on the same lanes in the same order:
// bitwise equal to the CSR form.
// SYM (A/B, env MAS_PCG_SYM=1; measured slower, so off by default: 1M +
// contacts SpMV 86 -> 94 us in this layout, 96 and 110 us in two earlier ones,
// profiles/round6/ab/pcg_sym/ -- the mirrored products cost a cross-lane round
// trip per pass and the compacted rows' loads wait on a word loaded a pass
// ahead): the matrix is symmetric block by block
// wherever the caller's CSR is, so a group's lower entries whose column is
// in the same group (25 % of the slots of the 1M cloth, 5 % of the 4M tet)
// need not be stored: the lane of its mirror slot in the same wave row holds
// the block transposed and forms the slot's product for it (k_pcg_spmv,
// three floats through ds_bpermute).  Only pairs whose
// blocks are bitwise transposes of each other are mirrored (checked here,
// once per solve), so every product -- and the SpMV -- is bitwise the full
// form's.  The n stored slots of a group are packed at the front of its
// 576 floats as four rows of component pairs and one row of the last
// component: (m[2 p], m[2 p + 1]) of the k-th stored slot at float2 p * n + k,
// m[8] at 8 n + k (n = ellCnt[group]; 48 in the cloth's 2 x 4 patches: each
// pair row is three whole 128-byte lines, 1 728 bytes per group instead of
// 2 304, and no line is read by two load instructions -- rows of single
// components would share lines between neighbouring rows).  ellIdx packs the neighbour id (bits
// 0-23), whether the slot is mirrored (bit 24) and the stored position k or
// the mirror slot (bits 25-30); -1 = no entry.
template <int G, bool SYM>
__global__ __launch_bounds__(256) void k_pcg_ell(int nV, int nGroups, const int* __restrict__ starts,
                                                 const int* __restrict__ idx, const float* __restrict__ off,
                                                 float* __restrict__ ellOff, int* __restrict__ ellIdx,
                                                 int* __restrict__ ellCnt) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int gi = t >> 6, slot = t & 63;
    if (gi >= nGroups) return;  // whole waves (nGroups * 64 threads, 256-thread blocks)
    constexpr int rpg = 64 / G;
    const int v = gi * rpg + slot / G, j = slot % G;
    int e = -1;
    if (v < nV) {
        const int e0 = starts[v] + j;
        if (e0 < starts[v + 1]) e = e0;
    }
    const int nb = e >= 0 ? idx[e] : -1;
    if (!SYM) {
        ellIdx[t] = nb;
        float* dst = ellOff + (size_t)gi * 576 + slot;
#pragma unroll
        for (int q = 0; q < 9; ++q) dst[q * 64] = e >= 0 ? off[9 * (size_t)e + q] : 0.f;
        return;
    }
    int src = -1;  // the mirror slot
    if (nb >= 0 && nb < v && nb / rpg == gi) {  // a lower entry inside the group: its mirror is in the ELL
        const int su = starts[nb], eu = min(starts[nb + 1], su + G);
        for (int k = su; k < eu; ++k) {
            if (idx[k] != v) continue;
            bool same = true;
#pragma unroll
            for (int q = 0; q < 9; ++q)
                same = same && __float_as_uint(off[9 * (size_t)e + q]) ==
                                   __float_as_uint(off[9 * (size_t)k + (q % 3) * 3 + q / 3]);
            if (same) src = (nb % rpg) * G + (k - su);
            break;
        }
    }
    const bool stored = nb >= 0 && src < 0;
    const unsigned long long mask = __ballot(stored);
    const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    const int n = __popcll(mask);
    ellIdx[t] = nb < 0 ? -1 : stored ? (nb | (pos << 25)) : (nb | (1 << 24) | (src << 25));
    if (stored) {
        float* g = ellOff + (size_t)gi * 576;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<float2*>(g)[q * n + pos] = make_float2(off[9 * (size_t)e + 2 * q], off[9 * (size_t)e + 2 * q + 1]);
        g[8 * n + pos] = off[9 * (size_t)e + 8];
    }
    if (slot == 0) ellCnt[gi] = n;
}

// spmv_rows on the ELL form (base is a multiple of 64/G: XcdRows deals whole
// row groups)
template <int G, int R>
__device__ __forceinline__ void spmv_rows_ell(int base, int nV, int lane, const int* __restrict__ starts,
                                              const int* __restrict__ idx, const float* __restrict__ diag,
                                              const float* __restrict__ off, const float* __restrict__ ellOff,
                                              const int* __restrict__ ellIdx, const float4* __restrict__ x,
                                              int (&v)[R], float3 (&acc)[R]) {
    const int sub = lane % G;
    const int g0 = base / (64 / G);
    int e[R], e1[R], nb[R];
    float m[R][9];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v[r] = base + r * (64 / G) + lane / G;
        // the matrix streams once per SpMV (302 MB at 1M, beyond the Infinity
        // Cache): nontemporal, so it does not evict the gathered vector
        if (MAS_SPMV_NT) {
            nb[r] = __builtin_nontemporal_load(ellIdx + (size_t)(g0 + r) * 64 + lane);
#pragma unroll
            for (int q = 0; q < 9; ++q)
                m[r][q] = __builtin_nontemporal_load(ellOff + (size_t)(g0 + r) * 576 + q * 64 + lane);
        } else {
            nb[r] = ellIdx[(size_t)(g0 + r) * 64 + lane];
#pragma unroll
            for (int q = 0; q < 9; ++q) m[r][q] = ellOff[(size_t)(g0 + r) * 576 + q * 64 + lane];
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {  // only rows longer than G read the CSR arrays
        const bool valid = v[r] < nV;
        e[r] = valid ? starts[v[r]] + sub : 0;
        e1[r] = valid ? starts[v[r] + 1] : 0;
    }
    float4 xn[R], xd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        xn[r] = x[nb[r] >= 0 ? nb[r] : 0];
        xd[r] = x[v[r] < nV ? v[r] : 0];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc[r] = make_float3(0.f, 0.f, 0.f);
        if (sub == 0 && v[r] < nV) acc[r] = mat3_mul(diag + 9 * (size_t)v[r], xd[r]);
        if (nb[r] >= 0) add3(acc[r], mat3_mul(m[r], xn[r]));
        for (int ee = e[r] + G; ee < e1[r]; ee += G) add3(acc[r], mat3_mul(off + 9 * (size_t)ee, x[idx[ee]]));
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            acc[r].x = __fadd_rn(acc[r].x, __shfl_xor(acc[r].x, o));
            acc[r].y = __fadd_rn(acc[r].y, __shfl_xor(acc[r].y, o));
            acc[r].z = __fadd_rn(acc[r].z, __shfl_xor(acc[r].z, o));
        }
    }
}


// XCD-aware row ranges: workgroups are dealt round-robin over the 8 XCDs
// (b and b + 8 share one; speed only, never correctness), so workgroups
// b % 8 == k sweep the k-th contiguous eighth of the rows.  A row's
// neighbours (+-1, +-W on the grid) then sit in the same XCD's L2 and the
// x gathers stop going to the Infinity Cache.
constexpr int kXcds = 8;
struct XcdRows {
    int first, end, stride;
    __device__ __forceinline__ XcdRows(int nV, int rowsPerWave) {
        const int xcd = blockIdx.x % kXcds, j = blockIdx.x / kXcds;
        const int wavesPerXcd = (kPcgBlocks / kXcds) * (kPcgThreads / 64);
        // chunks are whole row groups, so no group straddles two chunks
        const int chunk = ((nV + kXcds - 1) / kXcds + rowsPerWave - 1) / rowsPerWave * rowsPerWave;
        const int c0 = xcd * chunk;
        end = min(nV, c0 + chunk);
        first = c0 + (j * (kPcgThreads / 64) + (int)(threadIdx.x >> 6)) * rowsPerWave;
        stride = wavesPerXcd * rowsPerWave;
    }
};

__device__ __forceinline__ double dot3(float3 a, float4 b) {
    return (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z;
}

// workgroup sum of one double per thread -> partial[blockIdx.x] (fixed order)
__device__ __forceinline__ void block_partial(double a, double* __restrict__ partial) {
    __shared__ double sa[kPcgThreads / 64];
    // one static LDS slot array for every call in a kernel: thread 0 may still
    // be reading the previous call's sums (k_pcg_residual calls this twice)
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if ((threadIdx.x & 63) == 0) sa[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kPcgThreads / 64; ++i) t += sa[i];
        partial[blockIdx.x] = t;
    }
}

// every workgroup: the same fixed-order sum of n partials (kPcgBlocks by default)
__device__ __forceinline__ double sum_partials(const double* __restrict__ partial, int n = kPcgBlocks) {
    __shared__ double sa[kPcgThreads];
    __syncthreads();
    // thread t adds partials t, t + kPcgThreads, ... in order; a batch's loads
    // are all issued before its first add (the r.z partials of the fine
    // kernel are 8 456 at 1M: 17 per thread)
    constexpr int kBatch = 8;
    double t = 0.0;
    for (int i0 = threadIdx.x; i0 < n; i0 += kBatch * kPcgThreads) {
        double v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = i0 + k * kPcgThreads;
            v[k] = i < n ? partial[i] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (i0 + k * kPcgThreads < n) t += v[k];
    }
    sa[threadIdx.x] = t;
    __syncthreads();
    for (int s = kPcgThreads / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) sa[threadIdx.x] += sa[threadIdx.x + s];
        __syncthreads();
    }
    return sa[0];
}

// the solution's fp64 accumulator, one per vertex
struct X64 {  // 24 B: no padding lane (a quarter less traffic than a double4)
    double x, y, z;
};
__device__ __forceinline__ void ld3(const float4* __restrict__ p, int v, double (&o)[3]) {
    const float4 a = p[v];
    o[0] = a.x; o[1] = a.y; o[2] = a.z;
}
__device__ __forceinline__ void ld3(const X64* __restrict__ p, int v, double (&o)[3]) {
    const X64 a = p[v];
    o[0] = a.x; o[1] = a.y; o[2] = a.z;
}
// acc += M x with M a column-major 3x3 of fp32, in fp64; xr: the same with x rounded to fp32
__device__ __forceinline__ void mat3_mad_d(const float* __restrict__ src, const double (&x)[3], double (&acc)[3],
                                           double (&accR)[3]) {
    float m[9];
    __builtin_memcpy(m, src, 36);
    double xr[3];
    for (int j = 0; j < 3; ++j) xr[j] = (double)(float)x[j];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            acc[i] = fma((double)m[3 * j + i], x[j], acc[i]);
            accR[i] = fma((double)m[3 * j + i], xr[j], accR[i]);
        }
}

// The true residual in fp64 over this workgroup's rows (G lanes per row, a
// fixed xor butterfly): r = fp32(b - A x) is written, rr = |fp32 r|^2,
// bb = |b|^2, rrx = |b - A round32(x)|^2 (the residual of the fp32 vector
// the caller gets back).  XV: float4 (an fp32 x) or X64.
template <int G, class XV>
__device__ __forceinline__ void residual_rows(int nV, const int* __restrict__ starts, const int* __restrict__ idx,
                                              const float* __restrict__ diag, const float* __restrict__ off,
                                              const XV* __restrict__ x, const float4* __restrict__ b,
                                              float4* __restrict__ r, double& rr, double& bb, double& rrx) {
    const int lane = threadIdx.x & 63, sub = lane % G;
    XcdRows xr(nV, 64 / G);
    rr = 0.0;
    bb = 0.0;
    rrx = 0.0;
    for (int base = xr.first; base < xr.end; base += xr.stride) {
        const int v = base + lane / G;
        const bool valid = v < nV;
        double acc[3] = {0.0, 0.0, 0.0}, accR[3] = {0.0, 0.0, 0.0};
        if (valid) {
            double xv[3];
            if (sub == 0) {
                ld3(x, v, xv);
                mat3_mad_d(diag + 9 * (size_t)v, xv, acc, accR);
            }
            const int e1 = starts[v + 1];
            for (int e = starts[v] + sub; e < e1; e += G) {
                ld3(x, idx[e], xv);
                mat3_mad_d(off + 9 * (size_t)e, xv, acc, accR);
            }
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1)
            for (int i = 0; i < 3; ++i) {
                acc[i] += __shfl_xor(acc[i], o);
                accR[i] += __shfl_xor(accR[i], o);
            }
        if (sub == 0 && valid) {
            const float4 bv = b[v];
            const double bd[3] = {bv.x, bv.y, bv.z};
            float rf[3];
            for (int i = 0; i < 3; ++i) {
                rf[i] = (float)(bd[i] - acc[i]);
                rr += (double)rf[i] * rf[i];
                bb += bd[i] * bd[i];
                const double e = bd[i] - accR[i];
                rrx += e * e;
            }
            r[v] = make_float4(rf[0], rf[1], rf[2], 0.f);
        }
    }
}

// r = b - A x0 (fp64 evaluation); partials r.r (kPartRR) and b.b (kPartBB);
// x64 = x0 when given.  Also the final pass over the returned x (r = scratch,
// x64 null).
template <int G>
__global__ __launch_bounds__(kPcgThreads) void k_pcg_residual(int nV, const int* __restrict__ starts,
                                                              const int* __restrict__ idx,
                                                              const float* __restrict__ diag,
                                                              const float* __restrict__ off,
                                                              const float4* __restrict__ x,
                                                              const float4* __restrict__ b, float4* __restrict__ r,
                                                              X64* __restrict__ x64, double* __restrict__ part) {
    if (x64)
        for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
            const float4 a = x[v];
            x64[v] = X64{a.x, a.y, a.z};
        }
    double rr, bb, rrx;
    residual_rows<G>(nV, starts, idx, diag, off, x, b, r, rr, bb, rrx);
    block_partial(rr, part + kPartRR * kPcgBlocks);
    block_partial(bb, part + kPartBB * kPcgBlocks);
}

// Residual replacement after update_xr: only when the recursive residual
// passes the stop test (the same decision in every workgroup), r = b - A x64
// and the partials of |b - A round32(x64)|^2 (kPartRRX), from which update_p
// takes the decision.
template <int G>
__global__ __launch_bounds__(kPcgThreads) void k_pcg_true(int nV, const int* __restrict__ starts,
                                                          const int* __restrict__ idx, const float* __restrict__ diag,
                                                          const float* __restrict__ off, const X64* __restrict__ x64,
                                                          const float4* __restrict__ b, float4* __restrict__ r,
                                                          const PcgState* __restrict__ st, double* __restrict__ part) {
    if (st->done) return;
    const double rr = sum_partials(part + kPartRR * kPcgBlocks);
    if (!(rr <= st->tol2 * st->bb)) return;
    double rt, bb, rrx;
    residual_rows<G>(nV, starts, idx, diag, off, x64, b, r, rt, bb, rrx);
    block_partial(rrx, part + kPartRRX * kPcgBlocks);
}

// the returned solution: x = round32(x64)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_xout(int nV, const X64* __restrict__ x64, float4* __restrict__ x) {
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const X64 a = x64[v];
        x[v] = make_float4((float)a.x, (float)a.y, (float)a.z, 0.f);
    }
}

// 0 iterations done yet: stop at once if |r0| <= tol |b| (or max_iters == 0)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_start(const double* __restrict__ part,
                                                           PcgState* __restrict__ st) {
    const double rr = sum_partials(part + kPartRR * kPcgBlocks);
    const double bb = sum_partials(part + kPartBB * kPcgBlocks);
    if (threadIdx.x == 0) {
        st->rr = rr;
        st->bb = bb;
        st->iters = 0;
        st->done = (rr <= st->tol2 * bb) || st->maxIters <= 0;
    }
}

__global__ __launch_bounds__(kPcgThreads) void k_pcg_true_finish(const double* __restrict__ part,
                                                                 PcgState* __restrict__ st) {
    const double rr = sum_partials(part + kPartRR * kPcgBlocks);
    if (threadIdx.x == 0) st->rrTrue = rr;
}

struct PDecision {
    bool stop;
    float beta;
};
// The end of iteration it (every workgroup takes the same decision from the
// same partials; workgroup 0 records it): the stop test and beta.
__device__ __forceinline__ PDecision p_decision(int it, PcgState* __restrict__ st, const double* __restrict__ part,
                                                const double* __restrict__ rzPart, int nRz) {
    double rr = sum_partials(part + kPartRR * kPcgBlocks);
    const double lim = st->tol2 * st->bb;
    const bool replaced = rr <= lim;
    if (replaced) rr = sum_partials(part + kPartRRX * kPcgBlocks);
    const bool stop = (replaced && rr <= lim) || it + 1 >= st->maxIters;
    const double rzOld = st->rz[it & 1];
    const double rzNew = sum_partials(rzPart, nRz);
    __syncthreads();  // every thread has read st before workgroup 0 writes it
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->rr = rr;
        st->iters = it + 1;
        st->rz[(it + 1) & 1] = rzNew;
        if (replaced) {
            if (st->firstPass == 0) st->firstPass = it + 1;
            st->replacements++;
        }
        if (stop) st->done = 1;
    }
    return PDecision{stop, (float)(rzNew / rzOld)};
}

__device__ __forceinline__ float4 p_next(float beta, float4 pv, float4 zv) {
    return make_float4(__fmaf_rn(beta, pv.x, zv.x), __fmaf_rn(beta, pv.y, zv.y), __fmaf_rn(beta, pv.z, zv.z), 0.f);
}

// Ap = A p; partials p.Ap
// Occupancy: the fused form needs 70 VGPRs, i.e. 7 waves per SIMD, so a CU
// holds three of the fixed grid's 512-thread workgroups and the last quarter
// of the 1 024 runs as a second, quarter-full round.  Capped at 64 VGPRs (8
// waves per SIMD, 12 bytes per lane spilled: MAS_SPMV_WAVES=8) all 1 024 are
// resident at once, but the spills cost more: 1M + contacts 0.2280-0.2304 ->
// 0.2364-0.2365 ms per MAS iteration, unpreconditioned 0.1130-0.1155 ->
// 0.1217 (profiles/round6/ab/pcg_spmv_waves/).  0 (the default): no cap.
#ifndef MAS_SPMV_WAVES
#define MAS_SPMV_WAVES 0
#endif
constexpr int kSpmvWaves = MAS_SPMV_WAVES > 0 ? MAS_SPMV_WAVES : 1;
#ifndef MAS_SPMV_PIPE
#define MAS_SPMV_PIPE 1
#endif
// One ELL row group's matrix stream: the neighbour ids and the nine
// component rows of its 64 slots (spmv_rows_ell's layout).
struct EllSlot {
    int nb;  // neighbour id (-1: no entry); SYM: the packed word (k_pcg_ell)
    float m[9];
};
// SYM: w = the group's packed word for this lane and n its stored count,
// loaded a pass ahead (the component addresses depend on them)
template <int G, bool SYM>
__device__ __forceinline__ void ell_load(int g0, int lane, const float* __restrict__ ellOff,
                                         const int* __restrict__ ellIdx, int w, int n, EllSlot& e) {
    if (SYM) {
        e.nb = w;
        // a mirrored or empty slot loads the group's first stored block (a line
        // the stored slots fetch anyway) and ignores it
        typedef float v2 __attribute__((ext_vector_type(2)));
        const int k = (w & (1 << 24)) ? 0 : ((w >> 25) & 63);
        const float* g = ellOff + (size_t)g0 * 576;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v2 t = __builtin_nontemporal_load(reinterpret_cast<const v2*>(g) + q * n + k);
            e.m[2 * q] = t.x;
            e.m[2 * q + 1] = t.y;
        }
        e.m[8] = __builtin_nontemporal_load(g + 8 * n + k);
        return;
    }
    e.nb = __builtin_nontemporal_load(ellIdx + (size_t)g0 * 64 + lane);
    __builtin_amdgcn_sched_barrier(0);  // nb first: the gathers wait for it alone
#pragma unroll
    for (int q = 0; q < 9; ++q) e.m[q] = __builtin_nontemporal_load(ellOff + (size_t)g0 * 576 + q * 64 + lane);
}

// FUSE (MAS_PCG_FUSE_P, the default): the previous iteration's update_p
// inside this launch -- its stop decision and beta (p_decision), and
// p = z + beta p_old evaluated wherever a p entry is read (each neighbour's
// too: the same fma on the same inputs, so the same bits as the stored p of
// the unfused form); every row stores its own p into pOut (p_old stays
// intact for the other rows' gathers).  One launch and one pass over z and p
// less per iteration; the iterates are bitwise those of the unfused form.
template <int G, bool FUSE, bool SYM>
__global__ __launch_bounds__(kPcgThreads) __attribute__((amdgpu_waves_per_eu(SYM && kSpmvWaves == 1 ? 7 : kSpmvWaves))) void k_pcg_spmv(int nV, const int* __restrict__ starts,
                                                          const int* __restrict__ idx, const float* __restrict__ diag,
                                                          const float* __restrict__ off,
                                                          const float* __restrict__ ellOff,
                                                          const int* __restrict__ ellIdx, const int* __restrict__ ellCnt,
                                                          const float4* __restrict__ p,
                                                          float4* __restrict__ ap, PcgState* __restrict__ st,
                                                          double* __restrict__ part, const float4* __restrict__ zf,
                                                          float4* __restrict__ pOut, const double* __restrict__ rzPart,
                                                          int nRz, int itPrev) {
    if (st->done) return;
    float beta = 0.f;
    if (FUSE) {
        const PDecision d = p_decision(itPrev, st, part, rzPart, nRz);
        if (d.stop) return;
        beta = d.beta;
    }
    auto pv = [&](int j) { return FUSE ? p_next(beta, p[j], zf[j]) : p[j]; };
    const int lane = threadIdx.x & 63, sub = lane % G;
    constexpr int rowsPerWave = kSpmvRows * (64 / G);
    XcdRows xr(nV, rowsPerWave);
    double pap = 0.0;
    if (MAS_SPMV_PIPE && MAS_SPMV_NT && kSpmvRows == 1) {
        // Software-pipelined over the wave's passes: the next group's matrix
        // stream is issued after this group's vector gathers, so it is in
        // flight while they return and the block products run (the load
        // counter is in order: loads issued before the gathers would have to
        // land first).  Same entries, lanes and order as spmv_rows_ell.
        // Branch-free until the products (clamped addresses; a branch would
        // make the compiler drain every load at the join).
        const int lastGroup = (xr.end - 1) / (64 / G);
        auto groupOf = [&](int base) { return min(base / (64 / G), lastGroup); };
        // one pass: cur's products, nxt's stream issued after cur's gathers;
        // the two buffers alternate (a register copy would wait for the loads).
        // SYM: a group's packed words are loaded a pass before its components
        // (whose addresses they hold), after the current pass's stream, so the
        // in-order load counter waits for nothing newer; useW is nxt's,
        // loadW receives the group's after it
        auto pass = [&](int base, const EllSlot& cur, EllSlot& nxt, int useW, int useN, int& loadW, int& loadN) {
            const int v = base + lane / G;
            const int curNb = SYM ? (cur.nb < 0 ? -1 : (cur.nb & 0xFFFFFF)) : cur.nb;
            const bool valid = v < nV;
            const int vc = valid ? v : 0;
            const float4 xn = pv(curNb >= 0 ? curNb : 0);
            const float4 xd = pv(vc);
            const int e = starts[vc] + sub, e1 = valid ? starts[vc + 1] : 0;
            float dg[9];
            __builtin_memcpy(dg, diag + 9 * (size_t)vc, 36);
            ell_load<G, SYM>(groupOf(base + xr.stride), lane, ellOff, ellIdx, useW, useN, nxt);
            if (SYM) {
                const int g2 = groupOf(base + 2 * xr.stride);
                loadW = __builtin_nontemporal_load(ellIdx + (size_t)g2 * 64 + lane);
                loadN = __builtin_nontemporal_load(ellCnt + g2);
            }
            const float3 zero = make_float3(0.f, 0.f, 0.f);
            const float3 dp = mat3_mul(dg, xd);
            float3 acc = sub == 0 && valid ? dp : zero;
            float3 prod = mat3_mul(cur.m, xn);
            if (SYM) {
                // A mirrored slot (row v, column u) needs A_vu p_u = B^T p_u, B =
                // A_uv the block of its mirror slot (row u, column v): that lane
                // holds B and p_u (its own row's vector) and forms B^T p_u with
                // the same operations in the same order as mat3_mul on the
                // transposed block, so the same bits; three floats cross lanes
                const float3 tp = mat3_mul_t(cur.m, xd);
                const int a = ((cur.nb >> 25) & 63) << 2;
                const float3 fromMirror = make_float3(__int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(tp.x))),
                                                      __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(tp.y))),
                                                      __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(tp.z))));
                if (cur.nb >= 0 && ((cur.nb >> 24) & 1)) prod = fromMirror;
            }
            float3 withN = acc;
            add3(withN, prod);
            if (curNb >= 0) acc = withN;
            for (int ee = e + G; ee < e1; ee += G) add3(acc, mat3_mul(off + 9 * (size_t)ee, pv(idx[ee])));
#pragma unroll
            for (int o = G / 2; o > 0; o >>= 1) {
                acc.x = __fadd_rn(acc.x, __shfl_xor(acc.x, o));
                acc.y = __fadd_rn(acc.y, __shfl_xor(acc.y, o));
                acc.z = __fadd_rn(acc.z, __shfl_xor(acc.z, o));
            }
            if (sub == 0 && valid) {
                ap[v] = make_float4(acc.x, acc.y, acc.z, 0.f);
                if (FUSE) pOut[v] = xd;
                pap += dot3(acc, xd);
            }
        };
        EllSlot a, b;
        int wA = 0, wB = 0, nA = 0, nB = 0;
        if (SYM) {
            wA = ellIdx[(size_t)groupOf(xr.first) * 64 + lane];
            nA = ellCnt[groupOf(xr.first)];
            wB = ellIdx[(size_t)groupOf(xr.first + xr.stride) * 64 + lane];
            nB = ellCnt[groupOf(xr.first + xr.stride)];
        }
        ell_load<G, SYM>(groupOf(xr.first), lane, ellOff, ellIdx, wA, nA, a);
        for (int base = xr.first; base < xr.end;) {
            pass(base, a, b, wB, nB, wA, nA);
            base += xr.stride;
            if (base >= xr.end) break;
            pass(base, b, a, wA, nA, wB, nB);
            base += xr.stride;
        }
    } else {
        static_assert(!FUSE || (MAS_SPMV_PIPE && MAS_SPMV_NT && kSpmvRows == 1), "the fused p update needs the pipelined form");
        static_assert(!SYM || (MAS_SPMV_PIPE && MAS_SPMV_NT && kSpmvRows == 1), "the mirrored layout needs the pipelined form");
        for (int base = xr.first; base < xr.end; base += xr.stride) {
            int v[kSpmvRows];
            float3 y[kSpmvRows];
            spmv_rows_ell<G, kSpmvRows>(base, nV, lane, starts, idx, diag, off, ellOff, ellIdx, p, v, y);
#pragma unroll
            for (int q = 0; q < kSpmvRows; ++q) {
                if (sub == 0 && v[q] < nV) {
                    ap[v[q]] = make_float4(y[q].x, y[q].y, y[q].z, 0.f);
                    pap += dot3(y[q], p[v[q]]);
                }
            }
        }
    }
    block_partial(pap, part + kPartPAp * kPcgBlocks);
}

// alpha = rz / p.Ap; x64 += alpha p (fp64); r -= alpha Ap (fp32); partials r.r
__global__ __launch_bounds__(kPcgThreads) void k_pcg_update_xr(int nV, int it, const float4* __restrict__ p,
                                                               const float4* __restrict__ ap, X64* __restrict__ x,
                                                               float4* __restrict__ r, PcgState* __restrict__ st,
                                                               double* __restrict__ part) {
    if (st->done) return;
    const double pap = sum_partials(part + kPartPAp * kPcgBlocks);
    const double alphaD = st->rz[it & 1] / pap;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->alpha = alphaD;
    const float alpha = (float)alphaD;
    double rr = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 pv = p[v], av = ap[v], rv = r[v];
        const X64 xv = x[v];
        x[v] = X64{fma(alphaD, (double)pv.x, xv.x), fma(alphaD, (double)pv.y, xv.y), fma(alphaD, (double)pv.z, xv.z)};
        const float4 rn = make_float4(__fmaf_rn(-alpha, av.x, rv.x), __fmaf_rn(-alpha, av.y, rv.y),
                                      __fmaf_rn(-alpha, av.z, rv.z), 0.f);
        r[v] = rn;
        rr += dot3(make_float3(rn.x, rn.y, rn.z), rn);
    }
    block_partial(rr, part + kPartRR * kPcgBlocks);
}

// start: partials r.z and p = z
__global__ __launch_bounds__(kPcgThreads) void k_pcg_rz(int nV, const float4* __restrict__ r,
                                                        const float4* __restrict__ z, float4* __restrict__ p,
                                                        const PcgState* __restrict__ st, double* __restrict__ part) {
    if (st->done) return;
    double rz = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 zv = z[v];
        rz += dot3(make_float3(zv.x, zv.y, zv.z), r[v]);
        p[v] = zv;
    }
    block_partial(rz, part + kPartRZ * kPcgBlocks);
}

// start: rz[0] = r.z
__global__ __launch_bounds__(kPcgThreads) void k_pcg_rz0(PcgState* __restrict__ st, const double* __restrict__ part) {
    if (st->done) return;
    const double rz = sum_partials(part + kPartRZ * kPcgBlocks);
    if (threadIdx.x == 0) st->rz[0] = rz;
}

// After iteration it: the stop decision, then beta = r.z (new) / r.z (old)
// and p = z + beta p.  The recursive r.r decides whether a replaced residual
// exists (k_pcg_true ran); if so the returned vector's true r.r is the one
// tested and recorded.
// Stop when that passes or it + 1 == max_iters (workgroup 0 records the state;
// every workgroup takes the same decision).  rzPart: the nRz r.z partials of
// this iteration's apply (fine kernel workgroups) or copy.
__global__ __launch_bounds__(kPcgThreads) void k_pcg_update_p(int nV, int it, const float4* __restrict__ z,
                                                              float4* __restrict__ p, PcgState* __restrict__ st,
                                                              const double* __restrict__ part,
                                                              const double* __restrict__ rzPart, int nRz) {
    if (st->done) return;
    const PDecision d = p_decision(it, st, part, rzPart, nRz);
    if (d.stop) return;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads)
        p[v] = p_next(d.beta, p[v], z[v]);
}

// z = r (no preconditioner) with the r.z partials
__global__ __launch_bounds__(kPcgThreads) void k_pcg_copy(int nV, const float4* __restrict__ src,
                                                          float4* __restrict__ dst, const PcgState* __restrict__ st,
                                                          double* __restrict__ rzPart) {
    if (st->done) return;
    double rz = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 a = src[v];
        dst[v] = a;
        rz += dot3(make_float3(a.x, a.y, a.z), a);
    }
    if (rzPart) block_partial(rz, rzPart);
}

template <int G>
static int pcg_loop(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, float4* d_x,
                    const float4* d_b, int maxIters, int precondition, PcgState& host, PcgState* st, hipStream_t s,
                    hipEvent_t e1) {
    const int nV = h->nV;
    float4* r = P<float4>(h->pcgVec);
    float4* z = r + nV;
    float4* p = z + nV;
    float4* ap = p + nV;
    // the fused form's p of odd iterations, before x64: every float4 vector at
    // a 16-byte offset whatever nV is (x64 is 24 B per vertex)
    float4* p2 = ap + nV;
    X64* x64 = reinterpret_cast<X64*>(p2 + nV);
    const bool fuseP = h->pcgFuseP;
    double* part = P<double>(h->pcgPartial);
    const int* idx = P<int>(h->idx);
    const dim3 g(kPcgBlocks), b(kPcgThreads);
    int rc;
    // a pass reads kSpmvRows whole groups from a group-aligned base < nV, so
    // the last pass may read up to kSpmvRows - 1 groups past the rows: they
    // are allocated and filled as empty slots (idx -1)
    const int nGroups = cdiv(nV, 64 / G) + kSpmvRows;
    if ((rc = ensure(h, h->pcgEllOff, (size_t)nGroups * 576 * 4)) ||
        (rc = ensure(h, h->pcgEllIdx, (size_t)nGroups * 64 * 4)) ||
        (rc = ensure(h, h->pcgEllCnt, (size_t)nGroups * 4)))
        return rc;
    float* ellOff = P<float>(h->pcgEllOff);
    int* ellIdx = P<int>(h->pcgEllIdx);
    int* ellCnt = P<int>(h->pcgEllCnt);
    // the mirrored layout packs neighbour ids into 24 bits
    const bool sym = h->pcgSym && nV <= (1 << 24);
    // the apply kernels honour the done flag and the fine kernel emits the
    // r.z partials while this solve runs (cleared on every return path)
    const int nRz = precondition ? fine_grid(h) : kPcgBlocks;
    if ((rc = ensure(h, h->pcgRzPart, (size_t)std::max(nRz, 1) * sizeof(double)))) return rc;
    double* rzPart = P<double>(h->pcgRzPart);
    struct Hooks {
        mas_context* h;
        ~Hooks() { h->applyDone = nullptr; h->applyRzPart = nullptr; }
    } hooks{h};
    h->applyDone = &st->done;
    h->applyRzPart = rzPart;
    if (sym)
        k_pcg_ell<G, true><<<cdiv(nGroups * 64, 256), 256, 0, s>>>(nV, nGroups, d_ranges, idx, d_off9, ellOff, ellIdx,
                                                                  ellCnt);
    else
        k_pcg_ell<G, false><<<cdiv(nGroups * 64, 256), 256, 0, s>>>(nV, nGroups, d_ranges, idx, d_off9, ellOff,
                                                                   ellIdx, ellCnt);
    auto spmv = [&](bool fuse, const float4* pIn, float4* pOut, int itPrev) {
        if (fuse && sym)
            k_pcg_spmv<G, true, true><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, ellOff, ellIdx, ellCnt,
                                                      pIn, ap, st, part, z, pOut, rzPart, nRz, itPrev);
        else if (fuse)
            k_pcg_spmv<G, true, false><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, ellOff, ellIdx, ellCnt,
                                                       pIn, ap, st, part, z, pOut, rzPart, nRz, itPrev);
        else if (sym)
            k_pcg_spmv<G, false, true><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, ellOff, ellIdx, ellCnt,
                                                       pIn, ap, st, part, nullptr, nullptr, nullptr, 0, 0);
        else
            k_pcg_spmv<G, false, false><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, ellOff, ellIdx, ellCnt,
                                                        pIn, ap, st, part, nullptr, nullptr, nullptr, 0, 0);
    };
    k_pcg_residual<G><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, d_x, d_b, r, x64, part);
    k_pcg_start<<<1, b, 0, s>>>(part, st);
    if (precondition) {
        if ((rc = run_apply(h, z, r, s))) return rc;
    } else {
        k_pcg_copy<<<g, b, 0, s>>>(nV, r, z, st, nullptr);
    }
    k_pcg_rz<<<g, b, 0, s>>>(nV, r, z, p, st, part);
    k_pcg_rz0<<<1, b, 0, s>>>(st, part);
    // The host looks at the done flag once per chunk of iterations, one chunk
    // behind: chunk c + 1 is queued before the flag of chunk c is read
    // (through the pinned read-back words, no stream synchronisation), so
    // the GPU never idles on the host's check.  The price is one queued
    // chunk after convergence, whose kernels return at once on st->done.
    // MAS_PCG_LAG=0 selects the synchronous check (A/B).
    static const int lag = [] {
        const char* v = std::getenv("MAS_PCG_LAG");
        return v ? std::atoi(v) : 1;
    }();
    int pendingSeq = 0;
    bool pending = false;
    const int chunk = 4;
    int lastK = -1;
    for (int it = 0; it < maxIters; it += chunk) {
        for (int k = it; k < it + chunk && k < maxIters; ++k) {
            // the fused form: iteration k's p lives in (k even ? p : p2), formed by this SpMV from the last
            float4* pk = fuseP && (k & 1) ? p2 : p;
            if (!fuseP || k == 0)
                spmv(false, pk, nullptr, 0);
            else
                spmv(true, (k & 1) ? p : p2, pk, k - 1);
            k_pcg_update_xr<<<g, b, 0, s>>>(nV, k, pk, ap, x64, r, st, part);
            k_pcg_true<G><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, x64, d_b, r, st, part);
            if (precondition) {
                if ((rc = run_apply(h, z, r, s))) return rc;
            } else {
                k_pcg_copy<<<g, b, 0, s>>>(nV, r, z, st, rzPart);
            }
            if (!fuseP) k_pcg_update_p<<<g, b, 0, s>>>(nV, k, z, p, st, part, rzPart, nRz);
            lastK = k;
        }
        if (lag) {
            int seq = 0, done = 0;
            if ((rc = read_back_post(h, s, {&st->done}, &seq))) return rc;
            if (pending) {
                if ((rc = read_back_wait(h, s, pendingSeq, &done, 1))) return rc;
                if (done) break;
            }
            pendingSeq = seq;
            pending = true;
            continue;
        }
        if ((rc = hip_check(h, hipMemcpyAsync(&host, st, sizeof(host), hipMemcpyDeviceToHost, s), "D2H pcg state")) ||
            (rc = hip_check(h, hipStreamSynchronize(s), "pcg sync")))
            return rc;
        if (host.done) break;
    }
    // the fused form: the last queued iteration's stop decision (its update_p
    // would have been the next SpMV); a finished solve returns at once
    if (fuseP && lastK >= 0) {
        float4* pk = (lastK & 1) ? p2 : p;
        k_pcg_update_p<<<g, b, 0, s>>>(nV, lastK, z, pk, st, part, rzPart, nRz);
    }
    k_pcg_xout<<<g, b, 0, s>>>(nV, x64, d_x);
    hipEventRecord(e1, s);
    // the true residual of the returned x (fp64 evaluation)
    k_pcg_residual<G><<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, d_x, d_b, ap, nullptr, part);
    k_pcg_true_finish<<<1, b, 0, s>>>(part, st);
    return MAS_OK;
}

int run_pcg(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, float4* d_x,
            const float4* d_b, int maxIters, float tol, int precondition, mas_pcg_result* res, hipStream_t s) {
    const int nV = h->nV;
    int rc;
    if (precondition && (rc = pending_giveup(h))) return rc;  // an earlier apply's incomplete z, first
    if ((rc = ensure(h, h->pcgVec, (size_t)nV * (16 * 5 + sizeof(X64)))) ||
        (rc = ensure(h, h->pcgPartial, (size_t)kPcgBlocks * kParts * sizeof(double))) ||
        (rc = ensure(h, h->pcgState, sizeof(PcgState))))
        return rc;
    PcgState* st = P<PcgState>(h->pcgState);
    PcgState init{};
    init.tol2 = (double)tol * (double)tol;
    init.maxIters = maxIters;
    ScopedEvents ev;
    if (!ev.ok()) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1];
    hipEventRecord(e0, s);
    if ((rc = hip_check(h, hipMemcpyAsync(st, &init, sizeof(init), hipMemcpyHostToDevice, s), "H2D pcg state")))
        return rc;
    PcgState host{};
    const int valence = h->maxNbr - 1;  // max neighbours per row (maxNbr counts the vertex itself)
    if (valence <= 8)
        rc = pcg_loop<8>(h, d_diag9, d_off9, d_ranges, d_x, d_b, maxIters, precondition, host, st, s, e1);
    else if (valence <= 16)
        rc = pcg_loop<16>(h, d_diag9, d_off9, d_ranges, d_x, d_b, maxIters, precondition, host, st, s, e1);
    else
        rc = pcg_loop<32>(h, d_diag9, d_off9, d_ranges, d_x, d_b, maxIters, precondition, host, st, s, e1);
    if (rc) return rc;
    if ((rc = hip_check(h, hipMemcpyAsync(&host, st, sizeof(host), hipMemcpyDeviceToHost, s), "D2H pcg state")) ||
        (rc = hip_check(h, hipStreamSynchronize(s), "pcg sync")))
        return rc;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (res) {
        std::memset(res, 0, sizeof(*res));
        res->iterations = host.iters;
        res->converged = host.rrTrue <= host.tol2 * host.bb;  // the returned x's own residual
        res->rel_residual = host.bb > 0 ? sqrt(host.rr / host.bb) : 0.0;
        res->true_rel_residual = host.bb > 0 ? sqrt(host.rrTrue / host.bb) : 0.0;
        res->solve_ms = ms;
        res->first_pass_iterations = host.firstPass;
        res->replacements = host.replacements;
    }
    if ((rc = hip_check(h, hipGetLastError(), "pcg kernels"))) return rc;
    return pending_giveup(h);  // a preconditioner apply whose coarse hand-off gave up fails the solve
}

}  // namespace mas
