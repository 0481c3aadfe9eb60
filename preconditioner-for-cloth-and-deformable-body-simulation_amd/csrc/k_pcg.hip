// k_pcg.hip -- GPU-resident preconditioned conjugate gradients, the caller of
// the MAS apply ("A GPU-resident PCG driver ... CSR 3x3-block
// SpMV (HBM-bound), dot products and axpy in HIP, with a mas_pcg_solve
// C-ABI").  The reference ships no solver; its preconditioner is called from
// a PCG loop (Preconditioning per iteration, SeSchwarzPreconditioner.h:63),
// so this is the loop a simulator would run around it, kept on the device:
//
//   r = b - A x, z = M r, p = z, rz = r.z
//   repeat: Ap = A p; alpha = rz / p.Ap; x += alpha p; r -= alpha Ap;
//           stop when |r| <= tol |b|; z = M r; beta = r.z / rz; p = z + beta p
//
// A is the Prepare input in the caller's vertex order: diag9[nV] and
// off9[nnz] (3x3 column-major, SeMatrix.h:650-682) with the neighbour CSR
// (ranges == nbr_starts, nbr_idx from Allocate).  Vectors are float4[nV]
// (SeVec3fSimd).  Vector arithmetic is fp32; every dot product accumulates in
// fp64 over a fixed grid and is finished by one workgroup in a fixed order, so
// a solve is run-to-run deterministic.  The scalars (alpha, beta, |r|^2, the
// stop flag) live in device memory: the host enqueues iterations in chunks
// and reads the state once per chunk; every kernel of a finished solve exits
// at its first instruction.
#include "mas_internal.h"

namespace mas {

constexpr int kPcgThreads = 256;
constexpr int kPcgBlocks = 1024;  // fixed grid: partial sums in a fixed order

struct PcgState {
    double rz, pAp, rr, bb, alpha, beta, tol2, rrTrue;
    int done, iters, maxIters, pad;
};

__device__ __forceinline__ float3 mat3_mul(const float* __restrict__ m, float4 x) {
    // column-major 3x3: y_i = sum_j m[3 j + i] x_j
    return make_float3(__fadd_rn(__fadd_rn(__fmul_rn(m[0], x.x), __fmul_rn(m[3], x.y)), __fmul_rn(m[6], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[1], x.x), __fmul_rn(m[4], x.y)), __fmul_rn(m[7], x.z)),
                       __fadd_rn(__fadd_rn(__fmul_rn(m[2], x.x), __fmul_rn(m[5], x.y)), __fmul_rn(m[8], x.z)));
}

// y = A x for vertex v (diagonal first, then the neighbours in CSR order)
__device__ __forceinline__ float3 spmv_row(int v, const int* __restrict__ starts, const int* __restrict__ idx,
                                           const float* __restrict__ diag, const float* __restrict__ off,
                                           const float4* __restrict__ x) {
    float3 acc = mat3_mul(diag + 9 * (size_t)v, x[v]);
    const int e0 = starts[v], e1 = starts[v + 1];
    for (int e = e0; e < e1; ++e) {
        const float3 t = mat3_mul(off + 9 * (size_t)e, x[idx[e]]);
        acc.x = __fadd_rn(acc.x, t.x);
        acc.y = __fadd_rn(acc.y, t.y);
        acc.z = __fadd_rn(acc.z, t.z);
    }
    return acc;
}

__device__ __forceinline__ double dot3(float3 a, float4 b) {
    return (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z;
}

// block sum of up to two doubles -> partial[2 * blockIdx.x + {0, 1}]
__device__ __forceinline__ void block_partials(double a, double b, double* __restrict__ partial) {
    __shared__ double sa[kPcgThreads / 64], sb[kPcgThreads / 64];
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sa[w] = a;
        sb[w] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tb = 0.0;
        for (int i = 0; i < kPcgThreads / 64; ++i) {
            ta += sa[i];
            tb += sb[i];
        }
        partial[2 * blockIdx.x] = ta;
        partial[2 * blockIdx.x + 1] = tb;
    }
}

// one workgroup: fixed-order sums of the kPcgBlocks partial pairs
__device__ __forceinline__ void finish_sums(const double* __restrict__ partial, double& a, double& b) {
    __shared__ double sa[kPcgThreads], sb[kPcgThreads];
    double ta = 0.0, tb = 0.0;
    for (int i = threadIdx.x; i < kPcgBlocks; i += kPcgThreads) {
        ta += partial[2 * i];
        tb += partial[2 * i + 1];
    }
    sa[threadIdx.x] = ta;
    sb[threadIdx.x] = tb;
    __syncthreads();
    for (int s = kPcgThreads / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sa[threadIdx.x] += sa[threadIdx.x + s];
            sb[threadIdx.x] += sb[threadIdx.x + s];
        }
        __syncthreads();
    }
    a = sa[0];
    b = sb[0];
}

// r = b - A x; partials (r.r, b.b)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_init(int nV, const int* __restrict__ starts,
                                                          const int* __restrict__ idx, const float* __restrict__ diag,
                                                          const float* __restrict__ off, const float4* __restrict__ x,
                                                          const float4* __restrict__ b, float4* __restrict__ r,
                                                          double* __restrict__ partial) {
    double rr = 0.0, bb = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float3 ax = spmv_row(v, starts, idx, diag, off, x);
        const float4 bv = b[v];
        const float4 rv = make_float4(__fsub_rn(bv.x, ax.x), __fsub_rn(bv.y, ax.y), __fsub_rn(bv.z, ax.z), 0.f);
        r[v] = rv;
        rr += dot3(make_float3(rv.x, rv.y, rv.z), rv);
        bb += dot3(make_float3(bv.x, bv.y, bv.z), bv);
    }
    block_partials(rr, bb, partial);
}

__global__ __launch_bounds__(kPcgThreads) void k_pcg_init_finish(const double* __restrict__ partial,
                                                                 PcgState* __restrict__ st) {
    double rr, bb;
    finish_sums(partial, rr, bb);
    if (threadIdx.x == 0) {
        st->rr = rr;
        st->bb = bb;
        st->iters = 0;
        st->done = (rr <= st->tol2 * bb) || st->maxIters <= 0;
    }
}

// after the loop: |b - A x|^2 (into the spare Ap vector)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_true_finish(const double* __restrict__ partial,
                                                                 PcgState* __restrict__ st) {
    double rr, bb;
    finish_sums(partial, rr, bb);
    if (threadIdx.x == 0) st->rrTrue = rr;
}

// partials (r.z, 0); also p = z on the first call (copy_p)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_rz(int nV, const float4* __restrict__ r,
                                                        const float4* __restrict__ z, float4* __restrict__ p,
                                                        int copy_p, const PcgState* __restrict__ st,
                                                        double* __restrict__ partial) {
    if (st->done) return;
    double rz = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 zv = z[v];
        rz += dot3(make_float3(zv.x, zv.y, zv.z), r[v]);
        if (copy_p) p[v] = zv;
    }
    block_partials(rz, 0.0, partial);
}

// first: rz = r.z; later: beta = r.z / rz, rz = r.z
__global__ __launch_bounds__(kPcgThreads) void k_pcg_rz_finish(const double* __restrict__ partial, int first,
                                                               PcgState* __restrict__ st) {
    if (st->done) return;
    double rz, unused;
    finish_sums(partial, rz, unused);
    if (threadIdx.x == 0) {
        st->beta = first ? 0.0 : rz / st->rz;
        st->rz = rz;
    }
}

// p = z + beta p
__global__ __launch_bounds__(kPcgThreads) void k_pcg_update_p(int nV, const float4* __restrict__ z,
                                                              float4* __restrict__ p,
                                                              const PcgState* __restrict__ st) {
    if (st->done) return;
    const float beta = (float)st->beta;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 zv = z[v], pv = p[v];
        p[v] = make_float4(__fmaf_rn(beta, pv.x, zv.x), __fmaf_rn(beta, pv.y, zv.y), __fmaf_rn(beta, pv.z, zv.z), 0.f);
    }
}

// Ap = A p; partials (p.Ap, 0)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_spmv(int nV, const int* __restrict__ starts,
                                                          const int* __restrict__ idx, const float* __restrict__ diag,
                                                          const float* __restrict__ off, const float4* __restrict__ p,
                                                          float4* __restrict__ ap, const PcgState* __restrict__ st,
                                                          double* __restrict__ partial) {
    if (st->done) return;
    double pap = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float3 y = spmv_row(v, starts, idx, diag, off, p);
        ap[v] = make_float4(y.x, y.y, y.z, 0.f);
        pap += dot3(y, p[v]);
    }
    block_partials(pap, 0.0, partial);
}

__global__ __launch_bounds__(kPcgThreads) void k_pcg_alpha(const double* __restrict__ partial,
                                                           PcgState* __restrict__ st) {
    if (st->done) return;
    double pap, unused;
    finish_sums(partial, pap, unused);
    if (threadIdx.x == 0) {
        st->pAp = pap;
        st->alpha = st->rz / pap;
    }
}

// x += alpha p; r -= alpha Ap; partials (r.r, 0)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_update_xr(int nV, const float4* __restrict__ p,
                                                               const float4* __restrict__ ap, float4* __restrict__ x,
                                                               float4* __restrict__ r,
                                                               const PcgState* __restrict__ st,
                                                               double* __restrict__ partial) {
    if (st->done) return;
    const float alpha = (float)st->alpha;
    double rr = 0.0;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) {
        const float4 pv = p[v], av = ap[v], xv = x[v], rv = r[v];
        x[v] = make_float4(__fmaf_rn(alpha, pv.x, xv.x), __fmaf_rn(alpha, pv.y, xv.y), __fmaf_rn(alpha, pv.z, xv.z),
                           0.f);
        const float4 rn = make_float4(__fmaf_rn(-alpha, av.x, rv.x), __fmaf_rn(-alpha, av.y, rv.y),
                                      __fmaf_rn(-alpha, av.z, rv.z), 0.f);
        r[v] = rn;
        rr += dot3(make_float3(rn.x, rn.y, rn.z), rn);
    }
    block_partials(rr, 0.0, partial);
}

__global__ __launch_bounds__(kPcgThreads) void k_pcg_check(const double* __restrict__ partial,
                                                           PcgState* __restrict__ st) {
    if (st->done) return;
    double rr, unused;
    finish_sums(partial, rr, unused);
    if (threadIdx.x == 0) {
        st->rr = rr;
        st->iters += 1;
        st->done = (rr <= st->tol2 * st->bb) || st->iters >= st->maxIters;
    }
}

__global__ __launch_bounds__(kPcgThreads) void k_pcg_copy(int nV, const float4* __restrict__ src,
                                                          float4* __restrict__ dst, const PcgState* __restrict__ st) {
    if (st->done) return;
    for (int v = blockIdx.x * kPcgThreads + threadIdx.x; v < nV; v += kPcgBlocks * kPcgThreads) dst[v] = src[v];
}

int run_pcg(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, float4* d_x,
            const float4* d_b, int maxIters, float tol, int precondition, mas_pcg_result* res, hipStream_t s) {
    const int nV = h->nV;
    int rc;
    if ((rc = ensure(h, h->pcgVec, (size_t)nV * 16 * 4)) ||
        (rc = ensure(h, h->pcgPartial, (size_t)kPcgBlocks * 2 * sizeof(double))) ||
        (rc = ensure(h, h->pcgState, sizeof(PcgState))))
        return rc;
    float4* r = P<float4>(h->pcgVec);
    float4* z = r + nV;
    float4* p = z + nV;
    float4* ap = p + nV;
    double* part = P<double>(h->pcgPartial);
    PcgState* st = P<PcgState>(h->pcgState);
    const int* idx = P<int>(h->idx);
    PcgState init{};
    init.tol2 = (double)tol * (double)tol;
    init.maxIters = maxIters;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    if ((rc = hip_check(h, hipMemcpyAsync(st, &init, sizeof(init), hipMemcpyHostToDevice, s), "H2D pcg state")))
        return rc;
    const dim3 g(kPcgBlocks), b(kPcgThreads);
    k_pcg_init<<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, d_x, d_b, r, part);
    k_pcg_init_finish<<<1, b, 0, s>>>(part, st);
    if (precondition) {
        if ((rc = run_apply(h, z, r, s))) return rc;
    } else {
        k_pcg_copy<<<g, b, 0, s>>>(nV, r, z, st);
    }
    k_pcg_rz<<<g, b, 0, s>>>(nV, r, z, p, 1, st, part);
    k_pcg_rz_finish<<<1, b, 0, s>>>(part, 1, st);
    PcgState host{};
    const int chunk = 4;
    for (int it = 0; it < maxIters; it += chunk) {
        for (int k = 0; k < chunk && it + k < maxIters; ++k) {
            k_pcg_spmv<<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, p, ap, st, part);
            k_pcg_alpha<<<1, b, 0, s>>>(part, st);
            k_pcg_update_xr<<<g, b, 0, s>>>(nV, p, ap, d_x, r, st, part);
            k_pcg_check<<<1, b, 0, s>>>(part, st);
            if (precondition) {
                if ((rc = run_apply(h, z, r, s))) return rc;
            } else {
                k_pcg_copy<<<g, b, 0, s>>>(nV, r, z, st);
            }
            k_pcg_rz<<<g, b, 0, s>>>(nV, r, z, p, 0, st, part);
            k_pcg_rz_finish<<<1, b, 0, s>>>(part, 0, st);
            k_pcg_update_p<<<g, b, 0, s>>>(nV, z, p, st);
        }
        if ((rc = hip_check(h, hipMemcpyAsync(&host, st, sizeof(host), hipMemcpyDeviceToHost, s), "D2H pcg state")) ||
            (rc = hip_check(h, hipStreamSynchronize(s), "pcg sync")))
            return rc;
        if (host.done) break;
    }
    hipEventRecord(e1, s);
    // the true residual of the returned x (fp32 recursion drifts from it)
    k_pcg_init<<<g, b, 0, s>>>(nV, d_ranges, idx, d_diag9, d_off9, d_x, d_b, ap, part);
    k_pcg_true_finish<<<1, b, 0, s>>>(part, st);
    if ((rc = hip_check(h, hipMemcpyAsync(&host, st, sizeof(host), hipMemcpyDeviceToHost, s), "D2H pcg state")) ||
        (rc = hip_check(h, hipStreamSynchronize(s), "pcg sync")))
        return rc;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (res) {
        res->iterations = host.iters;
        res->converged = host.rr <= host.tol2 * host.bb;
        res->rel_residual = host.bb > 0 ? sqrt(host.rr / host.bb) : 0.0;
        res->true_rel_residual = host.bb > 0 ? sqrt(host.rrTrue / host.bb) : 0.0;
        res->solve_ms = ms;
    }
    return hip_check(h, hipGetLastError(), "pcg kernels");
}

}  // namespace mas
