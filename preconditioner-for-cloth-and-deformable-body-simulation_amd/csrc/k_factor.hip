// k_factor.hip -- batched no-pivot LDL^T of the 96x96 subdomain blocks and the
// packed symmetric inverse (LDLtInverse512, .cpp:1347-1546).
//
// One workgroup (128 threads) per block; the block lives in LDS (96 x 100
// floats: 16-byte aligned rows, conflict-free ds_read_b128 across rows).
//   1. load + zero-diagonal -> identity (.cpp:1365-1368)
//   2. row-oriented elimination x = 0..95, rows skip a zero multiplier, the
//      row update runs over all 96 columns with FMA so the strict lower part
//      accumulates L^-1 (.cpp:1395-1415) -- thread y owns row y and updates it
//      with 24 float4 FMAs against the broadcast pivot row
//   3. D^-1 by IEEE division (.cpp:1429-1433)
//   4. Inv[i][j] = sum_{k = 95 .. j} fma(D^-1_k, L^-1[k][i] * L^-1[k][j], acc),
//      the reference's accumulation order (.cpp:1437-1495), written in the
//      node-pair layout of layout.h (coalesced stores)
// Operation for operation this is the reference arithmetic, so identical
// input blocks give bit-identical inverses.
#include <vector>

#include "layout.h"
#include "mas_internal.h"

namespace mas {

constexpr int kLda = 100;
constexpr int kFactorThreads = 128;

__global__ __launch_bounds__(kFactorThreads) void k_factor(const float* __restrict__ dense,
                                                          const unsigned* __restrict__ slotTable,
                                                          float* __restrict__ inv) {
    __shared__ __attribute__((aligned(16))) float A[96 * kLda];
    __shared__ float dinv[96];
    const int t = threadIdx.x;
    const size_t blk = blockIdx.x;
    const float4* src = reinterpret_cast<const float4*>(dense + blk * kDenseFloats);
    for (int q = t; q < kDenseFloats / 4; q += kFactorThreads) {
        const int row = q / 24, c4 = q % 24;
        *reinterpret_cast<float4*>(&A[row * kLda + 4 * c4]) = src[q];
    }
    __syncthreads();
    if (t < 32 && A[(3 * t) * kLda + 3 * t] == 0.0f) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) A[(3 * t + i) * kLda + 3 * t + j] = (i == j) ? 1.f : 0.f;
    }
    __syncthreads();
    for (int x = 0; x < 96; ++x) {
        if (t > x && t < 96) {
            const float a = A[t * kLda + x];
            if (a != 0.0f) {
                const float r = __fdiv_rn(-a, A[x * kLda + x]);
                float4* row = reinterpret_cast<float4*>(&A[t * kLda]);
                const float4* piv = reinterpret_cast<const float4*>(&A[x * kLda]);
#pragma unroll
                for (int c4 = 0; c4 < 24; ++c4) {
                    float4 p = piv[c4], y = row[c4];
                    y.x = __fmaf_rn(r, p.x, y.x);
                    y.y = __fmaf_rn(r, p.y, y.y);
                    y.z = __fmaf_rn(r, p.z, y.z);
                    y.w = __fmaf_rn(r, p.w, y.w);
                    row[c4] = y;
                }
                A[t * kLda + x] = r;
            }
        }
        __syncthreads();
    }
    if (t < 96) dinv[t] = __fdiv_rn(1.0f, A[t * kLda + t]);
    __syncthreads();
    float* out = inv + blk * kBlockFloats;
    for (int o = t; o < kBlockFloats; o += kFactorThreads) {
        const unsigned ij = slotTable[o];
        const int i = ij & 0xff, j = ij >> 8;
        float acc = 0.f;
        for (int k = 95; k >= j; --k) {
            const float mi = (k == i) ? 1.f : A[k * kLda + i];
            const float mj = (k == j) ? 1.f : A[k * kLda + j];
            acc = __fmaf_rn(dinv[k], __fmul_rn(mi, mj), acc);
        }
        out[o] = acc;
    }
}

// One elimination step with the step index x a compile-time constant, so the
// row stays in VGPRs (v[x] is a static register; a runtime x would demote the
// row to scratch).  Elim<0>::run expands all 96 steps.
template <int X>
__device__ __forceinline__ void elim_step(float (&v)[96], float (*piv)[96], float* dinv, bool has, int row) {
    float* pr = piv[X & 1];
    if (has && row == X) {  // the owner publishes its final row
#pragma unroll
        for (int c4 = 0; c4 < 24; ++c4)
            *reinterpret_cast<float4*>(&pr[4 * c4]) = make_float4(v[4 * c4], v[4 * c4 + 1], v[4 * c4 + 2], v[4 * c4 + 3]);
        dinv[X] = __fdiv_rn(1.0f, v[X]);
    }
    __syncthreads();
    if (has && row > X) {
        const float a = v[X];
        if (a != 0.0f) {
            const float r = __fdiv_rn(-a, pr[X]);
#pragma unroll
            for (int c4 = 0; c4 < 24; ++c4) {
                const float4 p = *reinterpret_cast<const float4*>(&pr[4 * c4]);
                v[4 * c4] = __fmaf_rn(r, p.x, v[4 * c4]);
                v[4 * c4 + 1] = __fmaf_rn(r, p.y, v[4 * c4 + 1]);
                v[4 * c4 + 2] = __fmaf_rn(r, p.z, v[4 * c4 + 2]);
                v[4 * c4 + 3] = __fmaf_rn(r, p.w, v[4 * c4 + 3]);
            }
            v[X] = r;
        }
    }
}

template <int X>
struct Elim {
    static __device__ __forceinline__ void run(float (&v)[96], float (*piv)[96], float* dinv, bool has, int row) {
        elim_step<X>(v, piv, dinv, has, row);
        Elim<X + 1>::run(v, piv, dinv, has, row);
    }
};
template <>
struct Elim<96> {
    static __device__ __forceinline__ void run(float (&)[96], float (*)[96], float*, bool, int) {}
};

// Register-resident variant (default).  Same operations on every element in
// the same order as k_factor above, rescheduled for CDNA4:
//   * thread -> row: wave 0 lanes own rows 32..63+32 (busy for all 95 steps),
//     wave 1 lanes 0..31 own rows 0..31 (busy only for steps < 32), so no
//     lane of wave 0 idles on a row that is already final;
//   * each row lives in 96 VGPRs for the whole elimination (the x loop is
//     fully unrolled, so v[x] is a static register); step x's owner publishes
//     its final row to a double-buffered LDS pivot row -> one barrier per step
//     and no LDS traffic for the row updates;
//   * D^-1 is computed by the pivot owner when it publishes;
//   * the inverse is formed in 4x4 tiles (i-block <= j-block) from the
//     eliminated matrix in LDS with unit diagonal: per k two ds_read_b128 and
//     16 (fmul, fma) pairs, k descending from 95 as in the reference; results
//     go to the free strict upper triangle of A (never read as L^-1) and
//     invDiag, then out through the slot table with coalesced stores.
__global__ __launch_bounds__(kFactorThreads) void k_factor_reg(const float* __restrict__ dense,
                                                              const unsigned* __restrict__ slotTable,
                                                              float* __restrict__ inv) {
    __shared__ __attribute__((aligned(16))) float A[96 * kLda];
    __shared__ __attribute__((aligned(16))) float piv[2][96];
    __shared__ float dinv[96];
    __shared__ float invDiag[96];
    const int t = threadIdx.x;
    const size_t blk = blockIdx.x;
    const float4* src = reinterpret_cast<const float4*>(dense + blk * kDenseFloats);
    for (int q = t; q < kDenseFloats / 4; q += kFactorThreads) {
        const int row = q / 24, c4 = q % 24;
        *reinterpret_cast<float4*>(&A[row * kLda + 4 * c4]) = src[q];
    }
    __syncthreads();
    if (t < 32 && A[(3 * t) * kLda + 3 * t] == 0.0f) {  // .cpp:1365-1368
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) A[(3 * t + i) * kLda + 3 * t + j] = (i == j) ? 1.f : 0.f;
    }
    __syncthreads();
    const bool has = t < 96;
    const int row = t < 64 ? 32 + t : t - 64;
    float v[96];
    if (has) {
#pragma unroll
        for (int c4 = 0; c4 < 24; ++c4) {
            const float4 q = *reinterpret_cast<const float4*>(&A[row * kLda + 4 * c4]);
            v[4 * c4] = q.x;
            v[4 * c4 + 1] = q.y;
            v[4 * c4 + 2] = q.z;
            v[4 * c4 + 3] = q.w;
        }
    }
    Elim<0>::run(v, piv, dinv, has, row);
    if (has) {
#pragma unroll
        for (int c4 = 0; c4 < 24; ++c4)
            *reinterpret_cast<float4*>(&A[row * kLda + 4 * c4]) =
                make_float4(v[4 * c4], v[4 * c4 + 1], v[4 * c4 + 2], v[4 * c4 + 3]);
    }
    __syncthreads();
    if (has) A[t * kLda + t] = 1.0f;  // M[k][k] = 1 (the reference's k == i / k == j cases)
    __syncthreads();
    // 300 tiles (I <= J) of 4x4 entries; Inv[i][j] = sum_{k = 95 .. j} fma(dinv_k, M[k][i] * M[k][j], acc)
    for (int tile = t; tile < 300; tile += kFactorThreads) {
        int J = 0, rem = tile;  // tile -> (I, J), J-major: J has J + 1 tiles
        while (rem > J) { rem -= J + 1; ++J; }
        const int I = rem;
        float acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
        int k = 95;
        for (; k >= 4 * J + 3; --k) {
            const float4 mi = *reinterpret_cast<const float4*>(&A[k * kLda + 4 * I]);
            const float4 mj = *reinterpret_cast<const float4*>(&A[k * kLda + 4 * J]);
            const float d = dinv[k];
            const float fi[4] = {mi.x, mi.y, mi.z, mi.w}, fj[4] = {mj.x, mj.y, mj.z, mj.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = __fmaf_rn(d, __fmul_rn(fi[a], fj[b]), acc[a][b]);
        }
#pragma unroll
        for (int kk = 2; kk >= 0; --kk) {  // k = 4J + kk: only entries with j = 4J + b <= k
            k = 4 * J + kk;
            const float4 mi = *reinterpret_cast<const float4*>(&A[k * kLda + 4 * I]);
            const float4 mj = *reinterpret_cast<const float4*>(&A[k * kLda + 4 * J]);
            const float d = dinv[k];
            const float fi[4] = {mi.x, mi.y, mi.z, mi.w}, fj[4] = {mj.x, mj.y, mj.z, mj.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b <= kk; ++b) acc[a][b] = __fmaf_rn(d, __fmul_rn(fi[a], fj[b]), acc[a][b]);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int i = 4 * I + a, j = 4 * J + b;
                if (i < j) A[i * kLda + j] = acc[a][b];
                else if (i == j) invDiag[i] = acc[a][b];
            }
    }
    __syncthreads();
    float* out = inv + blk * kBlockFloats;
    for (int o = t; o < kBlockFloats; o += kFactorThreads) {
        const unsigned ij = slotTable[o];
        const int i = ij & 0xff, j = ij >> 8;
        out[o] = (i == j) ? invDiag[i] : A[i * kLda + j];
    }
}

int upload_slot_table(mas_context* h) {
    std::vector<unsigned> tab(kBlockFloats);
    for (int o = 0; o < kBlockFloats; ++o) {
        int i, j;
        slot_ij(o, i, j);
        tab[o] = (unsigned)i | ((unsigned)j << 8);
    }
    int rc = ensure(h, h->slotTable, tab.size() * 4);
    if (rc) return rc;
    return hip_check(h, hipMemcpy(h->slotTable.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice), "H2D slots");
}

int copy_block_inverse(mas_context* h, int blk, float* out96) {
    std::vector<float> packed(kBlockFloats);
    int rc = hip_check(h,
                       hipMemcpy(packed.data(), P<float>(h->inv) + (size_t)blk * kBlockFloats, kBlockFloats * 4,
                                 hipMemcpyDeviceToHost),
                       "D2H inverse");
    if (rc) return rc;
    for (int o = 0; o < kBlockFloats; ++o) {
        int i, j;
        slot_ij(o, i, j);
        out96[i * 96 + j] = packed[o];
        out96[j * 96 + i] = packed[o];
    }
    return MAS_OK;
}

int run_factor(mas_context* h, hipStream_t s) {
    int rc = ensure(h, h->inv, (size_t)h->nBlk * kBlockFloats * 4);
    if (rc) return rc;
    if (h->factorVariant == 0)
        k_factor<<<h->nBlk, kFactorThreads, 0, s>>>(P<float>(h->dense), P<unsigned>(h->slotTable), P<float>(h->inv));
    else
        k_factor_reg<<<h->nBlk, kFactorThreads, 0, s>>>(P<float>(h->dense), P<unsigned>(h->slotTable),
                                                         P<float>(h->inv));
    return hip_check(h, hipGetLastError(), "factor kernel");
}

}  // namespace mas
