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
    k_factor<<<h->nBlk, kFactorThreads, 0, s>>>(P<float>(h->dense), P<unsigned>(h->slotTable), P<float>(h->inv));
    return hip_check(h, hipGetLastError(), "factor kernel");
}

}  // namespace mas
