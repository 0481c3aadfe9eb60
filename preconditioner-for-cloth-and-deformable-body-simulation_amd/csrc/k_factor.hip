// k_factor.hip -- batched no-pivot LDL^T of the 96x96 subdomain blocks and the
// packed symmetric inverse (LDLtInverse512, .cpp:1347-1546).
//
// The reference arithmetic, per block:
//   1. zero-diagonal node -> identity 3x3 (.cpp:1365-1368)
//   2. row-oriented elimination x = 0..95, rows skip a zero multiplier, the
//      row update runs over all 96 columns with FMA so the strict lower part
//      accumulates L^-1 (.cpp:1395-1415)
//   3. D^-1 by IEEE division (.cpp:1429-1433)
//   4. Inv[i][j] = sum_{k = 95 .. j} fma(D^-1_k, L^-1[k][i] * L^-1[k][j], acc),
//      the reference's accumulation order (.cpp:1437-1495), stored in the
//      node-pair layout of layout.h
// Two kernels perform exactly these operations on every element in this
// order, so identical input blocks give bit-identical inverses:
//   k_factor     one 128-thread workgroup per block, block in LDS, thread y
//                owns row y (MAS_FACTOR_VARIANT=0; LDS-bandwidth bound:
//                every FMA reads its pivot value from LDS) -- 15.0 ms at 1M
//   k_factor_rb  (default) one wave per block, rows in VGPRs in 6x24 lane
//                tiles, the pivot row broadcast through LDS, multipliers and
//                quotients through DPP, inverse staged in LDS and stored
//                coalesced -- 1.63 ms at 1M (profiles/round1/ab);
//                MAS_FACTOR_VARIANT=3 forms the inverse on the matrix cores
//                instead (form_mfma, not bitwise, 1.47 ms)
#include <vector>

#include "layout.h"
#include "mas_internal.h"

namespace mas {

constexpr int kLda = 100;
constexpr int kFactorThreads = 128;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
static_assert(kDenseFloats / 4 % kFactorThreads == 0, "factor load tiling");

// Failure detection (the reference divides by every pivot unchecked,
// .cpp:1406,1431): a block whose D^-1 holds a zero, negative or non-finite
// entry -- a zero / negative / non-finite pivot, or one so small that its
// reciprocal overflows -- is counted in status[0] and the lowest such block
// kept in status[1] (MAS_ERR_NOT_SPD after Prepare).  One wave, lanes 0..63
// read D^-1 entries lane and 64 + lane; the inverses are unchanged.
__device__ __forceinline__ void check_pivots(const float* dinv, int* status, int blk, int lane) {
    const float d0 = dinv[lane], d1 = lane < 32 ? dinv[64 + lane] : 1.f;
    const bool bad = !(d0 > 0.f && d0 <= 3.402823466e38f) || !(d1 > 0.f && d1 <= 3.402823466e38f);
    if (__ballot(bad) && lane == 0) {
        atomicAdd(status, 1);
        atomicMin(status + 1, blk);
    }
}

__global__ __launch_bounds__(kFactorThreads) void k_factor(const float* __restrict__ dense,
                                                          const unsigned* __restrict__ slotTable,
                                                          float* __restrict__ inv, int blk0, int* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) float A[96 * kLda];
    __shared__ float dinv[96];
    const int t = threadIdx.x;
    const size_t blk = (size_t)blk0 + blockIdx.x;
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
    if (status && t < 64) check_pivots(dinv, status, (int)blk, t);
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

template <int SEL>
__device__ __forceinline__ float quad_bcast_c(float x) {
    constexpr int ctrl = SEL | (SEL << 2) | (SEL << 4) | (SEL << 6);  // quad_perm [SEL, SEL, SEL, SEL]
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), ctrl, 0xf, 0xf, false));
}
// sel is a constant after unrolling; the switch folds away
__device__ __forceinline__ float quad_bcast(float x, int sel) {
    switch (sel & 3) {
        case 0: return quad_bcast_c<0>(x);
        case 1: return quad_bcast_c<1>(x);
        case 2: return quad_bcast_c<2>(x);
        default: return quad_bcast_c<3>(x);
    }
}

template <int X>
__device__ __forceinline__ void rb_step(float (&v)[6][24], float* piv, float (&dv)[2], int rg, int cg) {
    constexpr int mX = X / 16, rX = X % 16, cgX = X / 24, cX = X % 24;
    constexpr int mLo = (X < 15) ? 0 : (X - 15) / 16 + 1;
    float* pr = piv;  // one buffer: a single wave's LDS operations complete in order
    // The pivot straight from its owner lane (lane 4 rX + cgX holds A[X][X] in
    // v[mX][cX]; the same value the pivot row carries through LDS), so the
    // step's three IEEE divisions -- D^-1_X and the quotients of two rows per
    // lane -- start at once, unconditionally and side by side, while the
    // pivot row makes its LDS round trip.  (Read from LDS after the row's
    // store, each division in the branch of its lanes, they ran one after the
    // other behind that round trip.)
    const float pd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[mX][cX]), 4 * rX + cgX));
    if (rg == rX) {
#pragma unroll
        for (int c4 = 0; c4 < 6; ++c4)
            *reinterpret_cast<float4*>(&pr[24 * cg + 4 * c4]) =
                make_float4(v[mX][4 * c4], v[mX][4 * c4 + 1], v[mX][4 * c4 + 2], v[mX][4 * c4 + 3]);
    }
    // the pivot is final from this step on: D^-1_X (.cpp:1429-1433) is taken
    // here; lane X % 64 keeps it (dv[X / 64], a select, no branch) and stores
    // it after the elimination
    if constexpr (mLo > 5) {
        const float d = __fdiv_rn(1.0f, pd);
        dv[X / 64] = (4 * rg + cg == X % 64) ? d : dv[X / 64];
    }
    if constexpr (mLo <= 5) {
        float a[6], r[6];
#pragma unroll
        for (int m = mLo; m < 6; ++m) a[m] = quad_bcast(v[m][cX], cgX);
        // lane cg divides for rows m = mLo + cg and mLo + 4 + cg
        float q0 = 0.f, q1 = 0.f;
        {
            const int m0 = mLo + cg, m1 = mLo + 4 + cg;
            float a0 = 0.f, a1 = 0.f;
#pragma unroll
            for (int m = mLo; m < 6; ++m) {
                a0 = (m == m0) ? a[m] : a0;
                a1 = (m == m1) ? a[m] : a1;
            }
            const bool act0 = m0 < 6 && rg + 16 * m0 > X && a0 != 0.0f;
            const bool act1 = m1 < 6 && rg + 16 * m1 > X && a1 != 0.0f;
            // (a shared-reciprocal division without the scale / fixup steps,
            // exact for operands in [2^-40, 2^40], measured 11 % slower)
            // every lane divides twice, then selects.  A cg == 3 lane never owns
            // row group m1 = mLo + 7 > 5, so its second division is -1 / pd
            // instead, and D^-1_X = -(-1 / pd) (IEEE division is symmetric in
            // sign): two division sequences per step instead of three
            const float d0 = __fdiv_rn(-a0, pd), d1 = __fdiv_rn(cg == 3 ? -1.0f : -a1, pd);
            q0 = act0 ? d0 : 0.f;
            q1 = act1 ? d1 : 0.f;
            const float d = -__int_as_float(__builtin_amdgcn_readlane(__float_as_int(d1), 3));
            dv[X / 64] = (4 * rg + cg == X % 64) ? d : dv[X / 64];
        }
#pragma unroll
        for (int m = mLo; m < 6; ++m) r[m] = quad_bcast((m - mLo) < 4 ? q0 : q1, (m - mLo) & 3);
        // the pivot row's LDS store before its loads below
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // the pivot row in two halves of 12 (register budget: 2 waves per SIMD)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            float p[12];
#pragma unroll
            for (int c4 = 0; c4 < 3; ++c4) {
                const float4 q = *reinterpret_cast<const float4*>(&pr[24 * cg + 12 * hh + 4 * c4]);
                p[4 * c4] = q.x;
                p[4 * c4 + 1] = q.y;
                p[4 * c4 + 2] = q.z;
                p[4 * c4 + 3] = q.w;
            }
#pragma unroll
            for (int m = mLo; m < 6; ++m)
#pragma unroll
                for (int c = 0; c < 12; ++c) v[m][12 * hh + c] = __fmaf_rn(r[m], p[c], v[m][12 * hh + c]);
            if (hh == 0) {  // keep the second half's loads behind the first half's updates
#pragma unroll
                for (int m = mLo; m < 6; ++m)
#pragma unroll
                    for (int c = 0; c < 12; c += 2) {
                        v2f q = {v[m][c], v[m][c + 1]};
                        asm volatile("" : "+v"(q)::"memory");
                        v[m][c] = q.x;
                        v[m][c + 1] = q.y;
                    }
            }
        }
#pragma unroll
        for (int m = mLo; m < 6; ++m) {
            // A[row][X] = r where the reference ran the update (row > X, a != 0)
            const bool upd = (cg == cgX) && (rg + 16 * m > X) && (a[m] != 0.0f);
            v[m][cX] = upd ? r[m] : v[m][cX];
        }
    }
    // Pin the step's results here: otherwise LLVM sinks the updates of rows
    // not needed by the next pivot into later steps and every step's pivot
    // row stays live (hundreds of VGPRs, then scratch).
#pragma unroll
    for (int m = mLo; m < 6; ++m)
#pragma unroll
        for (int c = 0; c < 24; c += 2) {  // as register pairs, so the updates stay v_pk_fma_f32
            v2f q = {v[m][c], v[m][c + 1]};
            asm volatile("" : "+v"(q));
            v[m][c] = q.x;
            v[m][c + 1] = q.y;
        }
}

template <int X>
struct ElimRB {
    static __device__ __forceinline__ void run(float (&v)[6][24], float* piv, float (&dv)[2], int rg, int cg) {
        rb_step<X>(v, piv, dv, rg, cg);
        ElimRB<X + 1>::run(v, piv, dv, rg, cg);
    }
};
template <>
struct ElimRB<96> {
    static __device__ __forceinline__ void run(float (&)[6][24], float*, float (&)[2], int, int) {}
};

// Zero diagonal -> identity node block (.cpp:1365-1368), applied in place to
// the assembled blocks before the register-resident factor kernels (which
// never see the whole block in one place).  mas_get_block_matrix reports the
// same rule, so the stored blocks read back unchanged.
__global__ __launch_bounds__(256) void k_identity_fix(float* __restrict__ dense, int node0, int node1) {
    const int node = node0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (node >= node1) return;
    float* d = dense + (size_t)(node >> 5) * kDenseFloats + (3 * (node & 31)) * 96 + 3 * (node & 31);
    if (*d != 0.0f) return;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) d[i * 96 + j] = (i == j) ? 1.f : 0.f;
}

// Packed lower-triangular M in LDS: row k holds columns [0, ceil4(k+1)), so the
// formation's float4 reads stay aligned; 4 800 floats = 19.2 KB.
__device__ __forceinline__ int m_row(int k) {
    const int g = k >> 2;
    return 8 * g * (g + 1) + (k & 3) * 4 * (g + 1);
}
constexpr int kPackedM = 4800;

// Inv entries from the packed M (unit diagonal) in 4x4 tiles (I <= J), k
// descending from 95 with (fmul, fma) as the reference.  One wave: each lane
// keeps its <= 5 tiles (tile = lane + 64 t) in registers, then M's LDS is
// reused to assemble the packed inverse (slots from the host-built table
// valuSlot: 16 ushorts per tile, 0xFFFF below the diagonal), which leaves as
// 1 KiB coalesced stores: the scattered 4-byte slot stores this replaced made
// the formation ~0.9 ms of a 1.96 ms factor at 1M (now 1.63 ms, bitwise equal).
__device__ __forceinline__ void form_packed_staged(float* M, const float* dinv, float* out,
                                                   const uint4* __restrict__ valuSlot, int lane) {
    float acc[5][4][4];
#pragma unroll
    for (int tt = 0; tt < 5; ++tt) {
        const int tile = lane + 64 * tt;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[tt][a][b] = 0.f;
        if (tile >= 300) continue;
        int J = 0, rem = tile;
        while (rem > J) { rem -= J + 1; ++J; }
        const int I = rem;
        for (int k = 95; k >= 4 * J + 3; --k) {
            const int base = m_row(k);
            const float4 mi = *reinterpret_cast<const float4*>(&M[base + 4 * I]);
            const float4 mj = *reinterpret_cast<const float4*>(&M[base + 4 * J]);
            const float d = dinv[k];
            const float fi[4] = {mi.x, mi.y, mi.z, mi.w}, fj[4] = {mj.x, mj.y, mj.z, mj.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[tt][a][b] = __fmaf_rn(d, __fmul_rn(fi[a], fj[b]), acc[tt][a][b]);
        }
#pragma unroll
        for (int kk = 2; kk >= 0; --kk) {
            const int k = 4 * J + kk, base = m_row(k);
            const float4 mi = *reinterpret_cast<const float4*>(&M[base + 4 * I]);
            const float4 mj = *reinterpret_cast<const float4*>(&M[base + 4 * J]);
            const float d = dinv[k];
            const float fi[4] = {mi.x, mi.y, mi.z, mi.w}, fj[4] = {mj.x, mj.y, mj.z, mj.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b <= kk; ++b) acc[tt][a][b] = __fmaf_rn(d, __fmul_rn(fi[a], fj[b]), acc[tt][a][b]);
        }
    }
    uint4 sl[10];
#pragma unroll
    for (int tt = 0; tt < 5; ++tt) {
        const int tile = lane + 64 * tt < 300 ? lane + 64 * tt : 0;
        sl[2 * tt] = valuSlot[2 * tile];
        sl[2 * tt + 1] = valuSlot[2 * tile + 1];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every M read done before M is overwritten
    __builtin_amdgcn_wave_barrier();
    float* O = M;
#pragma unroll
    for (int tt = 0; tt < 5; ++tt) {
        if (lane + 64 * tt >= 300) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const uint4 w = sl[2 * tt + (e >> 3)];
            const int h = (e & 7) >> 1;
            const unsigned word = h == 0 ? w.x : h == 1 ? w.y : h == 2 ? w.z : w.w;
            const unsigned slot = (e & 1) ? word >> 16 : word & 0xFFFFu;
            if (slot != 0xFFFFu) O[slot] = acc[tt][e >> 2][e & 3];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const float4* O4 = reinterpret_cast<const float4*>(O);
    float4* out4 = reinterpret_cast<float4*>(out);
    for (int q = lane; q < kBlockF4; q += 64) out4[q] = O4[q];
}

// Inv = M^T D M on the matrix cores (MAS_FACTOR_VARIANT=3): M = L^-1 (unit
// lower triangular, packed in LDS), D = diag(D^-1).  Six 32x32 output tiles
// (I <= J) of v_mfma_f32_32x32x2_f32: A = M[k..k+1][32I..32I+31]^T,
// B = D^-1_k M[k..k+1][32J..32J+31]; rows k < 32 J are zero in B and skipped,
// k runs downwards as in the reference's sum.  160 MFMAs per block replace
// ~2.6k VALU instructions and ~20k LDS reads of form_packed_staged.  An f32 MFMA is an
// exact fmaf chain, but of M_ik * fl(D^-1_k M_jk) where the reference rounds
// fl(M_ik M_jk) first: inverses agree within 4.6e-8 relative
// (tests/test_gpu_factor_mfma.py), not bitwise; 1.96 -> 1.47 ms at 1M.
typedef float v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ float m_at(const float* M, int k, int i) {
    return i < k ? M[m_row(k) + i] : (i == k ? 1.f : 0.f);
}
// Tile (I, J), fully unrolled and branch-free: row k of M starts at the
// uniform m_row(k) (a select between the two rows of a k pair by the lane's
// half), columns past k read the row's stored unit diagonal (clamped address)
// and are zeroed by a select -- the same operands as m_at, so the same bits.
// (The first form evaluated m_at per operand with branches and a runtime k
// loop: ~30 instructions and an LDS wait per MFMA, 0.57 ms of the 2.10 ms
// fused kernel at 1M + contacts.)
template <int I, int J>
__device__ __forceinline__ v16f mfma_tile(const float* M, const float* dinv, int col, int kh) {
    v16f acc = {};
    const int ci = 32 * I + col, cj = 32 * J + col;
#pragma unroll
    for (int k0 = 94; k0 >= 32 * J; k0 -= 2) {
        const int k = k0 + 1 - kh;  // the instruction is the fmaf chain k-half 0 then 1: strictly k-descending
        const int rb = kh ? m_row(k0) : m_row(k0 + 1);
        float a;
        if constexpr (I < J) {
            a = M[rb + ci];  // ci < 32 J <= k: strictly below the diagonal
        } else {
            a = M[rb + min(ci, k)];
            a = ci <= k ? a : 0.f;
        }
        float m = M[rb + min(cj, k)];
        m = cj <= k ? m : 0.f;
        const float b = __fmul_rn(dinv[k], m);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    return acc;
}
// All six tiles are accumulated first (96 accumulator registers: the
// elimination's 144 tile registers are dead by now), then M's LDS is reused to
// stage the packed inverse, which leaves as 1 KiB coalesced stores (with
// scattered slot stores the MFMA formation saved only 4 %).
// tileSlot: for tile t, accumulator register r and lane l, the packed slot of
// the entry that register holds (0xFFFF: below the diagonal), 8 ushorts per
// uint4 at [(2 t + r / 8) * 64 + l] -- 12 coalesced loads per lane instead of
// 96 evaluations of slot_of (built on the host by upload_slot_table).
__device__ __forceinline__ void form_mfma(float* M, const float* dinv, float* out, const uint4* __restrict__ tileSlot,
                                          int lane) {
    const int col = lane & 31, kh = lane >> 5;
    uint4 sl[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) sl[q] = tileSlot[q * 64 + lane];
    v16f acc[6];
    acc[0] = mfma_tile<0, 0>(M, dinv, col, kh);
    acc[1] = mfma_tile<0, 1>(M, dinv, col, kh);
    acc[2] = mfma_tile<1, 1>(M, dinv, col, kh);
    acc[3] = mfma_tile<0, 2>(M, dinv, col, kh);
    acc[4] = mfma_tile<1, 2>(M, dinv, col, kh);
    acc[5] = mfma_tile<2, 2>(M, dinv, col, kh);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every M read done before M is overwritten
    __builtin_amdgcn_wave_barrier();
    float* O = M;  // 4 656 <= kPackedM floats
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint4 w = sl[2 * t + (r >> 3)];
            const int h = (r & 7) >> 1;
            const unsigned word = h == 0 ? w.x : h == 1 ? w.y : h == 2 ? w.z : w.w;
            const unsigned slot = (r & 1) ? word >> 16 : word & 0xFFFFu;
            if (slot != 0xFFFFu) O[slot] = acc[t][r];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const float4* O4 = reinterpret_cast<const float4*>(O);
    float4* out4 = reinterpret_cast<float4*>(out);
    for (int q = lane; q < kBlockF4; q += 64) out4[q] = O4[q];
}

// The block in the lane tiles v (lane t: rows t / 4 + 16 m, columns
// 24 (t % 4) .. + 23) -> elimination, M, the packed inverse at out.
template <bool MFMA>
__device__ __forceinline__ void factor_tiles(float (&v)[6][24], float* M, float* piv, float* dinv, float* out,
                                             const uint4* __restrict__ tileSlot, const uint4* __restrict__ valuSlot,
                                             int t, int* status, int blk) {
    const int rg = t >> 2, cg = t & 3;
    float dv[2] = {0.f, 0.f};  // D^-1 of steps t and 64 + t
#ifndef MAS_TIMING_NO_ELIM  // timing probe only (A/B build): the kernel without its elimination
    ElimRB<0>::run(v, piv, dv, rg, cg);
#else
    dv[0] = dv[1] = 1.f;
#endif
    dinv[t] = dv[0];
    if (t < 32) dinv[64 + t] = dv[1];
    // M rows: unit diagonal, L^-1 below, only the stored (padded) columns
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const int k = rg + 16 * m, len = (k & ~3) + 4;
#pragma unroll
        for (int c4 = 0; c4 < 6; ++c4) {
            const int col = 24 * cg + 4 * c4;
            if (col < len) {
                float4 q = make_float4(v[m][4 * c4], v[m][4 * c4 + 1], v[m][4 * c4 + 2], v[m][4 * c4 + 3]);
                if (col == (k & ~3)) {  // the diagonal lies in this float4
                    const int d = k & 3;
                    q.x = d == 0 ? 1.f : q.x;
                    q.y = d == 1 ? 1.f : q.y;
                    q.z = d == 2 ? 1.f : q.z;
                    q.w = d == 3 ? 1.f : q.w;
                }
                *reinterpret_cast<float4*>(&M[m_row(k) + col]) = q;
            }
        }
    }
    __syncthreads();
    if (status) check_pivots(dinv, status, blk, t);
#ifdef MAS_TIMING_NO_FORM  // timing probe only (A/B build): no inverse formation
    if (t == 0) out[0] = M[0] + dinv[0];
    return;
#endif
    if (MFMA) form_mfma(M, dinv, out, tileSlot, t);  // one wave: no barrier around M
    else form_packed_staged(M, dinv, out, valuSlot, t);
}

// Register-blocked factor: LDS holds only the pivot row, D^-1 and the packed
// M (~19.5 KB -> 8 blocks per CU at <= 256 VGPRs), the block is loaded from
// HBM straight into the lane tiles, and M's LDS is reused to stage the packed
// inverse once M is consumed.
template <bool MFMA>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_factor_rb(
    const float* __restrict__ dense, float* __restrict__ inv, const uint4* __restrict__ tileSlot,
    const uint4* __restrict__ valuSlot, int blk0, int* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) float M[kPackedM];
    __shared__ __attribute__((aligned(16))) float piv[96];
    __shared__ float dinv[96];
    const int t = threadIdx.x;
    const size_t blk = (size_t)blk0 + blockIdx.x;
    const int rg = t >> 2, cg = t & 3;
    float v[6][24];
    {
        const float* src = dense + blk * kDenseFloats + 24 * cg;
#pragma unroll
        for (int m = 0; m < 6; ++m)
#pragma unroll
            for (int c4 = 0; c4 < 6; ++c4) {
                const v4f q = __builtin_nontemporal_load(
                    reinterpret_cast<const v4f*>(src + (size_t)(rg + 16 * m) * 96 + 4 * c4));
                v[m][4 * c4] = q.x;
                v[m][4 * c4 + 1] = q.y;
                v[m][4 * c4 + 2] = q.z;
                v[m][4 * c4 + 3] = q.w;
            }
    }
    factor_tiles<MFMA>(v, M, piv, dinv, inv + blk * kBlockFloats, tileSlot, valuSlot, t, status, (int)blk);
}

// ---------------------------------------------------------------------------
// Fused level-0 assemble + factor (the default, MAS_FACTOR_VARIANT=4)
// ---------------------------------------------------------------------------
//
// One wave per level-0 block builds the block in two LDS slabs of 16 nodes
// (48 rows x 96 columns, 18 KB, aliased with the factor's packed M, so LDS
// stays ~20 KB and two waves per SIMD still fit), moves each slab into the
// factor's lane tiles and factors as k_factor_rb.  The assembled block never
// reaches HBM: 2 x 36 KB of traffic per block less than k_level0_block +
// k_factor_rb (2.4 GB at 1M), and the assembly's load latency hides behind the
// other wave's elimination.  Per entry the sums are the reference's: the
// block's contact entries first (one prefolded run sum per entry, added to
// zero), then the CSR terms in ELL order -- the diagonal node's
// diag + additional (.cpp:1270-1271), each same-bank neighbour's off-diagonal
// (.cpp:1275-1282) -- then the zero-diagonal identity rule (.cpp:1365-1368).
// Bitwise equal to k_level0_block + k_identity_fix + k_factor_rb.
template <int H>
__device__ __forceinline__ void build_slab(const FineAsm& a, int blk, float* S, int lane) {
    float4* S4 = reinterpret_cast<float4*>(S);
    for (int q = lane; q < 48 * 96 / 4; q += 64) S4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (a.coff) {
        // the block's contact records, 16 at a time staged past the slab in
        // M's LDS (entry code + 9 values each); lane q < 9 adds component q
        // (column-major: row q % 3, column q / 3) of every record in order, so
        // each entry gets its records in stencil order, added to the zero
        // entry before the CSR terms (.cpp:88-97)
        float* stg = S + 48 * 96;
        const int q = lane < 9 ? lane : 0, qr = q % 3, qc = q / 3;
        const int j0 = a.coff[blk], j1 = a.coff[blk + 1];
        for (int jb = j0; jb < j1; jb += 16) {
            const int cnt = min(16, j1 - jb);
            if (lane < cnt) {
                const int id = a.cids[jb + lane];
                stg[10 * lane] = __int_as_float(a.cent[id]);
                const float* src = a.cvals + 9 * (size_t)id;
#pragma unroll
                for (int e = 0; e < 9; ++e) stg[10 * lane + 1 + e] = src[e];
            }
            __syncthreads();
            if (lane < 9)
                for (int k = 0; k < cnt; ++k) {
                    const int ent = __float_as_int(stg[10 * k]);
                    const int nl = (ent >> 5) - 16 * H, col = ent & 31;
                    if (nl >= 0 && nl < 16) {
                        float* p = S + (3 * nl + qr) * 96 + 3 * col + qc;
                        *p = __fadd_rn(*p, stg[10 * k + 1 + q]);
                    }
                }
            __syncthreads();
        }
    }
    // CSR terms: lane = (node n = lane % 16, slot group g = lane / 16), ELL slot
    // k = k0 + g + 4 p; a pass loads 4 slots per lane, then adds them in slot order
    const int n = lane & 15, g = lane >> 4;
    const int v = 32 * blk + 16 * H + n;
    const bool live = v < a.nV;
    int o = 0, num = 0, base = 0;
    if (live) {
        o = a.s2o[v];
        num = a.nbrNum[v];
        base = a.ranges[o];
    }
    // Column masks per node (past the staging area): a slab whose slots never
    // name one (node, column) entry twice -- no duplicate neighbour, no self
    // loop, the usual case -- gives every entry at most one CSR term, so all
    // slots' adds can go at once; otherwise they go in slot order (below).
    unsigned* colMask = reinterpret_cast<unsigned*>(S + 48 * 96 + 16 * 10);
    if (lane < 16) colMask[lane] = 0u;
    __syncthreads();
    for (int k0 = 0; k0 < a.maxNbr; k0 += 16) {
        float m[4][9];
        int col[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int k = k0 + g + 4 * p;
            col[p] = -1;
            if (!live || k >= num) continue;
            if (k == 0) {  // diag (column-major) + additional (row-major), .cpp:1270
                const float* d = a.diag9 + 9 * (size_t)o;
                const float* ad = a.additional + 9 * (size_t)v;
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) m[p][r * 3 + c] = __fadd_rn(d[c * 3 + r], ad[r * 3 + c]);
                col[p] = 16 * H + n;
            } else {
                const unsigned ot = (unsigned)a.nbr[(size_t)k * a.nV + v];
                if ((ot >> 5) != ((unsigned)v >> 5)) continue;  // cross-bank: a coarse record
                const float* src = a.off9 + 9 * ((size_t)base + k - 1);
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) m[p][r * 3 + c] = src[c * 3 + r];
                col[p] = (int)(ot & 31);
            }
        }
        bool dup = false;
#pragma unroll
        for (int p = 0; p < 4; ++p)
            if (col[p] >= 0) dup |= (atomicOr(&colMask[n], 1u << col[p]) >> col[p]) & 1u;
        if (!__ballot(dup)) {  // every entry of this pass gets one term: all adds at once
#pragma unroll
            for (int p = 0; p < 4; ++p)
                if (col[p] >= 0) {
                    float* e = S + (3 * n) * 96 + 3 * col[p];
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c) e[r * 96 + c] = __fadd_rn(e[r * 96 + c], m[p][r * 3 + c]);
                }
        } else {
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int gg = 0; gg < 4; ++gg)  // slot order within the vertex (duplicate neighbours add in ELL order)
                    if (g == gg && col[p] >= 0) {
                        float* e = S + (3 * n) * 96 + 3 * col[p];
#pragma unroll
                        for (int r = 0; r < 3; ++r)
#pragma unroll
                            for (int c = 0; c < 3; ++c) e[r * 96 + c] = __fadd_rn(e[r * 96 + c], m[p][r * 3 + c]);
                    }
        }
    }
    __syncthreads();
    if (lane < 16) {  // zero diagonal -> identity node block (.cpp:1365-1368)
        float* e = S + (3 * lane) * 96 + 3 * (16 * H + lane);
        if (*e == 0.0f)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) e[r * 96 + c] = (r == c) ? 1.f : 0.f;
    }
    __syncthreads();
    if (a.keep) {
        float4* dst = reinterpret_cast<float4*>(a.keep + (size_t)blk * kDenseFloats + 48 * 96 * H);
        for (int q = lane; q < 48 * 96 / 4; q += 64) dst[q] = S4[q];
    }
}

template <int H>
__device__ __forceinline__ void slab_to_tiles(float (&v)[6][24], const float* S, int lane) {
    const int rg = lane >> 2, cg = lane & 3;
#pragma unroll
    for (int mm = 0; mm < 3; ++mm)
#pragma unroll
        for (int c4 = 0; c4 < 6; ++c4) {
            const float4 q = *reinterpret_cast<const float4*>(&S[(rg + 16 * mm) * 96 + 24 * cg + 4 * c4]);
            v[3 * H + mm][4 * c4] = q.x;
            v[3 * H + mm][4 * c4 + 1] = q.y;
            v[3 * H + mm][4 * c4 + 2] = q.z;
            v[3 * H + mm][4 * c4 + 3] = q.w;
        }
}

template <bool MFMA>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_factor_fused(
    FineAsm a, float* __restrict__ inv, const uint4* __restrict__ tileSlot, const uint4* __restrict__ valuSlot,
    int blk0, int* __restrict__ status) {
    static_assert(48 * 96 + 16 * 10 + 16 <= kPackedM, "a slab, 16 staged contact records and 16 column masks fit in M's LDS");
    __shared__ __attribute__((aligned(16))) float M[kPackedM];
    __shared__ __attribute__((aligned(16))) float piv[96];
    __shared__ float dinv[96];
    const int t = threadIdx.x;
    const int blk = blk0 + blockIdx.x;
    float v[6][24];
#ifndef MAS_TIMING_NO_ASM  // timing probe only (A/B build): the kernel without its assembly
    build_slab<0>(a, blk, M, t);
    slab_to_tiles<0>(v, M, t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab 0 read before slab 1 overwrites it
    __syncthreads();
    build_slab<1>(a, blk, M, t);
    slab_to_tiles<1>(v, M, t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#else
    for (int m = 0; m < 6; ++m)
        for (int c = 0; c < 24; ++c) v[m][c] = (t >> 2) + 16 * m == 24 * (t & 3) + c ? 2.f : 0.01f * (float)(c + m);
#endif
    factor_tiles<MFMA>(v, M, piv, dinv, inv + (size_t)blk * kBlockFloats, tileSlot, valuSlot, t, status, blk);
}

// (A two-wave-per-block form of this kernel -- wave w holding the row groups
// m = w, w + 2, w + 4, the pivot row through a double-buffered LDS row and one
// workgroup barrier per step -- was bitwise equal but slower, 2.18 -> 2.75 ms
// at 1M + contacts: LDS and VGPRs already allow 8 blocks per CU either way,
// so it only added a barrier to every step; profiles/round5/ab/.)
int launch_factor_fused(mas_context* h, const FineAsm& a, int blk0, int blk1, hipStream_t s) {
    // The blocks in C launches in a row (round 6): between two of them the
    // queue waits for the earlier one to drain, and the coarse assembly's
    // kernels on the caller's queue take the slots it frees -- what the
    // CU-masked queue did before (mas_internal.h prepCuReserve).  Measured
    // (steady-state Prepare, device Hessian, ms, profiles/round6/prepare/):
    // 1M + contacts C = 1 / 2 / 4 / 8 / 12 / 16 -> 2.75 / 2.77 / 2.79 / 2.56 /
    // 2.70 / 2.75 (32-CU mask 2.45); 4M tet 1 / 4 / 8 / 16 -> 8.88 / 8.33 /
    // 8.30 / 8.55 (mask 8.58); 256k 1 / 2 / 4 / 8 -> 0.589 / 0.579 / 0.570 /
    // 0.699; a world-8 rank of 1M 1 / 2 / 4 / 8 -> 1.03 / 1.03 / 0.98 / 1.09.
    // With od in the early path (early_od: unsharded 2 048 .. 32 768 blocks),
    // fewer launches do better: 1M + contacts 4 / 6 / 8 -> 2.450 / 2.518 /
    // 2.569 ms, 256k 2 / 4 -> 0.547 / 0.591 (profiles/round6/prepare/r6y, r6z).
    // Env MAS_FUSED_CHUNKS overrides.
    const int nb = blk1 - blk0;
    int chunks = nb < 2048 ? 1 : nb <= 16384 ? 4 : 8;
    if (h->prepWorld == 1 && nb >= 2048 && nb <= 32768) chunks = nb <= 8192 ? 2 : 4;
    if (h->fusedChunks > 0) chunks = h->fusedChunks;
    for (int c = 0; c < chunks; ++c) {
        const int b0 = blk0 + (int)((long long)(blk1 - blk0) * c / chunks);
        const int b1 = blk0 + (int)((long long)(blk1 - blk0) * (c + 1) / chunks);
        // MAS_FACTOR_VARIANT=5: the matrix-core formation (form_mfma, not bitwise)
        if (b1 > b0 && h->factorVariant == 5)
            k_factor_fused<true><<<b1 - b0, 64, 0, s>>>(a, P<float>(h->inv), P<uint4>(h->tileSlot),
                                                        P<uint4>(h->valuSlot), b0, P<int>(h->devStatus));
        else if (b1 > b0)
            k_factor_fused<false><<<b1 - b0, 64, 0, s>>>(a, P<float>(h->inv), P<uint4>(h->tileSlot),
                                                         P<uint4>(h->valuSlot), b0, P<int>(h->devStatus));
    }
    return hip_check(h, hipGetLastError(), "fused factor kernel");
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
    if ((rc = hip_check(h, hipMemcpy(h->slotTable.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice), "H2D slots")))
        return rc;
    // form_mfma's per-(tile, register, lane) slots: MFMA 32x32 D layout, lane l,
    // register r -> row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32
    const int tI[6] = {0, 0, 1, 0, 1, 2}, tJ[6] = {0, 1, 1, 2, 2, 2};
    std::vector<uint16_t> ts(12 * 64 * 8);
    for (int t = 0; t < 6; ++t)
        for (int r = 0; r < 16; ++r)
            for (int l = 0; l < 64; ++l) {
                const int i = 32 * tI[t] + 8 * (r >> 2) + 4 * (l >> 5) + (r & 3), j = 32 * tJ[t] + (l & 31);
                ts[((2 * t + (r >> 3)) * 64 + l) * 8 + (r & 7)] =
                    (tI[t] < tJ[t] || i <= j) ? (uint16_t)slot_of(i, j) : (uint16_t)0xFFFF;
            }
    if ((rc = ensure(h, h->tileSlot, ts.size() * 2)) ||
        (rc = hip_check(h, hipMemcpy(h->tileSlot.p, ts.data(), ts.size() * 2, hipMemcpyHostToDevice), "H2D tile slots")))
        return rc;
    // form_packed_staged's slots: 4x4 tile (I, J), I <= J, tile = J (J + 1) / 2 + I, entry 4 a + b
    std::vector<uint16_t> vs(300 * 16);
    for (int J = 0, tile = 0; J < 24; ++J)
        for (int I = 0; I <= J; ++I, ++tile)
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) {
                    const int i = 4 * I + a, j = 4 * J + b;
                    vs[tile * 16 + 4 * a + b] = i <= j ? (uint16_t)slot_of(i, j) : (uint16_t)0xFFFF;
                }
    if ((rc = ensure(h, h->valuSlot, vs.size() * 2))) return rc;
    return hip_check(h, hipMemcpy(h->valuSlot.p, vs.data(), vs.size() * 2, hipMemcpyHostToDevice), "H2D valu slots");
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

int factor_blocks(mas_context* h, int b0, int b1, hipStream_t s) {
    const int nb = b1 - b0;
    if (nb <= 0) return MAS_OK;
    float* dense = dense_base(h);
    float* inv = P<float>(h->inv);
    if (h->factorVariant == 0) {
        k_factor<<<nb, kFactorThreads, 0, s>>>(dense, P<unsigned>(h->slotTable), inv, b0, P<int>(h->devStatus));
    } else {
        k_identity_fix<<<cdiv(nb * 32, 256), 256, 0, s>>>(dense, b0 * 32, b1 * 32);
        // the matrix-core formation for the coarse blocks too unless the
        // reference's order is asked for (variant 4): 0.125 -> 0.104 ms at
        // 1M + contacts, coarse inverses within 4.4e-8 relative
        // (profiles/round5/ab/coarse_formation/)
        if (h->factorVariant == 3 || h->factorVariant == 5)
            k_factor_rb<true><<<nb, 64, 0, s>>>(dense, inv, P<uint4>(h->tileSlot), P<uint4>(h->valuSlot), b0,
                                                P<int>(h->devStatus));
        else
            k_factor_rb<false><<<nb, 64, 0, s>>>(dense, inv, P<uint4>(h->tileSlot), P<uint4>(h->valuSlot), b0,
                                                 P<int>(h->devStatus));
    }
    return hip_check(h, hipGetLastError(), "factor kernel");
}

int run_factor(mas_context* h, hipStream_t s) {
    // the prepared level-0 blocks (all, or a shard's; the fused variant factored
    // them already, on prepStream), then the coarse blocks: every one, or on a
    // Prepare with the coarse exchange those the rank alone has rows in (the
    // rest after the exchange, complete_coarse_rows)
    const bool fused = h->factorVariant >= 4;
    int rc;
    if (!fused && (rc = factor_blocks(h, h->fineBlk0, h->fineBlk1, s))) return rc;
    if (h->splitPlanned) {
        if (h->preFactored) return MAS_OK;  // on foldStream already (run_assemble)
        for (size_t i = 0; i + 1 < h->splitPre.size(); i += 2)
            if ((rc = factor_blocks(h, h->splitPre[i], h->splitPre[i + 1], s))) return rc;
        return MAS_OK;
    }
    return factor_blocks(h, h->nFineBlk, h->nBlk, s);  // run_prepare joins the fused kernel
}

}  // namespace mas
