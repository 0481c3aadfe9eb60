// fold_rate.hip -- how fast can one wave run a dependent fp32 left fold?
// (the level-3 residual fold, k_coarse1.hip / deep_fold.h).  One wave per
// launch; lanes 0..2 fold x, y, z of N values each; cycles from s_memtime.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off scripts/dev/fold_rate.hip -o scripts/dev/bin/fold_rate
#include <hip/hip_runtime.h>

#include "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/csrc/deep_fold.h"

#include <cstdio>
#include <vector>

constexpr int N = 4096;

// s_memtime: shader-clock cycles; s_memrealtime: the 100 MHz constant clock
__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long now_rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// (a) the current form: component-major LDS rows, float4 reads, 8 in flight
__global__ void k_lds(const float* __restrict__ in, float* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float st[3][N];
    const int lane = threadIdx.x;
    for (int i = lane; i < N; i += 64)
        for (int c = 0; c < 3; ++c) st[c][i] = in[c * N + i];
    __syncthreads();
    const unsigned long long r0 = now_rt(), t0 = now();
    float acc = 0.f;
    if (lane < 3) {
        const float4* row = reinterpret_cast<const float4*>(st[lane]);
        const int n4 = N / 4;
        float4 cur[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = row[k];
        for (int k0 = 0; k0 < n4; k0 += 8) {
            const int kn = k0 + 8 < n4 ? k0 + 8 : k0;
            float4 nxt[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) nxt[k] = row[kn + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                acc = __fadd_rn(acc, cur[k].x);
                acc = __fadd_rn(acc, cur[k].y);
                acc = __fadd_rn(acc, cur[k].z);
                acc = __fadd_rn(acc, cur[k].w);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        }
    }
    const unsigned long long t1 = now(), r1 = now_rt();
    if (lane < 3) out[lane] = acc;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

// (a2) mas::fold_row<B>, the product's fold (deep_fold.h)
template <int B>
__global__ void k_lds_b(const float* __restrict__ in, float* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float st[3][N];
    const int lane = threadIdx.x;
    for (int i = lane; i < N; i += 64)
        for (int c = 0; c < 3; ++c) st[c][i] = in[c * N + i];
    __syncthreads();
    const unsigned long long r0 = now_rt(), t0 = now();
    float acc = 0.f;
    if (lane < 3) acc = mas::fold_row<B>(reinterpret_cast<const float4*>(st[lane]), N / 4, 0.f);
    const unsigned long long t1 = now(), r1 = now_rt();
    if (lane < 3) out[lane] = acc;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

// (b) values already in registers: a pure dependent add chain
__global__ void k_reg(const float* __restrict__ in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    float v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = in[(lane % 3) * N + k];
    const unsigned long long r0 = now_rt(), t0 = now();
    float acc = 0.f;
    for (int r = 0; r < N / 64; ++r) {
#pragma unroll
        for (int k = 0; k < 64; ++k) acc = __fadd_rn(acc, v[k]);
        asm volatile("" : "+v"(acc));
    }
    const unsigned long long t1 = now(), r1 = now_rt();
    if (lane < 3) out[lane] = acc;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

// (c) two independent chains interleaved (what the issue rate allows)
__global__ void k_reg2(const float* __restrict__ in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    float v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = in[(lane % 3) * N + k];
    const unsigned long long r0 = now_rt(), t0 = now();
    float a0 = 0.f, a1 = 0.f;
    for (int r = 0; r < N / 128; ++r) {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            a0 = __fadd_rn(a0, v[k]);
            a1 = __fadd_rn(a1, v[63 - k]);
        }
        asm volatile("" : "+v"(a0), "+v"(a1));
    }
    const unsigned long long t1 = now(), r1 = now_rt();
    if (lane < 3) out[lane] = a0 + a1;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

int main() {
    std::vector<float> h(3 * N);
    for (int i = 0; i < 3 * N; ++i) h[i] = 1.0f / (1 + i % 97);
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, h.size() * 4);
    hipMalloc(&dout, 64);
    hipMalloc(&dc, 16);
    hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    auto run = [&](const char* name, void (*k)(const float*, float*, unsigned long long*)) {
        unsigned long long best = ~0ull, rt = 0;
        for (int it = 0; it < 5; ++it) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, dc);
            unsigned long long c[2];
            hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
            if (c[0] < best) { best = c[0]; rt = c[1]; }
        }
        float o[3];
        hipMemcpy(o, dout, 12, hipMemcpyDeviceToHost);
        printf("  acc %08x %08x %08x\n", *(unsigned*)&o[0], *(unsigned*)&o[1], *(unsigned*)&o[2]);
        printf("%-34s %8llu cycles for %d dependent adds = %.2f cycles/add, %.2f us (%.2f ns/add)\n", name, best, N,
               (double)best / N, rt / 100.0, rt * 10.0 / N);
    };
    run("(a) LDS float4 rows, 8 in flight", k_lds);
    run("(a2) fold_row<8>", k_lds_b<8>);
    run("(a2) fold_row<16>", k_lds_b<16>);
    run("(a2) fold_row<32>", k_lds_b<32>);
    run("(b) registers, one chain", k_reg);
    run("(c) registers, two chains", k_reg2);
    hipDeviceSynchronize();
    return 0;
}
