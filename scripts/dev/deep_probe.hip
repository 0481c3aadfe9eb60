// Dev probe: the pieces of a deep-level (l >= 3) residual fold at 1M scale
// (32 nodes x 1024 level-1 values, one 32-node block):
//   chain    a 1024-step dependent fadd chain, operands in registers / in LDS
//   node     one workgroup per node: contiguous 16 KB load -> LDS -> 3-lane fold
//   handoff  + acq_rel arrival counter, last arriver reads the 32 results
//   block    one workgroup folds all 32 nodes, streaming 384 KB through one CU
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off deep_probe.hip -o deep_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kLen = 1024, kNodes = 32;

__global__ void k_chain(const float* in, float* out, unsigned long long* t) {
    __shared__ float st[3][kLen];
    for (int i = threadIdx.x; i < 3 * kLen; i += blockDim.x) st[i / kLen][i % kLen] = in[i];
    __syncthreads();
    float acc = 0.f, r = in[threadIdx.x];
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 3)
        for (int k = 0; k < kLen; k += 4) {
            const float4 q = *reinterpret_cast<const float4*>(&st[threadIdx.x][k]);
            acc = __fadd_rn(acc, q.x);
            acc = __fadd_rn(acc, q.y);
            acc = __fadd_rn(acc, q.z);
            acc = __fadd_rn(acc, q.w);
        }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    float a2 = 0.f;
#pragma unroll 16
    for (int k = 0; k < kLen; ++k) {
        a2 = __fadd_rn(a2, r);
        asm volatile("" : "+v"(r));
    }
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = acc + a2;
    if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
}

// one workgroup per node; HANDOFF: arrival counter, last one reads all results
template <bool HANDOFF>
__global__ __launch_bounds__(256) void k_node(const float4* src, float4* res, int* cnt, float4* out) {
    __shared__ float st[3][kLen];
    __shared__ int last;
    const int t = threadIdx.x, node = blockIdx.x;
    float4 v[4];
    for (int q = 0; q < 4; ++q) v[q] = src[(size_t)node * kLen + t + 256 * q];
    for (int q = 0; q < 4; ++q) {
        st[0][t + 256 * q] = v[q].x;
        st[1][t + 256 * q] = v[q].y;
        st[2][t + 256 * q] = v[q].z;
    }
    __syncthreads();
    float acc = 0.f;
    if (t < 3)
        for (int k = 0; k < kLen; k += 4) {
            const float4 q = *reinterpret_cast<const float4*>(&st[t][k]);
            acc = __fadd_rn(acc, q.x);
            acc = __fadd_rn(acc, q.y);
            acc = __fadd_rn(acc, q.z);
            acc = __fadd_rn(acc, q.w);
        }
    if (t < 64) {
        const float ax = __shfl(acc, 0), ay = __shfl(acc, 1), az = __shfl(acc, 2);
        if (t == 0) {
            res[node] = make_float4(ax, ay, az, 0.f);
            if (HANDOFF) last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == kNodes - 1;
        }
    }
    if (!HANDOFF) return;
    __syncthreads();
    if (!last || t >= 64) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (t == 0) *cnt = 0;
    if (t < 32) out[t] = res[t];
}

// one workgroup (NT threads) folds all 32 nodes: 2 fold waves (lane 3j+c),
// the list streamed in steps of 64 entries per node through a 2-slot LDS ring
template <int NT>
__global__ __launch_bounds__(NT) void k_block(const float4* src, float4* out) {
    constexpr int kStep = 64;
    __shared__ float st[2][kNodes * 3][kStep + 4];
    const int t = threadIdx.x;
    constexpr int kPer = kNodes * kStep / NT;  // entries per thread per step
    float4 v[kPer];
    auto load = [&](int b) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int e = t + NT * q, node = e / kStep, i = e % kStep;
            v[q] = src[(size_t)node * kLen + b + i];
        }
    };
    load(0);
    float acc = 0.f;
    const int fl = t < 64 ? t : t - 64 + 63;  // fold lanes: wave 0 lanes 0..62, wave 1 lanes 0..32
    const bool folder = (t < 63) || (t >= 64 && t < 64 + 33);
    for (int b = 0, buf = 0; b < kLen; b += kStep, buf ^= 1) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int e = t + NT * q, node = e / kStep, i = e % kStep;
            st[buf][3 * node + 0][i] = v[q].x;
            st[buf][3 * node + 1][i] = v[q].y;
            st[buf][3 * node + 2][i] = v[q].z;
        }
        __syncthreads();
        if (b + kStep < kLen) load(b + kStep);
        if (folder)
            for (int k = 0; k < kStep; k += 4) {
                const float4 q = *reinterpret_cast<const float4*>(&st[buf][fl][k]);
                acc = __fadd_rn(acc, q.x);
                acc = __fadd_rn(acc, q.y);
                acc = __fadd_rn(acc, q.z);
                acc = __fadd_rn(acc, q.w);
            }
    }
    if (folder) reinterpret_cast<float*>(out)[fl] = acc;
}

template <class F>
static float time_us(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 20; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

__global__ void k_empty(float4* out) {
    if (threadIdx.x == 0 && blockIdx.x == 100000) out[0] = make_float4(0, 0, 0, 0);
}

int main() {
    float4 *src, *res, *out;
    float* fin;
    int* cnt;
    unsigned long long* t;
    hipMalloc(&src, (size_t)kNodes * kLen * 16);
    hipMalloc(&res, 64 * 16);
    hipMalloc(&out, 4096 * 16);
    hipMalloc(&fin, 4 * kLen * 4);
    hipMalloc(&cnt, 64);
    hipMalloc(&t, 64);
    hipMemset(cnt, 0, 64);
    std::vector<float4> h((size_t)kNodes * kLen);
    for (size_t i = 0; i < h.size(); ++i) h[i] = make_float4(1e-3f * (i % 97), 2e-3f * (i % 89), 3e-3f * (i % 83), 0);
    hipMemcpy(src, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    hipMemcpy(fin, h.data(), 4 * kLen * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        k_chain<<<1, 256>>>(fin, reinterpret_cast<float*>(out), t);
        unsigned long long ht[2];
        hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost);
        printf("1024-step chain: LDS-fed %.3f us, register %.3f us\n", ht[0] / 100.0, ht[1] / 100.0);
    }
    const int reps = 2000;
    printf("empty 1 wg          %.2f us\n", time_us([&] { k_empty<<<1, 256>>>(out); }, reps));
    printf("empty 1056 wg       %.2f us\n", time_us([&] { k_empty<<<1056, 256>>>(out); }, reps));
    printf("node x32            %.2f us\n", time_us([&] { k_node<false><<<kNodes, 256>>>(src, res, cnt, out); }, reps));
    printf("node x32 + handoff  %.2f us\n", time_us([&] { k_node<true><<<kNodes, 256>>>(src, res, cnt, out); }, reps));
    printf("block 256 thr       %.2f us\n", time_us([&] { k_block<256><<<1, 256>>>(src, out); }, reps));
    printf("block 512 thr       %.2f us\n", time_us([&] { k_block<512><<<1, 512>>>(src, out); }, reps));
    printf("block 1024 thr      %.2f us\n", time_us([&] { k_block<1024><<<1, 1024>>>(src, out); }, reps));
    return 0;
}
