// Do two HIP streams run kernels concurrently on this box?  A long streaming
// kernel (many workgroups) on stream A and a short latency-bound kernel (few
// workgroups) on stream B, launched after A; each records its first/last
// s_memrealtime.  Also tries a high-priority B stream.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_stream(const float4* __restrict__ a, float4* __restrict__ b, size_t n, unsigned long long* ts) {
    if (threadIdx.x == 0 && blockIdx.x == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        v.x += 1.f;
        b[i] = v;
    }
    if (threadIdx.x == 0) atomicMax(&ts[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

__global__ void k_small(unsigned long long* ts, int spin) {
    if (threadIdx.x == 0) atomicMin(&ts[2], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) {}
    if (threadIdx.x == 0) atomicMax(&ts[3], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int main() {
    const size_t n = 64ull << 20;  // 64M float4 = 1 GiB each
    float4 *a, *b;
    unsigned long long* ts;
    hipMalloc(&a, n * 16);
    hipMalloc(&b, n * 16);
    hipMalloc(&ts, 64);
    int lo, hi;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    for (int variant = 0; variant < 3; ++variant) {
        hipStream_t sa, sb;
        hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
        if (variant == 1) hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, hi);
        else hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
        for (int rep = 0; rep < 3; ++rep) {
            std::vector<unsigned long long> h = {0, 0, ~0ull, 0};
            hipMemcpy(ts, h.data(), 32, hipMemcpyHostToDevice);
            hipDeviceSynchronize();
            if (variant == 2) {  // B first, then A
                k_small<<<8, 64, 0, sb>>>(ts, 2000);  // ~20 us at 100 MHz
                k_stream<<<8192, 256, 0, sa>>>(a, b, n, ts);
            } else {
                k_stream<<<8192, 256, 0, sa>>>(a, b, n, ts);
                k_small<<<8, 64, 0, sb>>>(ts, 2000);
            }
            hipDeviceSynchronize();
            hipMemcpy(h.data(), ts, 32, hipMemcpyDeviceToHost);
            // s_memrealtime runs at 100 MHz
            printf("variant %d rep %d: stream [0, %.1f] us, small [%.1f, %.1f] us\n", variant, rep,
                   (h[1] - h[0]) / 100.0, ((long long)(h[2] - h[0])) / 100.0, ((long long)(h[3] - h[0])) / 100.0);
        }
        hipStreamDestroy(sa);
        hipStreamDestroy(sb);
    }
    return 0;
}
