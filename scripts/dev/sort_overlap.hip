// Why does a radix sort on one stream stall behind the fused level-0 kernel
// on another?  An "occupier" kernel on stream A holds one-wave workgroups
// resident for ~2 ms (VGPRs forced high by a clobber, optional LDS); stream B
// then runs a hipcub pair sort of 1M 27-bit keys, or 1024-/256-/64-thread
// probe kernels with LDS.  Prints B's time alone and beside each occupier.
// hipcc --offload-arch=gfx950 -O3 scripts/dev/sort_overlap.hip -o /tmp/sort_overlap
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>

template <int LDS, bool HIGHV, bool SCRATCH = false>
__global__ __launch_bounds__(64) void k_occupy(unsigned long long spin, int* sink) {
    __shared__ int buf[LDS / 4 > 0 ? LDS / 4 : 1];
    if (LDS > 0) buf[threadIdx.x] = threadIdx.x;
    if (SCRATCH) {  // a dynamically indexed private array lives in scratch
        volatile int arr[32];
        for (int i = 0; i < 32; ++i) arr[i] = i * threadIdx.x;
        if (arr[(threadIdx.x * 7) & 31] == -5) sink[0] = 2;
    }
    if (HIGHV) asm volatile("" ::: "v247");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
    if (LDS > 0 && buf[(threadIdx.x + 1) & 63] == -1) sink[0] = 1;
}

// streams memory for ~spin ticks (the real fused kernel is bandwidth- and latency-heavy)
__global__ __launch_bounds__(64) void k_occupy_mem(unsigned long long spin, const float4* __restrict__ src, size_t n,
                                                  int* sink) {
    __shared__ int buf[19968 / 4];
    buf[threadIdx.x] = threadIdx.x;
    asm volatile("" ::: "v247");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc = 0.f;
    size_t i = (blockIdx.x * 64 + threadIdx.x) * 97;
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
        for (int k = 0; k < 16; ++k) { acc += src[i % n].x; i += 65536 * 13; }
    }
    if (acc == -1.f || buf[(threadIdx.x + 1) & 63] == -1) sink[0] = 3;
}

// keeps one-wave workgroups busy for ~spin ticks (to disturb the placement)
__global__ __launch_bounds__(64) void k_busy(unsigned long long spin) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
}

template <int THREADS, int LDS>
__global__ __launch_bounds__(THREADS) void k_probe(int* out) {
    __shared__ int buf[LDS / 4];
    buf[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[blockIdx.x * THREADS + threadIdx.x] = buf[(threadIdx.x + 1) % THREADS];
}

int main() {
    const int n = 1 << 20;
    unsigned *k0, *k1;
    int *v0, *v1, *sink, *out;
    hipMalloc(&k0, n * 4); hipMalloc(&k1, n * 4); hipMalloc(&v0, n * 4); hipMalloc(&v1, n * 4);
    hipMalloc(&sink, 4); hipMalloc(&out, 64 << 20);
    std::vector<unsigned> hk(n);
    unsigned x = 1;
    for (auto& k : hk) { x = x * 1664525u + 1013904223u; k = x >> 5; }
    hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
    size_t tmp = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k0, k1, v0, v1, n, 0, 27);
    void* t; hipMalloc(&t, tmp);
    hipStream_t sa, sb;
    hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned long long spin = 200000;  // 2 ms at 100 MHz
    auto job = [&](int which) {
        switch (which) {
        case 0: hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, v0, v1, n, 0, 27, sb); break;
        case 1: k_probe<1024, 21504><<<cus * 4, 1024, 0, sb>>>(out); break;
        case 2: k_probe<256, 21504><<<cus * 4, 256, 0, sb>>>(out); break;
        case 3: k_probe<64, 2560><<<cus * 16, 64, 0, sb>>>(out); break;
        }
    };
    const char* jobName[] = {"hipcub sort 1M pairs", "1024-thr WGs 21KB", "256-thr WGs 21KB", "64-thr WGs 2.5KB"};
    auto occ = [&](int v, int wgs) {
        switch (v) {
        case 1: k_occupy<19968, true><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 2: k_occupy<0, true><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 3: k_occupy<19968, false><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 4: k_occupy<0, false><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 5: k_occupy<19968, true, true><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 6: k_occupy<0, false, true><<<wgs, 64, 0, sa>>>(spin, sink); break;
        case 7: k_occupy_mem<<<wgs, 64, 0, sa>>>(spin, reinterpret_cast<const float4*>(out), (64 << 20) / 16, sink); break;
        case 8:  // placement disturbed: single-wave work on B's stream first
            k_busy<<<cus * 3, 64, 0, sb>>>(5000);
            k_occupy<19968, true, true><<<wgs, 64, 0, sa>>>(spin, sink);
            break;
        }
    };
    const char* occName[] = {"alone", "LDS20K+248VGPR", "248VGPR", "LDS20K", "bare", "LDS+VGPR+scratch", "scratch", "mem-streaming", "after busy B"};
    for (int j = 0; j < 4; ++j) {
        for (int v = 0; v < 9; ++v) {
            for (int per = 4; per <= 8; per += 4) {
                if (v == 0 && per == 8) continue;
                float best = 1e9f;
                for (int rep = 0; rep < 3; ++rep) {
                    hipDeviceSynchronize();
                    if (v) occ(v, per * cus);
                    hipEventRecord(e0, sb);
                    job(j);
                    hipEventRecord(e1, sb);
                    hipDeviceSynchronize();
                    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                printf("%-22s beside %-16s (%d/CU): %8.1f us\n", jobName[j], occName[v], v ? per : 0, best * 1e3f);
            }
        }
    }
    return 0;
}
