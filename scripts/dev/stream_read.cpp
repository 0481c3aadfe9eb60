// Streaming-read ceiling probe: how fast can one kernel read N bytes of HBM on
// this chip (float4 loads, nontemporal or default policy, W waves per SIMD by
// occupancy), for comparison with k_solve_fine's 6.5-6.7 TB/s over 660.6 MB.
// hipcc --offload-arch=gfx950 -O3 scripts/dev/stream_read.cpp -o scripts/dev/bin/stream_read
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));
template <bool NT, int UNROLL>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ src, size_t n4, float* __restrict__ out) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x * UNROLL;
    for (size_t i = (size_t)blockIdx.x * blockDim.x * UNROLL + threadIdx.x; i < n4; i += stride) {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * blockDim.x;
            const size_t jc = j < n4 ? j : 0;
            v[u] = NT ? __builtin_nontemporal_load(src + jc) : src[jc];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.678f) out[blockIdx.x] = acc;  // keeps the loads
}

template <bool NT, int UNROLL>
static float run(const f4* d, size_t n4, float* out, int grid, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_read<NT, UNROLL><<<grid, 256>>>(d, n4, out);
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) k_read<NT, UNROLL><<<grid, 256>>>(d, n4, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 660602880ull;
    const size_t n4 = bytes / 16;
    f4* d = nullptr;
    float* out = nullptr;
    if (hipMalloc(&d, n4 * 16) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    hipMemset(d, 0, n4 * 16);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int wpc : {8, 16, 32}) {  // 256-thread workgroups: 4 waves each
        const int grid = cus * wpc / 4;
        const float t1 = run<true, 4>(d, n4, out, grid, 20), t2 = run<false, 4>(d, n4, out, grid, 20);
        const float t3 = run<true, 8>(d, n4, out, grid, 20);
        std::printf("bytes %zu waves/CU %d: nt x4 %.1f us %.2f TB/s | default x4 %.1f us %.2f TB/s | nt x8 %.1f us %.2f TB/s\n",
                    bytes, wpc, t1 * 1e3, bytes / (t1 * 1e-3) / 1e12, t2 * 1e3, bytes / (t2 * 1e-3) / 1e12, t3 * 1e3,
                    bytes / (t3 * 1e-3) / 1e12);
    }
    return 0;
}
