// Dev probe: latency of one wave's 32-node block solve (block_solve.h) when
// nothing else runs -- the cost that bounds the coarse levels >= 2 (1-32
// blocks) -- next to a dependent (cache-resident) load and an agent-scope
// atomic round trip.  Measured on MI355X: 1.25 us / 0.09 us / 0.40 us.  An
// LDS-staged variant of the solve (operands through LDS in two bursts instead
// of ds_bpermute steps, same arithmetic) measured 1.8 us and was dropped.  Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../preconditioner-for-cloth-and-deformable-body-simulation_amd/csrc solve_latency.hip -o solve_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "block_solve.h"

using namespace mas;

__global__ void k_probe(const float4* inv, float4* out, unsigned* ctr, unsigned long long* t, int iters) {
    const int lane = threadIdx.x;
    float g[kRecord], tl[3];
    load_record<false>(inv, 0, lane, g, tl);
    float3 r = make_float3(1.f + lane, 2.f, 3.f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) r = block_solve(g, tl, r, lane);
    asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z));
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    // dependent loads (pointer chase through out[])
    int idx = lane;
    for (int i = 0; i < iters; ++i) idx = (int)(out[idx].w) & 1023;
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    // atomic round trips
    unsigned v = 0;
    for (int i = 0; i < iters; ++i) {
        if (lane == 0) v += __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = __shfl(v, 0);
    }
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    if (lane < 32) out[2048 + lane] = make_float4(r.x, r.y, r.z, (float)(idx + v));
    if (lane == 0) { t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; }
}

int main() {
    float4 *inv, *out; unsigned* ctr; unsigned long long* t;
    hipMalloc(&inv, kBlockF4 * 16);
    hipMalloc(&out, 4096 * 16);
    hipMalloc(&ctr, 64);
    hipMalloc(&t, 64);
    std::vector<float4> h(kBlockF4, make_float4(0.01f, 0.02f, 0.03f, 0.f));
    hipMemcpy(inv, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    std::vector<float4> o(4096);
    for (int i = 0; i < 4096; ++i) o[i] = make_float4(0, 0, 0, (float)((i * 37 + 11) & 1023));
    hipMemcpy(out, o.data(), o.size() * 16, hipMemcpyHostToDevice);
    const int iters = 100;
    for (int rep = 0; rep < 3; ++rep) {
        k_probe<<<1, 64>>>(inv, out, ctr, t, iters);
        unsigned long long ht[3];
        hipMemcpy(ht, t, 24, hipMemcpyDeviceToHost);
        printf("block_solve %.3f us   dependent load %.3f us   atomic round trip %.3f us\n", ht[0] / 100.0 / iters,
               ht[1] / 100.0 / iters, ht[2] / 100.0 / iters);
    }
    return 0;
}
