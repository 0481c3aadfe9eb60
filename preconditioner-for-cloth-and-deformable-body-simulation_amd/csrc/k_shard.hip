// k_shard.hip -- Morton-range sharding of the apply across ranks.
//
// Rank g owns level-0 blocks [g*nb/W, (g+1)*nb/W).  Level-1 nodes are
// components of one level-0 bank and their ids are assigned in bank order, so
// the rank's level-1 nodes are the contiguous segment [l1_first[fb0],
// l1_first[fb1]).  Per apply and rank:
//   k_restrict_seg   R1 of the own segment (same ordered sums as k_coarse_l1)
//   -- caller: allgather of the padded segments over RCCL --
//   k_unpack_r1      gathered segments -> R1 of every level-1 node
//   k_solve_nodes    own level-1 blocks: Z1 = Inv R1
//   k_coarse_up      every block of levels >= 2 (tiny, redundant on all ranks)
//   k_solve_fine     own level-0 blocks + prolongation, z of own vertices
// Every value is computed by the same kernel arithmetic as the unsharded
// apply, so the union of the ranks' outputs is bitwise equal to it.
#include <algorithm>
#include <vector>

#include "block_solve.h"

namespace mas {

void launch_fine(mas_context* h, int blk0, int blkEnd, const float4* r, float4* z, hipStream_t s);
void launch_coarse_levels(mas_context* h, int lFirst, const float4* d_r, hipStream_t s);

__global__ __launch_bounds__(256) void k_restrict_seg(int l1Begin, int count, int segMax,
                                                      const int2* __restrict__ members, const int* __restrict__ s2o,
                                                      const float4* __restrict__ r, float4* __restrict__ seg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= segMax) return;
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (i < count) {
        const int2 mb = members[l1Begin + i];  // level-1 local id == coarse index
        const unsigned msk = (unsigned)mb.y;
        const int4* s4 = reinterpret_cast<const int4*>(s2o + mb.x * 32);
        int src[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int4 t = s4[q];
            src[4 * q] = t.x;
            src[4 * q + 1] = t.y;
            src[4 * q + 2] = t.z;
            src[4 * q + 3] = t.w;
        }
        float vx[32], vy[32], vz[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if ((msk >> j) & 1u) v = r[src[j]];
            vx[j] = v.x;
            vy[j] = v.y;
            vz[j] = v.z;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j)
            if ((msk >> j) & 1u) {
                ax = __fadd_rn(ax, vx[j]);
                ay = __fadd_rn(ay, vy[j]);
                az = __fadd_rn(az, vz[j]);
            }
    }
    seg[i] = make_float4(ax, ay, az, 0.f);
}

__global__ __launch_bounds__(256) void k_unpack_r1(int segMax, int world, const int* __restrict__ off,
                                                   const float4* __restrict__ gathered, float4* __restrict__ rc) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= segMax * world) return;
    const int rk = t / segMax, i = t % segMax;
    if (i < off[rk + 1] - off[rk]) rc[off[rk] + i] = gathered[t];
}

// Z = Inv R for blocks [blk0, blk0 + nb) whose R is already in Rc.
__global__ __launch_bounds__(kApplyThreads) void k_solve_nodes(const float4* __restrict__ inv, int blk0, int nb,
                                                              const float4* __restrict__ rc, float4* __restrict__ zc,
                                                              int begin1) {
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int w = blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= nb) return;
    const int blk = blk0 + w;
    const int node = blk * 32 + n - begin1;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    const float4 rr = rc[node];
    const float3 out = block_solve(g, tl, make_float3(rr.x, rr.y, rr.z), lane);
    if (lane < 32) zc[node] = make_float4(out.x, out.y, out.z, 0.f);
}

int compute_l1_first(mas_context* h, hipStream_t s) {
    const int nb = h->nFineBlk;
    h->l1First.assign(nb + 1, 0);
    if (h->L < 2) return MAS_OK;
    std::vector<int> gn((size_t)h->nV);
    int rc = hip_check(h, hipMemcpyAsync(gn.data(), h->goingNext.p, gn.size() * 4, hipMemcpyDeviceToHost, s),
                       "D2H goingNext");
    if (rc || (rc = hip_check(h, hipStreamSynchronize(s), "l1 sync"))) return rc;
    const int begin1 = h->levelSize[3];
    for (int b = 0; b < nb; ++b) {
        int m = 0x7fffffff;
        for (int v = 32 * b; v < std::min(32 * b + 32, h->nV); ++v) m = std::min(m, gn[v] - begin1);
        h->l1First[b] = m;
    }
    h->l1First[nb] = h->levelSize[2];
    return MAS_OK;
}

}  // namespace mas

using namespace mas;

extern "C" {

int mas_shard_plan(int nV, const int* l1_first, int rank, int world, mas_shard* out) {
    if (nV <= 0 || !l1_first || !out || world <= 0 || rank < 0 || rank >= world) return MAS_ERR_ARG;
    const int nb = (nV + 31) / 32;
    auto fb = [&](int g) { return (int)((long long)g * nb / world); };
    int segMax = 1;
    for (int g = 0; g < world; ++g) segMax = std::max(segMax, l1_first[fb(g + 1)] - l1_first[fb(g)]);
    out->rank = rank;
    out->world = world;
    out->fine_block_begin = fb(rank);
    out->fine_block_end = fb(rank + 1);
    out->vert_begin = std::min(32 * fb(rank), nV);
    out->vert_end = std::min(32 * fb(rank + 1), nV);
    out->l1_begin = l1_first[fb(rank)];
    out->l1_end = l1_first[fb(rank + 1)];
    out->seg_max = segMax;
    return MAS_OK;
}

int mas_shard_setup(mas_handle h, int rank, int world, mas_shard* out) {
    if (!h || !out) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "shard setup before prepare");
    return mas_shard_plan(h->nV, h->l1First.data(), rank, world, out);
}

int mas_apply_shard_restrict(mas_handle h, int rank, int world, const float* d_r4, float* d_seg4, void* stream) {
    if (!h || !d_r4 || !d_seg4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (h->L < 2) return hip_check(h, hipMemsetAsync(d_seg4, 0, (size_t)sh.seg_max * 16, s), "zero segment");
    k_restrict_seg<<<cdiv(sh.seg_max, 256), 256, 0, s>>>(sh.l1_begin, sh.l1_end - sh.l1_begin, sh.seg_max,
                                                         P<int2>(h->members), P<int>(h->s2o),
                                                         reinterpret_cast<const float4*>(d_r4),
                                                         reinterpret_cast<float4*>(d_seg4));
    return hip_check(h, hipGetLastError(), "shard restrict");
}

int mas_apply_shard_finish(mas_handle h, int rank, int world, const float* d_gathered4, const float* d_r4,
                           float* d_z4, void* stream) {
    if (!h || !d_gathered4 || !d_r4 || !d_z4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const float4* r = reinterpret_cast<const float4*>(d_r4);
    float4* z = reinterpret_cast<float4*>(d_z4);
    hipEvent_t* ev = nullptr;
    if (h->profiling && h->profRecorded < kProfRing) ev = &h->prof[4 * h->profRecorded++];
    if (ev) hipEventRecord(ev[0], s);
    if (h->L > 1) {
        if (h->shardWorld != world) {  // per-rank segment offsets (level-1 local ids)
            std::vector<int> off(world + 1);
            for (int g = 0; g <= world; ++g) off[g] = h->l1First[(int)((long long)g * h->nFineBlk / world)];
            if ((rc = ensure(h, h->shardOff, (size_t)(world + 1) * 4)) ||
                (rc = hip_check(h, hipMemcpy(h->shardOff.p, off.data(), off.size() * 4, hipMemcpyHostToDevice),
                                "H2D shard offsets")))
                return rc;
            h->shardWorld = world;
        }
        const int begin1 = h->levelSize[3];
        k_unpack_r1<<<cdiv((long long)sh.seg_max * world, 256), 256, 0, s>>>(
            sh.seg_max, world, P<int>(h->shardOff), reinterpret_cast<const float4*>(d_gathered4), P<float4>(h->Rc));
        if (sh.l1_end > sh.l1_begin) {
            const int b0 = sh.l1_begin / 32, b1 = (sh.l1_end + 31) / 32;
            k_solve_nodes<<<cdiv(b1 - b0, kApplyThreads / 64), kApplyThreads, 0, s>>>(
                P<float4>(h->inv), begin1 / 32 + b0, b1 - b0, P<float4>(h->Rc), P<float4>(h->Zc), begin1);
        }
        launch_coarse_levels(h, 2, r, s);
    }
    if (ev) hipEventRecord(ev[1], s);
    launch_fine(h, sh.fine_block_begin, sh.fine_block_end, r, z, s);
    if (ev) hipEventRecord(ev[2], s);
    if (ev) hipEventRecord(ev[3], s);
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "shard finish");
}

}  // extern "C"
