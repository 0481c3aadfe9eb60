// k_shard.hip -- Morton-range sharding of the apply across ranks.
//
// Rank g owns level-0 blocks [g*nb/W, (g+1)*nb/W).  Level-1 nodes are
// components of one level-0 bank and their ids are assigned in bank order, so
// the rank's level-1 nodes are the contiguous segment [l1_first[fb0],
// l1_first[fb1]).  Per apply and rank:
//   k_restrict_seg   R1 of the own segment (same ordered sums as k_coarse_l1)
//   -- caller: allgather of the padded segments over RCCL --
//   k_shard_coarse12 own level-1 blocks (Z1 = Inv R1) and every level-2 block
//                    (R2 from the gathered R1, Z2), straight from the
//                    gathered segments, one launch
//                    and, in the same launch, every level-3 node (R folded
//                    from the gathered R1 in the reference's order; redundant
//                    on all ranks)
//   k_solve_fine     own level-0 blocks + prolongation, z of own vertices
// or, overlapped (mas_apply_shard_fine / _complete): k_solve_fine without the
// coarse terms while the allgather is in flight, then the coarse kernels and
// k_prolong over the own vertices.
// Every value is computed by the same kernel arithmetic as the unsharded
// apply, so the union of the ranks' outputs is bitwise equal to it.
#include <algorithm>
#include <string>
#include <vector>

#include "block_solve.h"
#include "deep_fold.h"

namespace mas {


// R1 of the own level-1 segment, one thread per node: the children's
// original ids come from l1src (32 per node, -1 where none, built at Prepare),
// so the r gather is the second dependent load; summed in lane order from +0
// as k_coarse_l1.
__global__ __launch_bounds__(64) void k_restrict_seg(int l1Begin, int count, int segMax, const int* __restrict__ l1src,
                                                      const float4* __restrict__ r, float4* __restrict__ seg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= segMax) return;
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (i < count) {
        const int4* s4 = reinterpret_cast<const int4*>(l1src + (size_t)(l1Begin + i) * 32);
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
            const float4 v = r[src[j] >= 0 ? src[j] : 0];
            vx[j] = v.x;
            vy[j] = v.y;
            vz[j] = v.z;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j)
            if (src[j] >= 0) {
                ax = __fadd_rn(ax, vx[j]);
                ay = __fadd_rn(ay, vy[j]);
                az = __fadd_rn(az, vz[j]);
            }
    }
    seg[i] = make_float4(ax, ay, az, 0.f);
}

// pos1[i] = index of level-1 node i's R1 in the gathered buffer
// (g * segMax + i - off[g] for the rank g whose segment holds i); rebuilt when
// the world size changes.
__global__ __launch_bounds__(256) void k_shard_pos1(int n1, int world, int segMax, const int* __restrict__ off,
                                                    int* __restrict__ pos1) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n1) return;
    int lo = 0, hi = world;  // largest g with off[g] <= i (skips empty segments)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid;
        else hi = mid;
    }
    pos1[i] = lo * segMax + (i - off[lo]);
}

// Grouped level 3 of a sharded apply (mas_config.reference_restriction = 0):
// node T's children are the lanes of one component of one level-2 bank
// (members); lane j computes child j's R2 from the gathered R1 exactly as the
// level-2 waves below (its children in lane order from +0), then R3 is those
// R2 folded in lane order from +0 -- bitwise the unsharded grouped level 3
// (k_coarse.hip solve3_grouped_wave over k_restrict12's R2).  Wave 0 computes
// and publishes R3 and counts the arrival; the block's last arriver solves
// the block with the inverse wave 1 prefetched (deep_fold.h protocol).
__device__ __forceinline__ void deep_node_grouped(const float4* __restrict__ inv, int node,
                                                  const float4* __restrict__ gathered, const int* __restrict__ pos1,
                                                  const int2* __restrict__ members, int lv2Begin, int begin1,
                                                  float4* __restrict__ rc, float4* __restrict__ zc, const DeepArgs& d) {
    __shared__ int last;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, j = lane & 31;
    const int blk = node >> 5;
    float g[kRecord], tl[3];
    if (w == 1) load_record<true>(inv, blk, lane, g, tl);
    if (w == 0) {
        const int2 mbT = members[node - begin1];  // (level-2 bank, children)
        const bool child = lane < 32 && (((unsigned)mbT.y >> j) & 1u);
        float ax = 0.f, ay = 0.f, az = 0.f;
        if (child) {
            const int2 mb = members[lv2Begin + mbT.x * 32 + j - begin1];  // (level-1 bank, children)
            const unsigned msk = (unsigned)mb.y;
            const int4* p4 = reinterpret_cast<const int4*>(pos1 + mb.x * 32);
            int src[32];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int4 v = p4[q];
                src[4 * q] = v.x;
                src[4 * q + 1] = v.y;
                src[4 * q + 2] = v.z;
                src[4 * q + 3] = v.w;
            }
            float vx[32], vy[32], vz[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                const float4 v = gathered[(msk >> k) & 1u ? src[k] : 0];
                vx[k] = v.x; vy[k] = v.y; vz[k] = v.z;
            }
#pragma unroll
            for (int k = 0; k < 32; ++k)
                if ((msk >> k) & 1u) {
                    ax = __fadd_rn(ax, vx[k]);
                    ay = __fadd_rn(ay, vy[k]);
                    az = __fadd_rn(az, vz[k]);
                }
        }
        // R3: the children's R2 in lane order from +0 (others +0.0)
        float bx = 0.f, by = 0.f, bz = 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            bx = __fadd_rn(bx, __shfl(ax, k));
            by = __fadd_rn(by, __shfl(ay, k));
            bz = __fadd_rn(bz, __shfl(az, k));
        }
        if (t == 0) {
            st_wt(rc + node - begin1, make_float4(bx, by, bz, 0.f));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int old = __hip_atomic_fetch_add(d.cnt + (blk - d.lv3Begin / 32), 1, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            last = old == 31;
        }
    }
    __syncthreads();
    if (!last || w != 1) return;
    if (lane == 0) d.cnt[blk - d.lv3Begin / 32] = 0;  // for the next apply (visible after this kernel)
    const int n = lane & 31;
    const float4 R = ld_wt(rc + blk * 32 + n - begin1);
    const float3 out = block_solve(g, tl, make_float3(R.x, R.y, R.z), lane);
    if (lane < 32) zc[blk * 32 + n - begin1] = make_float4(out.x, out.y, out.z, 0.f);
}

// Levels 1 and 2 of a sharded apply in ONE launch, straight from the gathered
// segments (no unpack pass): waves [0, nOwn1) solve the rank's own level-1
// blocks (Z1 = Inv R1), waves [nOwn1, nOwn1 + nb2) compute R2 of every level-2
// block -- each node sums its children's R1 in child-lane order from +0, as
// k_coarse_up -- and solve it.  Both only read the gathered R1, so they are
// independent.  The first nDeep workgroups fold level 3 (every node, from the
// gathered R1 through deepIdxShard, in the reference's order: deep_fold.h)
// in the same launch.  Replaces unpack + own level-1 solve + one launch per
// coarser level (latency-bound launches).
__global__ __launch_bounds__(kApplyThreads) void k_shard_coarse12(
    const float4* __restrict__ inv, const float4* __restrict__ gathered, const int* __restrict__ pos1, int own1Blk0,
    int nOwn1, int n1, int lv2Blk0, int nb2, int n2, const int2* __restrict__ members, int begin1,
    float4* __restrict__ rc, float4* __restrict__ zc, DeepArgs d, int nDeep, int groupedLv2Begin) {
    if ((int)blockIdx.x < nDeep) {  // workgroup-uniform
        if (groupedLv2Begin >= 0)
            deep_node_grouped(inv, d.lv3Begin + blockIdx.x, gathered, pos1, members, groupedLv2Begin, begin1, rc, zc,
                              d);
        else
            deep_node<true>(inv, d.lv3Begin + blockIdx.x, d, rc, zc, begin1);
        return;
    }
    // the level-1/2 waves have slack: held back as in k_solve123 (one-rank
    // sharded complete 31.0-31.5 -> 30.5-30.8 us)
    if (nDeep > 0) __builtin_amdgcn_s_sleep(64);
    const int lane = threadIdx.x & 63, n = lane & 31;
    const int w = (blockIdx.x - nDeep) * (kApplyThreads / 64) + (threadIdx.x >> 6);
    if (w >= nOwn1 + nb2) return;  // wave-uniform
    const bool l1 = w < nOwn1;
    const int blk = l1 ? own1Blk0 + w : lv2Blk0 + (w - nOwn1);
    const int node = blk * 32 + n;
    float g[kRecord], tl[3];
    load_record<true>(inv, blk, lane, g, tl);
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (l1) {
        const int i = node - begin1;
        if (lane < 32 && i < n1) {
            const float4 v = gathered[pos1[i]];
            ax = v.x; ay = v.y; az = v.z;
        }
    } else if (lane < 32 && node - lv2Blk0 * 32 < n2) {
        const int2 mb = members[node - begin1];
        const unsigned msk = (unsigned)mb.y;
        const int4* p4 = reinterpret_cast<const int4*>(pos1 + mb.x * 32);  // the child bank's 32 level-1 ids
        int src[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int4 t = p4[q];
            src[4 * q] = t.x;
            src[4 * q + 1] = t.y;
            src[4 * q + 2] = t.z;
            src[4 * q + 3] = t.w;
        }
        float vx[32], vy[32], vz[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const float4 v = gathered[(msk >> j) & 1u ? src[j] : 0];
            vx[j] = v.x; vy[j] = v.y; vz[j] = v.z;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((msk >> j) & 1u) {
                ax = __fadd_rn(ax, vx[j]);
                ay = __fadd_rn(ay, vy[j]);
                az = __fadd_rn(az, vz[j]);
            }
        }
    }
    // half 1 takes node n's residual from lane n
    ax = __shfl(ax, n);
    ay = __shfl(ay, n);
    az = __shfl(az, n);
    const float3 out = block_solve(g, tl, make_float3(ax, ay, az), lane);
    if (lane < 32) {
        rc[node - begin1] = make_float4(ax, ay, az, 0.f);
        zc[node - begin1] = make_float4(out.x, out.y, out.z, 0.f);
    }
}

__global__ __launch_bounds__(256) void k_copy16(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[i];
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

static const char* const kRowsPending =
    "sharded Prepare: its coarse rows were not exchanged yet (mas_prepare_shard_rows / mas_prepare_shard_complete)";

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
    if (h->l1First.empty()) {  // first shard call after a Prepare (kept out of Prepare's time)
        hipSetDevice(h->device);
        if (int rc = compute_l1_first(h, h->stream)) return rc;
    }
    return mas_shard_plan(h->nV, h->l1First.data(), rank, world, out);
}

int mas_apply_shard_restrict(mas_handle h, int rank, int world, const float* d_r4, float* d_seg4, void* stream) {
    if (!h || !d_r4 || !d_seg4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    if (h->rowsPending) return fail(h, MAS_ERR_STATE, kRowsPending);
    hipSetDevice(h->device);  // ensure() allocates on the current device (shard_coarse's tables)
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (h->L < 2) return hip_check(h, hipMemsetAsync(d_seg4, 0, (size_t)sh.seg_max * 16, s), "zero segment");
    k_restrict_seg<<<cdiv(sh.seg_max, 64), 64, 0, s>>>(sh.l1_begin, sh.l1_end - sh.l1_begin, sh.seg_max,
                                                         P<int>(h->l1src), reinterpret_cast<const float4*>(d_r4),
                                                         reinterpret_cast<float4*>(d_seg4));
    return hip_check(h, hipGetLastError(), "shard restrict");
}

// The coarse levels of a sharded apply from the gathered level-1 segments:
// R1 of every level-1 node, Z1 of the own level-1 blocks, every block of
// levels >= 2.
static int shard_coarse(mas_context* h, const mas_shard& sh, int world, const float* d_gathered4, hipStream_t s) {
    int rc;
    if (h->L >= 4 && !h->deepOff.p) return fail(h, MAS_ERR_STATE, "shard apply: deep-level lists not built");
    const int n1 = h->levelSize[2];
    if (h->shardWorld != world) {  // per-rank segment offsets (level-1 local ids) -> pos1
        std::vector<int> off(world + 1);
        for (int g = 0; g <= world; ++g) off[g] = h->l1First[(int)((long long)g * h->nFineBlk / world)];
        if ((rc = ensure(h, h->shardOff, (size_t)(world + 1) * 4)) ||
            (rc = ensure(h, h->shardPos1, (size_t)ceil32(n1) * 4)) ||
            (rc = hip_check(h, hipMemcpy(h->shardOff.p, off.data(), off.size() * 4, hipMemcpyHostToDevice),
                            "H2D shard offsets")) ||
            (rc = hip_check(h, hipMemsetAsync(h->shardPos1.p, 0, (size_t)ceil32(n1) * 4, s), "memset pos1")))
            return rc;
        k_shard_pos1<<<cdiv(n1, 256), 256, 0, s>>>(n1, world, sh.seg_max, P<int>(h->shardOff), P<int>(h->shardPos1));
        if ((rc = build_deep_shard_idx(h, s))) return rc;
        h->shardWorld = world;
    }
    const int begin1 = h->levelSize[3];
    const int own0 = sh.l1_end > sh.l1_begin ? sh.l1_begin / 32 : 0;
    const int nOwn1 = sh.l1_end > sh.l1_begin ? (sh.l1_end + 31) / 32 - own0 : 0;
    const int nb2 = h->L > 2 ? ceil32(h->levelSize[4]) / 32 : 0;
    const int n2 = h->L > 2 ? h->levelSize[4] : 0;
    const int lv2Blk0 = h->L > 2 ? h->levelSize[5] / 32 : 0;
    // level 3 in the same launch: R from the gathered R1, grouped by level-2
    // node (the default) or folded in the reference's order
    const DeepArgs d = deep_args(h, reinterpret_cast<const float4*>(d_gathered4), P<int>(h->deepIdxShard));
    const int nDeep = deep_nodes(h);
    if (nDeep + nOwn1 + nb2 > 0)
        k_shard_coarse12<<<nDeep + cdiv(nOwn1 + nb2, kApplyThreads / 64), kApplyThreads, 0, s>>>(
            P<float4>(h->inv), reinterpret_cast<const float4*>(d_gathered4), P<int>(h->shardPos1), begin1 / 32 + own0,
            nOwn1, n1, lv2Blk0, nb2, n2, P<int2>(h->members), begin1, P<float4>(h->Rc), P<float4>(h->Zc), d, nDeep,
            h->groupedR3 ? h->levelSize[5] : -1);
    return MAS_OK;
}

// the shard's level-0 blocks must be among those the last Prepare factored
static int check_fine_prepared(mas_context* h, const mas_shard& sh) {
    if (sh.fine_block_begin < h->fineBlk0 || sh.fine_block_end > h->fineBlk1)
        return fail(h, MAS_ERR_STATE, "sharded apply: level-0 blocks [" + std::to_string(sh.fine_block_begin) + ", " +
                                          std::to_string(sh.fine_block_end) + ") were not prepared on this handle");
    return MAS_OK;
}

static hipEvent_t* shard_events(mas_context* h) {
    return h->profiling && h->profRecorded < kProfRing ? &h->prof[4 * h->profRecorded++] : nullptr;
}

int mas_apply_shard_finish(mas_handle h, int rank, int world, const float* d_gathered4, const float* d_r4,
                           float* d_z4, void* stream) {
    if (!h || !d_gathered4 || !d_r4 || !d_z4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    if (h->rowsPending) return fail(h, MAS_ERR_STATE, kRowsPending);
    hipSetDevice(h->device);  // ensure() allocates on the current device (shard_coarse's tables)
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    if ((rc = check_fine_prepared(h, sh))) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const float4* r = reinterpret_cast<const float4*>(d_r4);
    float4* z = reinterpret_cast<float4*>(d_z4);
    hipEvent_t* ev = shard_events(h);
    if (ev) hipEventRecord(ev[0], s);
    if (h->L > 1 && (rc = shard_coarse(h, sh, world, d_gathered4, s))) return rc;
    if (ev) hipEventRecord(ev[1], s);
    launch_fine(h, sh.fine_block_begin, sh.fine_block_end, r, z, s);
    if (ev) hipEventRecord(ev[2], s);
    if (ev) hipEventRecord(ev[3], s);
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "shard finish");
}

// Profiling events of the overlapped form: [0] = [1] before the level-0
// kernel (fine), [2] after it, [3] after complete (allgather wait + coarse +
// prolongation), so fine_ms_avg is the level-0 kernel as in the other forms.
int mas_apply_shard_fine(mas_handle h, int rank, int world, const float* d_r4, float* d_z4, void* stream) {
    if (!h || !d_r4 || !d_z4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    if (h->rowsPending) return fail(h, MAS_ERR_STATE, kRowsPending);
    hipSetDevice(h->device);  // ensure() allocates on the current device (shard_coarse's tables)
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    if ((rc = check_fine_prepared(h, sh))) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    hipEvent_t* ev = shard_events(h);
    h->shardPendingEv = ev;
    if (ev) {
        hipEventRecord(ev[0], s);
        hipEventRecord(ev[1], s);
    }
    launch_fine_z0(h, sh.fine_block_begin, sh.fine_block_end, reinterpret_cast<const float4*>(d_r4),
                   reinterpret_cast<float4*>(d_z4), s);
    if (ev) hipEventRecord(ev[2], s);
    return hip_check(h, hipGetLastError(), "shard fine");
}

int mas_apply_shard_complete(mas_handle h, int rank, int world, const float* d_gathered4, float* d_z4,
                             void* stream) {
    if (!h || !d_gathered4 || !d_z4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    if (h->rowsPending) return fail(h, MAS_ERR_STATE, kRowsPending);
    hipSetDevice(h->device);  // ensure() allocates on the current device (shard_coarse's tables)
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (h->L > 1) {
        if ((rc = shard_coarse(h, sh, world, d_gathered4, s))) return rc;
        launch_prolong(h, sh.vert_begin, sh.vert_end, reinterpret_cast<float4*>(d_z4), s);
    }
    if (h->shardPendingEv) hipEventRecord(h->shardPendingEv[3], s);
    h->shardPendingEv = nullptr;
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "shard complete");
}

// The whole per-rank apply with the collective inside (include/mas_capi.h).
// Default (shardMode 0): everything on `stream` -- restrict, the allgather
// hook enqueued on `stream` itself, the coarse levels, the own level-0 blocks
// with the prolongation fused (mas_apply_shard_finish).  No cross-stream
// dependency: on MI355X a hipStreamWaitEvent hop between two queues measured
// ~14 us each (world-8 rank at 1M + contacts with the loopback collective:
// inline 31 us per apply; the collective on a communication stream joined
// back by events 60 us; profiles/round6/shard/), and a level-0 kernel queued
// beside the collective fills every CU, so the collective's kernel starts
// only as it drains (the same as the round-1 probe of a kernel queued behind
// an 8k-workgroup one: 50-70 us late).  shardMode 1 / 2 (env
// MAS_SHARD_MODE, A/B): the collective on the handle's communication stream
// while `stream` solves the own level-0 blocks, the coarse levels on the
// communication stream behind it (1) or on `stream` after the solves (2, the
// round-5 form), `stream` joining before the prolongation.
int mas_shard_apply_device(mas_handle h, int rank, int world, mas_allgather_fn allgather, void* user, float* d_z4,
                           const float* d_r4, void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!d_z4 || !d_r4) return fail(h, MAS_ERR_ARG, "mas_shard_apply_device: null vector");
    if ((reinterpret_cast<uintptr_t>(d_z4) | reinterpret_cast<uintptr_t>(d_r4)) & 15)
        return fail(h, MAS_ERR_ARG, "mas_shard_apply_device: vectors must be 16-byte aligned");
    if (!allgather && world != 1) return fail(h, MAS_ERR_ARG, "mas_shard_apply_device: no allgather for world > 1");
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    if (h->rowsPending) return fail(h, MAS_ERR_STATE, kRowsPending);
    hipSetDevice(h->device);
    mas_shard sh;
    int rc = mas_shard_setup(h, rank, world, &sh);
    if (rc) return rc;
    const size_t segBytes = (size_t)sh.seg_max * 16;
    if ((rc = ensure(h, h->shardSeg, segBytes)) || (rc = ensure(h, h->shardGathered, segBytes * world))) return rc;
    if (!h->evShardDone &&
        ((rc = hip_check(h, hipEventCreateWithFlags(&h->evRestrict, hipEventDisableTiming), "event")) ||
         (rc = hip_check(h, hipEventCreateWithFlags(&h->evGathered, hipEventDisableTiming), "event")) ||
         (rc = hip_check(h, hipEventCreateWithFlags(&h->evShardDone, hipEventDisableTiming), "event"))))
        return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    // The segments (shardSeg, shardGathered, Rc / Zc) belong to the handle: a
    // call on another stream than the previous one starts after it has ended
    // (on one stream the order is implicit; the communication stream waits for
    // this call's restrict, which then follows the previous call's complete).
    if (h->shardLastStream && h->shardLastStream != s &&
        (rc = hip_check(h, hipStreamWaitEvent(s, h->evShardDone, 0), "previous apply wait")))
        return rc;
    h->shardLastStream = s;
    struct DoneMark {
        mas_handle h;
        hipStream_t s;
        ~DoneMark() { hipEventRecord(h->evShardDone, s); }
    } done{h, s};
    float* seg = P<float>(h->shardSeg);
    float* gathered = P<float>(h->shardGathered);
    if ((rc = mas_apply_shard_restrict(h, rank, world, d_r4, seg, s))) return rc;
    if (world == 1 && !allgather) {
        if ((rc = hip_check(h, hipMemcpyAsync(gathered, seg, segBytes, hipMemcpyDeviceToDevice, s), "segment copy")))
            return rc;
        return mas_apply_shard_finish(h, rank, world, gathered, d_r4, d_z4, s);
    }
    if (h->shardMode == 0) {  // inline: the collective on `stream`, then the rest behind it
        if (int e = allgather(seg, gathered, segBytes, s, user))
            return fail(h, MAS_ERR_COMM, "allgather hook returned " + std::to_string(e));
        return mas_apply_shard_finish(h, rank, world, gathered, d_r4, d_z4, s);
    }
    if (!h->commStream) {
        // modes 1 / 2 only (a queue of its own: the default inline form keeps
        // every kernel on `stream`): the coarse levels run on it beside the
        // level-0 solves, the higher priority letting their workgroups in
        // ahead of the solves' remaining ones
        int lo = 0, hi = 0;
        hipDeviceGetStreamPriorityRange(&lo, &hi);
        if ((rc = hip_check(h, hipStreamCreateWithPriority(&h->commStream, hipStreamNonBlocking, hi), "comm stream")))
            return rc;
    }
    if ((rc = hip_check(h, hipEventRecord(h->evRestrict, s), "record")) ||
        (rc = hip_check(h, hipStreamWaitEvent(h->commStream, h->evRestrict, 0), "comm wait")))
        return rc;
    if (int e = allgather(seg, gathered, segBytes, h->commStream, user))
        return fail(h, MAS_ERR_COMM, "allgather hook returned " + std::to_string(e));
    // the coarse levels on the communication stream behind the gather (1) or
    // on `stream` after the level-0 solves (2)
    const bool side = h->shardMode == 1;
    if (side && h->L > 1 && (rc = shard_coarse(h, sh, world, gathered, h->commStream))) return rc;
    if ((rc = hip_check(h, hipEventRecord(h->evGathered, h->commStream), "record")) ||
        (rc = mas_apply_shard_fine(h, rank, world, d_r4, d_z4, s)) ||
        (rc = hip_check(h, hipStreamWaitEvent(s, h->evGathered, 0), "coarse wait")))
        return rc;
    if (!side && h->L > 1 && (rc = shard_coarse(h, sh, world, gathered, s))) return rc;
    if (h->L > 1) launch_prolong(h, sh.vert_begin, sh.vert_end, reinterpret_cast<float4*>(d_z4), s);
    if (h->shardPendingEv) hipEventRecord(h->shardPendingEv[3], s);
    h->shardPendingEv = nullptr;
    h->stats.apply_calls++;
    return hip_check(h, hipGetLastError(), "shard apply");
}

// A one-process stand-in for the allgather (mas_allgather_fn): copies this
// rank's segment into its own slot of recv (user = const int* rank).  For
// per-rank timing and tests on one GPU; the other ranks' slots are left as
// they are.
int mas_allgather_loopback(const void* send, void* recv, size_t bytes, void* stream, void* user) {
    if (!send || !recv || !user || (bytes & 15)) return 1;
    const int rank = *static_cast<const int*>(user);
    // a copy kernel, as a collective's would be (hipMemcpyAsync may go to a
    // DMA engine, whose start-up latency a timing run would then measure)
    const size_t n = bytes / 16;
    if (n > 0)
        k_copy16<<<cdiv((long long)n, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const float4*>(send), reinterpret_cast<float4*>(static_cast<char*>(recv) + (size_t)rank * bytes),
            n);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
