// coarse_split.hip -- the coarse assembly of a sharded Prepare, split over the
// ranks (SURVEY §8(e) "each GPU assembles ... coarse-block partial
// contributions come from its own vertices").
//
// Every term a coarse row receives comes from that row's subtree
// (PrepareHessian .cpp:1229-1345: the CSR terms of the vertices below the
// row's node, their od and diagonal tables; AdditionalSchwarzHessian2
// .cpp:1164-1199: the contact terms of stencils touching the subtree, pushed
// to the node and its ancestors), folded in the reference's single-thread
// order restricted to that subtree.  So a rank whose vertex range holds a
// row's whole subtree folds that row bitwise by itself
// (tests/test_oracle_shard_locality.py).  Rank g owns the level-0 blocks of
// the equal split (mas_shard_plan); its level-l rows are the ids
// [anc_l(first vertex of g), anc_l(first vertex of g + 1)), which are exactly
// the rows whose subtree lies in its range when no subtree crosses a rank
// boundary -- checked on the device once per hierarchy (k_split_check; the
// BASELINE configs' equal splits at world 2 / 4 / 8 never cut one,
// scripts/dev/row_cuts.py).  Then a rank
//   * assembles only its rows: od, the coarse edge records, k_diag1, the
//     table folds and the contact records restricted to them (OwnNodes);
//   * factors its "pre" level-1 blocks (every row its own) right away;
//   * packs its rows that other ranks need -- its rows of the (at most two)
//     level-1 blocks it shares with a neighbour and every level >= 2 row --
//     into one segment (k_rows_copy), exchanged by one allgather
//     (mas_prepare_shard_rows / mas_prepare_shard_complete, or inside
//     Prepare over the handle's RCCL communicator / a registered hook);
//   * unpacks the other ranks' rows and factors the shared level-1 blocks and
//     every level >= 2 block ("post"): exactly the coarse inverses the
//     sharded apply reads (own level-1 blocks, all levels >= 2).
// When a split does cut a subtree, every rank assembles every row (the
// replicated coarse assembly of round 5) and the same exchange runs; the
// rows it delivers are then bitwise the ones already in place.
#include <algorithm>
#include <climits>
#include <string>
#include <vector>

#include "mas_internal.h"

namespace mas {

__host__ __device__ static inline int split_block(int g, int nb, int W) { return (int)((long long)g * nb / W); }

// bnd[g] = the level-1..4 ancestors of rank g's first vertex (g < W);
// bnd[W] = every level's end
__global__ __launch_bounds__(64) void k_split_bounds(int W, int nb, const int4* __restrict__ anc, int4 ends,
                                                     int4* __restrict__ bnd) {
    const int g = blockIdx.x * 64 + threadIdx.x;
    if (g > W) return;
    bnd[g] = g == W ? ends : anc[32 * (size_t)split_block(g, nb, W)];
}

// flag = 1 when some vertex's level-l ancestor (1 <= l < L) lies outside its
// rank's level-l range: then the ranges are not the subtrees of the ranks'
// vertices and the split cuts a row
__global__ __launch_bounds__(256) void k_split_check(int nV, int nb, int W, int L, const int4* __restrict__ anc,
                                                     const int4* __restrict__ bnd, int* __restrict__ flag) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= nV) return;
    const int b = v >> 5;
    const int g = min((int)(((long long)(b + 1) * W - 1) / nb), W - 1);  // largest g with split_block(g) <= b
    const int4 a = anc[v], lo = bnd[g], hi = bnd[g + 1];
    bool bad = a.x < lo.x || a.x >= hi.x;
    if (L > 2) bad |= a.y < lo.y || a.y >= hi.y;
    if (L > 3) bad |= a.z < lo.z || a.z >= hi.z;
    if (L > 4) bad |= a.w < lo.w || a.w >= hi.w;
    if (bad) atomicOr(flag, 1);
}

// Row copies between the dense coarse blocks and a segment: part p (x = first
// node, y = rows, z = first segment row, w = rows before it) moves rows
// node .. node + y - 1 (288 floats each: node n's three rows of its block,
// at dense_base + 288 n) to (toSeg) or from the segment.  A wave per row.
__global__ __launch_bounds__(256) void k_rows_copy(const int4* __restrict__ parts, int nParts, int totalRows,
                                                   float4* __restrict__ dense, float4* __restrict__ seg, int toSeg) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= totalRows) return;
    int lo = 0, hi = nParts;  // the last part starting at or before row
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (parts[mid].w <= row) lo = mid;
        else hi = mid;
    }
    const int4 p = parts[lo];
    const int k = row - p.w;
    float4* d = dense + (size_t)(p.x + k) * 72;
    float4* q = seg + (size_t)(p.z + k) * 72;
    for (int i = threadIdx.x & 63; i < 72; i += 64) {
        if (toSeg) q[i] = d[i];
        else d[i] = q[i];
    }
}

static OwnNodes every_node(const mas_context* h) {
    OwnNodes o{};
    for (int l = 0; l < 5; ++l) {
        o.lo[l] = 0;
        o.hi[l] = INT_MAX;
        o.begin[l] = l == 0 ? 0 : (l < h->L ? h->levelSize[2 * l + 1] : INT_MAX);
    }
    return o;
}

int plan_coarse_split(mas_context* h, hipStream_t s) {
    const int W = h->prepWorld, L = h->L, nb = h->nFineBlk, r = h->prepRank;
    h->own = every_node(h);
    h->rowsPending = false;
    h->splitPlanned = W > 1 && L > 1 && h->factorVariant >= 4;
    if (!h->splitPlanned) {
        h->splitClean = false;
        return MAS_OK;
    }
    int rc;
    if (h->splitHierId != h->hierId || h->splitRank != r || h->splitWorld != W) {
        // once per hierarchy and shard: the ranks' boundary ancestors and the cut check
        const size_t bytes = (size_t)(W + 1) * 16 + 16;
        if ((rc = ensure(h, h->splitDev, bytes))) return rc;
        int4* bnd = P<int4>(h->splitDev);
        int* flag = reinterpret_cast<int*>(bnd + W + 1);
        int e[4] = {0, 0, 0, 0};
        for (int l = 1; l < L && l <= 4; ++l) e[l - 1] = h->levelSize[2 * l + 1] + h->levelSize[2 * l];
        if ((rc = hip_check(h, hipMemsetAsync(flag, 0, 4, s), "memset split flag"))) return rc;
        k_split_bounds<<<cdiv(W + 1, 64), 64, 0, s>>>(W, nb, P<int4>(h->coarseTables), make_int4(e[0], e[1], e[2], e[3]),
                                                     bnd);
        k_split_check<<<cdiv(h->nV, 256), 256, 0, s>>>(h->nV, nb, W, L, P<int4>(h->coarseTables), bnd, flag);
        std::vector<int> hb((size_t)(W + 1) * 4 + 1);
        if ((rc = hip_check(h, hipMemcpyAsync(hb.data(), bnd, hb.size() * 4, hipMemcpyDeviceToHost, s), "D2H split")) ||
            (rc = hip_check(h, hipStreamSynchronize(s), "split sync")))
            return rc;
        h->splitClean = hb[(size_t)(W + 1) * 4] == 0;
        auto B = [&](int g, int l) { return hb[(size_t)g * 4 + (l - 1)]; };  // global id of the first level-l row of g
        // per rank: its rows in the exchange segment
        h->splitParts.assign(W, {});
        h->splitSegRows = 1;
        for (int g = 0; g < W; ++g) {
            std::vector<RowPart>& pt = h->splitParts[g];
            int seg = 0;
            auto add = [&](int a, int b) {
                if (b > a) {
                    pt.push_back(RowPart{a, b - a, seg});
                    seg += b - a;
                }
            };
            const int lo1 = B(g, 1), hi1 = B(g + 1, 1);
            if (hi1 > lo1) {  // its rows of level-1 blocks shared with a neighbour
                int aEnd = lo1;
                if (lo1 % 32) add(lo1, aEnd = std::min(hi1, ceil32(lo1)));
                if (hi1 % 32) add(std::max(aEnd, hi1 & ~31), hi1);
            }
            for (int l = 2; l < L; ++l) add(B(g, l), B(g + 1, l));  // every level >= 2 row
            h->splitSegRows = std::max(h->splitSegRows, seg);
        }
        // this rank's blocks: level-1 blocks all of whose rows are its own
        // (factored before the exchange), the shared ones and every level >= 2
        // block (after it)
        const int lo1 = B(r, 1), hi1 = B(r + 1, 1);
        h->splitPre.clear();
        h->splitPost.clear();
        if (hi1 > lo1) {
            const int p0 = ceil32(lo1) / 32, p1 = (hi1 & ~31) / 32;
            if (p1 > p0) h->splitPre = {p0, p1};
            if (lo1 % 32) h->splitPost.insert(h->splitPost.end(), {lo1 / 32, lo1 / 32 + 1});
            if (hi1 % 32 && (hi1 - 1) / 32 != (lo1 % 32 ? lo1 / 32 : -1))
                h->splitPost.insert(h->splitPost.end(), {(hi1 - 1) / 32, (hi1 - 1) / 32 + 1});
        }
        if (L > 2) h->splitPost.insert(h->splitPost.end(), {h->levelSize[5] / 32, h->nBlk});
        // device part table: the pack parts (this rank's), then the unpack
        // parts (every other rank's, segment rows relative to the gathered buffer)
        std::vector<int4> tab;
        auto push = [&](const RowPart& p, int segBase, int& rows) {
            tab.push_back(make_int4(p.node0, p.count, segBase + p.seg0, rows));
            rows += p.count;
        };
        h->splitPackRows = h->splitUnpackRows = 0;
        for (const RowPart& p : h->splitParts[r]) push(p, 0, h->splitPackRows);
        h->splitPackParts = (int)tab.size();
        for (int g = 0; g < W; ++g)
            if (g != r)
                for (const RowPart& p : h->splitParts[g]) push(p, g * h->splitSegRows, h->splitUnpackRows);
        h->splitUnpackParts = (int)tab.size() - h->splitPackParts;
        if (tab.empty()) tab.push_back(make_int4(0, 0, 0, 0));
        if ((rc = ensure(h, h->splitPartsDev, tab.size() * 16)) ||
            (rc = hip_check(h, hipMemcpyAsync(h->splitPartsDev.p, tab.data(), tab.size() * 16, hipMemcpyHostToDevice,
                                              s), "H2D split parts")) ||
            (rc = hip_check(h, hipStreamSynchronize(s), "split parts sync")))
            return rc;
        h->splitHierId = h->hierId;
        h->splitRank = r;
        h->splitWorld = W;
        // the own ranges, kept with the plan
        std::vector<int>& keep = h->splitBnd;
        keep.assign(10, 0);
        for (int l = 1; l < L && l <= 4; ++l) {
            keep[2 * l] = B(r, l);
            keep[2 * l + 1] = B(r + 1, l);
        }
    }
    if (h->splitClean) {
        h->own.lo[0] = 32 * split_block(r, nb, W);
        h->own.hi[0] = std::min(32 * split_block(r + 1, nb, W), h->nV);
        for (int l = 1; l < L && l <= 4; ++l) {
            h->own.lo[l] = h->splitBnd[2 * l];
            h->own.hi[l] = h->splitBnd[2 * l + 1];
        }
    }
    return MAS_OK;
}

int pack_coarse_rows(mas_context* h, hipStream_t s) {
    int rc;
    if ((rc = ensure(h, h->prepSeg, (size_t)h->splitSegRows * 1152))) return rc;
    if (h->splitPackRows > 0)
        k_rows_copy<<<cdiv(h->splitPackRows, 4), 256, 0, s>>>(P<int4>(h->splitPartsDev), h->splitPackParts,
                                                             h->splitPackRows, reinterpret_cast<float4*>(dense_base(h)),
                                                             P<float4>(h->prepSeg), 1);
    h->rowsPending = true;
    return hip_check(h, hipGetLastError(), "pack coarse rows");
}

int complete_coarse_rows(mas_context* h, const float* gathered, hipStream_t s) {
    int rc;
    if (h->splitUnpackRows > 0)
        k_rows_copy<<<cdiv(h->splitUnpackRows, 4), 256, 0, s>>>(
            P<int4>(h->splitPartsDev) + h->splitPackParts, h->splitUnpackParts, h->splitUnpackRows,
            reinterpret_cast<float4*>(dense_base(h)), reinterpret_cast<float4*>(const_cast<float*>(gathered)), 0);
    if ((rc = hip_check(h, hipGetLastError(), "unpack coarse rows"))) return rc;
    for (size_t i = 0; i + 1 < h->splitPost.size(); i += 2)
        if ((rc = factor_blocks(h, h->splitPost[i], h->splitPost[i + 1], s))) return rc;
    h->rowsPending = false;
    return MAS_OK;
}

}  // namespace mas

using namespace mas;

extern "C" {

int mas_set_prepare_allgather(mas_handle h, mas_allgather_fn fn, void* user) {
    if (!h) return MAS_ERR_ARG;
    h->prepAllgather = fn;
    h->prepAllgatherUser = user;
    return MAS_OK;
}

int mas_prepare_shard_rows(mas_handle h, void** d_seg, size_t* seg_bytes) {
    if (!h || !d_seg || !seg_bytes) return MAS_ERR_ARG;
    if (!h->rowsPending)
        return fail(h, MAS_ERR_STATE, "mas_prepare_shard_rows: no coarse rows pending (not a sharded Prepare, "
                                      "or its exchange already ran)");
    *d_seg = h->prepSeg.p;
    *seg_bytes = (size_t)h->splitSegRows * 1152;
    return MAS_OK;
}

int mas_prepare_shard_complete(mas_handle h, const void* d_gathered, void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!d_gathered) return fail(h, MAS_ERR_ARG, "mas_prepare_shard_complete: null gathered buffer");
    if (!h->rowsPending) return fail(h, MAS_ERR_STATE, "mas_prepare_shard_complete: no coarse rows pending");
    hipSetDevice(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    ScopedEvents ev;
    if (!ev.ok()) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    hipEventRecord(ev.e[0], s);
    int rc = complete_coarse_rows(h, static_cast<const float*>(d_gathered), s);
    if (rc) return rc;
    hipEventRecord(ev.e[1], s);
    if ((rc = hip_check(h, hipStreamSynchronize(s), "complete sync"))) return rc;
    float ms = 0.f;
    hipEventElapsedTime(&ms, ev.e[0], ev.e[1]);
    h->stats.prepare_complete_ms = ms;
    return report_pivots(h, s);
}

}  // extern "C"
