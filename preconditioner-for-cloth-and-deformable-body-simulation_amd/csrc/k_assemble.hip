// k_assemble.hip -- dense 96x96 subdomain blocks from the CSR Hessian and the
// contact stencils (PrepareCollisionHessian .cpp:1164-1227, PrepareHessian
// .cpp:1229-1345).
//
// Layout: block b is a row-major 96x96 fp32 matrix at dense + 9216 b; the 3x3
// entry (row node x, column node y) of block b holds what the reference keeps
// in m_hessian32[y][32 b + x] (.cpp:1363-1375).
//
// Why the summation order is reproduced exactly: inside a cluster the spring
// terms of the diagonal and off-diagonal blocks cancel (K - K), so a coarse
// entry is a small difference of large fp32 sums, and coarse blocks are badly
// conditioned (~1e5).  A different association moves z by ~1e-4 relative.
// Every sum below is therefore a strict left fold in the reference's
// single-thread order (vertex order, then ELL neighbour order; hash-map pushes
// in node-id order, see oracle/mas_oracle.c), computed in parallel over
// independent targets:
//   k_level0_block  one workgroup per level-0 block, per vertex: block-0
//                 diagonal and same-bank entries (single writer, tile in LDS,
//                 block written whole), od(u) = diag + additional + level-0
//                 entries (oldDiagonal, .cpp:1270-1298), count of coarse edges
//   k_records     coarse edges (u, k) with first common-bank level 1..L-1, in
//                 (u, k) order
//   k_fold_runs   per coarse entry (row, col), (key, mat)
//                 pairs sorted stably by key = (row, col): entry += mat in
//                 (u, k) order (short runs: a thread; long runs: a wave)
//   k_diag1       one thread per level-0 bank: diag(anc1(u)) += od(u) (.cpp:1309-1312)
//   k_term_*, k_table_fold  the diagTable fold (.cpp:1299-1343) per level-l
//                 node (l >= 2): over member vertices in order, level-(l-1)
//                 edge mats and (l = 2) od(u); then the children's tables in
//                 id order; diag += table.  Terms are flattened in parallel,
//                 then folded strictly left by one wave per node.
// Contact stencils (only present in the contact configuration) are folded in
// the reference's single-thread order as well (below, before k_contact_*).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <type_traits>

#include "mas_internal.h"
#include "radix.h"

namespace mas {

static int bit_width(unsigned x) { return x ? 32 - __builtin_clz(x) : 0; }

// block-entry sort keys (RecKey below): 32 bits, enough for 2^27 nodes
using EntryKey = unsigned;

struct EdgeRec {
    int lam;  // first common-bank level, 1..L-1
    int row;  // anc_lam(u) (global node id)
    int col;  // anc_lam(v)
    int mat;  // index into off9
};

__device__ __forceinline__ float* entry(float* dense, unsigned rowNode, unsigned colNode) {
    return dense + (size_t)(rowNode >> 5) * kDenseFloats + (3 * (rowNode & 31)) * 96 + 3 * (colNode & 31);
}

__device__ __forceinline__ int climb(const int* __restrict__ gn, int L, unsigned& my, unsigned& ot) {
    int level = 0;
    while ((my >> 5) != (ot >> 5) && level < L) {
        level++;
        my = (unsigned)gn[my];
        ot = (unsigned)gn[ot];
    }
    return level;
}

// 3x3 stored column-major in the inputs; entries of the dense block are row-major.
__device__ __forceinline__ void add_colmajor(float* e, const float* __restrict__ m) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) e[r * 96 + c] = __fadd_rn(e[r * 96 + c], m[c * 3 + r]);
}

// ---------------------------------------------------------------------------
// contacts (deterministic, the reference's single-thread order)
// ---------------------------------------------------------------------------
//
// PrepareCollisionHessian (.cpp:1201-1227) runs stencil by stencil: first
// additional[idx[it]] += h w_it^2 for every vertex of the stencil, then per
// pair (a, b) in order AdditionalSchwarzHessian2 (.cpp:1164-1199): at the
// first level where both ids share a bank, block entry (my, ot) += t then
// (ot, my) += t (t = w_a w_b h, the same matrix both times), and below the top
// level additional[parent] += t for both parents (2t when they coincide).
// PrepareHessian (.cpp:1229-1345) then pushes every coarse additional[x], x
// ascending, into x's own diagonal and every ancestor's, and only then adds
// the CSR terms.  The reference does the contact sums with float atomics
// (order-free with threads, B-10); at CPU_THREAD_NUM = 1 they are these
// ordered left folds, which is what is computed here:
//   k_contact_count / _write  per stencil, its records in stencil order: a
//                 block-entry record (key (my, ot)) per pair half, an
//                 additional record (key node) per w^2 term and parent term;
//                 values stored column-major, 9 floats
//   radix sort    stable by key, so a key's records stay in stencil order
//   fine entries  (rows < begin_1) are added by k_level0_block into its LDS
//                 tile before the CSR terms
//   coarse entries, additional rows: k_fold_runs_t folds each key's run left
//                 from the zeroed target
//   pushes        per coarse node x with an additional row: records (target,
//                 x) for x and each ancestor, sorted stably by target (x
//                 ascending), folded into the target's diagonal
// Contact-free inputs skip all of it.

// The contact terms (.cpp:1190,1208-1223), column-major 3x3; pinned bit for
// bit against the reference's own headers (mas_dev_contact_terms,
// tests/test_gpu_ref_pinned.py; fixtures tests/golden/ref_contact.npz).
__device__ __forceinline__ void contact_outer(const float* dir, float stiff, float (&hm)[9]) {
    // OuterProduct(d, d * stiff), SeMatrix.h:352-363; column-major: hm[c * 3 + r] = d_r (d_c stiff)
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) hm[c * 3 + r] = __fmul_rn(dir[r], __fmul_rn(dir[c], stiff));
}
__device__ __forceinline__ void contact_h(const DevStencil& s, float (&hm)[9]) { contact_outer(s.dir, s.stiff, hm); }
// hessian * Math::Square(w), SeMath.h:98 / SeMatrix.h:741
__device__ __forceinline__ void contact_self(const float (&hm)[9], float w, float* out) {
    const float w2 = __fmul_rn(w, w);
    for (int e = 0; e < 9; ++e) out[e] = __fmul_rn(hm[e], w2);
}
// w_a * w_b * hessian, SeMatrix.h:977
__device__ __forceinline__ void contact_pair(const float (&hm)[9], float wa, float wb, float (&t)[9]) {
    const float ww = __fmul_rn(wa, wb);
    for (int e = 0; e < 9; ++e) t[e] = __fmul_rn(ww, hm[e]);
}
// AdditionalSchwarzHessian2's hessian * 2.0f (.cpp:1190)
__device__ __forceinline__ float contact_double(float t) { return __fmul_rn(t, 2.0f); }

// mas_dev_contact_terms: the terms of n stencils (orc_contact_terms layout, 234 floats each)
__global__ __launch_bounds__(64) void k_contact_terms(const float* __restrict__ dir3, const float* __restrict__ stiff,
                                                      const float* __restrict__ w5, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float hm[9], t[9];
    contact_outer(dir3 + 3 * (size_t)i, stiff[i], hm);
    float* o = out + 234 * (size_t)i;
    for (int e = 0; e < 9; ++e) o[e] = hm[e];
    const float* w = w5 + 5 * (size_t)i;
    for (int it = 0; it < 5; ++it) contact_self(hm, w[it], o + 9 + 9 * it);
    for (int a = 0, p = 0; a < 5; ++a)
        for (int b = a + 1; b < 5; ++b, ++p) {
            contact_pair(hm, w[a], w[b], t);
            for (int e = 0; e < 9; ++e) {
                o[54 + 9 * p + e] = t[e];
                o[144 + 9 * p + e] = contact_double(t[e]);
            }
        }
}

// A stencil's vertices at every level, from the per-vertex ancestor table
// (coarseTables: the level-1..4 ancestors, AggregationKernel .cpp:1119-1147):
// five independent 16-byte loads instead of the dependent goingNext walk of
// each pair (AdditionalSchwarzHessian2's while loop, .cpp:1171-1176).
// nd[k][l] = vertex k's node at level l (l <= min(L - 1, 4)).
__device__ __forceinline__ void stencil_nodes(const DevStencil& s, const int4* __restrict__ anc, unsigned (&nd)[5][5]) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int4 a = k < s.n ? anc[s.idx[k]] : make_int4(0, 0, 0, 0);
        nd[k][0] = (unsigned)s.idx[k];
        nd[k][1] = (unsigned)a.x;
        nd[k][2] = (unsigned)a.y;
        nd[k][3] = (unsigned)a.z;
        nd[k][4] = (unsigned)a.w;
    }
}
// the first level where vertices x and y share a bank (L: none); my / ot their nodes there
__device__ __forceinline__ int climb_nodes(const unsigned (&nd)[5][5], int x, int y, int L, unsigned& my,
                                           unsigned& ot) {
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        if (l >= L) break;
        my = nd[x][l];
        ot = nd[y][l];
        if ((my >> 5) == (ot >> 5)) return l;
    }
    return L;
}

// counts: dCnt[i] block-entry records, aCnt[i] additional records of stencil i
// skip0: without the level-0 records (block entries of same-bank pairs, the
// w^2 additional rows), which run_level0_early built already
// own: the rows this Prepare assembles (every row unless the coarse
// assembly is split over shards, coarse_split.hip): a record whose target row
// (block entry: its row node; additional: its node) is another rank's is not
// written
__global__ __launch_bounds__(256) void k_contact_count(const DevStencil* __restrict__ st, int n,
                                                       const int4* __restrict__ anc, int L, int* __restrict__ dCnt,
                                                       int* __restrict__ aCnt, bool skip0, OwnNodes own) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) {  // closes the exclusive scans
        dCnt[n] = aCnt[n] = 0;
        return;
    }
    const DevStencil s = st[i];
    unsigned nd[5][5];
    stencil_nodes(s, anc, nd);
    int d = 0, a = 0;
    if (!skip0)
        for (int it = 0; it < s.n; ++it) a += own.own((unsigned)s.idx[it]);
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
        for (int y = 1; y < 5; ++y) {
            if (y <= x || y >= s.n) continue;
            unsigned my = 0, ot = 0;
            const int level = climb_nodes(nd, x, y, L, my, ot);
            if (level >= L) continue;
            if (level > 0 || !skip0) d += (int)own.own(my) + (int)own.own(ot);
            if (level < L - 1) {
                const unsigned pm = nd[x][level + 1], po = nd[y][level + 1];
                a += pm == po ? (int)own.own(pm) : (int)own.own(pm) + (int)own.own(po);
            }
        }
    dCnt[i] = d;
    aCnt[i] = a;
}

// The records of stencil i at dOff[i] / aOff[i], in the reference's order;
// keys: block entry my * 32 + (ot & 31) (RecKey with begin1 = 0: the pair
// shares a bank at its level), additional node id.
__global__ __launch_bounds__(256) void k_contact_write(const DevStencil* __restrict__ st, int n,
                                                       const int4* __restrict__ anc, int L,
                                                       const int* __restrict__ dOff, const int* __restrict__ aOff,
                                                       EntryKey* __restrict__ dKeys, int* __restrict__ dIds,
                                                       float* __restrict__ dVal, int* __restrict__ dEnt,
                                                       unsigned* __restrict__ aKeys, int* __restrict__ aIds,
                                                       float* __restrict__ aVal, bool skip0, unsigned kb,
                                                       OwnNodes own) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DevStencil s = st[i];
    unsigned nd[5][5];
    stencil_nodes(s, anc, nd);
    float hm[9];
    contact_h(s, hm);
    int d = dOff[i], a = aOff[i];
    for (int it = 0; it < s.n && !skip0; ++it) {  // .cpp:1214-1217: additional[idx] += h w^2
        if (!own.own((unsigned)s.idx[it])) continue;
        aKeys[a] = (unsigned)s.idx[it];
        aIds[a] = a;
        contact_self(hm, s.w[it], aVal + 9 * (size_t)a);
        ++a;
    }
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
        for (int y = 1; y < 5; ++y) {
            if (y <= x || y >= s.n) continue;
            unsigned my = 0, ot = 0;
            const int level = climb_nodes(nd, x, y, L, my, ot);
            if (level >= L) continue;
            float t[9];
            contact_pair(hm, s.w[x], s.w[y], t);
            if (level > 0 || !skip0) {
                // pDenseHessian[ot % bank][my] (entry row my, column ot), then [my % bank][ot];
                // rows relative to kb (begin_1 when only coarse records are written)
                const unsigned rows[2] = {my, ot}, cols[2] = {ot, my};
                for (int hf = 0; hf < 2; ++hf) {
                    if (!own.own(rows[hf])) continue;
                    dKeys[d] = (EntryKey)(((rows[hf] - kb) << 5) | (cols[hf] & 31u));
                    dIds[d] = d;
                    dEnt[d] = (int)(((rows[hf] & 31u) << 5) | (cols[hf] & 31u));  // FineAsm::cent (level-0 records)
                    for (int e = 0; e < 9; ++e) dVal[9 * (size_t)d + e] = t[e];
                    ++d;
                }
            }
            if (level < L - 1) {
                const unsigned pm = nd[x][level + 1], po = nd[y][level + 1];
                if (pm == po) {
                    if (own.own(pm)) {
                        aKeys[a] = pm - kb;
                        aIds[a] = a;
                        for (int e = 0; e < 9; ++e) aVal[9 * (size_t)a + e] = contact_double(t[e]);
                        ++a;
                    }
                } else {
                    const unsigned ps[2] = {pm, po};
                    for (int hf = 0; hf < 2; ++hf) {
                        if (!own.own(ps[hf])) continue;
                        aKeys[a] = ps[hf] - kb;
                        aIds[a] = a;
                        for (int e = 0; e < 9; ++e) aVal[9 * (size_t)a + e] = t[e];
                        ++a;
                    }
                }
            }
        }
}

// Level-0 records alone (run_level0_early): per stencil the block-entry
// records of its same-bank pairs (level 0 of k_contact_write's loop: same
// order, same values) at dOff[i] -- keyed by their level-0 block, with the
// entry inside the block in dEnt (the fused kernel adds a block's records in
// order, FineAsm) -- and its w^2 additional records at the fixed slots
// kA0 i + it (slots past s.n keep the sentinel key).  No level ids are
// needed: a pair is a level-0 entry iff both vertices share a level-0 bank.
constexpr int kA0 = 5;  // most vertices per stencil (EF)
// The early path's fills and the level-0 record counts in one launch (they
// were five hipMemsetAsync calls and a count kernel, each a host API call on
// the early path's critical path): add0 zeroed, the record and row keys set
// to the sentinel (all ones) and their ids to 0, and threads i <= n count
// stencil i's same-bank records, two per pair (n < 0: fills only).
__global__ __launch_bounds__(256) void k_contact0_init(const DevStencil* __restrict__ st, int n, int* __restrict__ dCnt,
                                                       float4* __restrict__ add0, size_t nAdd4,
                                                       EntryKey* __restrict__ c0Keys, int* __restrict__ c0Ids,
                                                       size_t ubD, unsigned* __restrict__ a0Keys,
                                                       int* __restrict__ a0Ids, size_t ubA) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, T = (size_t)gridDim.x * blockDim.x;
    if (n >= 0 && i <= (size_t)n) {
        if (i == (size_t)n) {
            dCnt[n] = 0;
        } else {
            const DevStencil s = st[i];
            int d = 0;
            for (int x = 0; x < s.n; ++x)
                for (int y = x + 1; y < s.n; ++y) d += ((unsigned)s.idx[x] >> 5) == ((unsigned)s.idx[y] >> 5) ? 2 : 0;
            dCnt[i] = d;
        }
    }
    for (size_t q = i; q < nAdd4; q += T) add0[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t q = i; q < ubD; q += T) {
        c0Keys[q] = ~(EntryKey)0;
        c0Ids[q] = 0;
    }
    for (size_t q = i; q < ubA; q += T) {
        a0Keys[q] = ~0u;
        a0Ids[q] = 0;
    }
}

__global__ __launch_bounds__(256) void k_contact0_write(const DevStencil* __restrict__ st, int n,
                                                        const int* __restrict__ dOff, EntryKey* __restrict__ dKeys,
                                                        int* __restrict__ dIds, float* __restrict__ dVal,
                                                        int* __restrict__ dEnt, unsigned* __restrict__ aKeys,
                                                        int* __restrict__ aIds, float* __restrict__ aVal) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DevStencil s = st[i];
    float hm[9];
    contact_h(s, hm);
    for (int it = 0; it < s.n; ++it) {  // .cpp:1214-1217: additional[idx] += h w^2
        const int a = kA0 * i + it;
        aKeys[a] = (unsigned)s.idx[it];
        aIds[a] = a;
        contact_self(hm, s.w[it], aVal + 9 * (size_t)a);
    }
    int d = dOff[i];
    for (int x = 0; x < s.n; ++x)
        for (int y = x + 1; y < s.n; ++y) {
            const unsigned my = (unsigned)s.idx[x], ot = (unsigned)s.idx[y];
            if ((my >> 5) != (ot >> 5)) continue;
            float t[9];
            contact_pair(hm, s.w[x], s.w[y], t);
            dKeys[d] = dKeys[d + 1] = (EntryKey)(my >> 5);  // the level-0 block
            dEnt[d] = (int)(((my & 31u) << 5) | (ot & 31u));
            dEnt[d + 1] = (int)(((ot & 31u) << 5) | (my & 31u));
            dIds[d] = d;
            dIds[d + 1] = d + 1;
            for (int e = 0; e < 9; ++e) dVal[9 * (size_t)d + e] = dVal[9 * (size_t)(d + 1) + e] = t[e];
            d += 2;
        }
}

// Per level-0 block, the range of its contact block-entry records in the
// sorted array (rows < begin_1 sort first): fineOff[b] .. fineOff[b + 1].
__global__ __launch_bounds__(256) void k_contact_fine_bounds(int nD, int B, int begin1, int nFineBlk,
                                                             const EntryKey* __restrict__ keys,
                                                             int* __restrict__ fineOff) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > nD) return;
    auto blockOf = [&](int q) {
        if (q >= nD) return nFineBlk;
        const unsigned row = (unsigned)(keys[q] >> B);
        return row < (unsigned)begin1 ? (int)(row >> 5) : nFineBlk;
    };
    const int b = blockOf(j), prev = j == 0 ? -1 : blockOf(j - 1);
    for (int k = prev + 1; k <= b; ++k) fineOff[k] = j;  // blocks (prev, b] start here
}

// The same from keys that are level-0 block ids (run_level0_early; the
// sentinel, all ones, and any key >= nFineBlk count as past the last block).
__global__ __launch_bounds__(256) void k_block_bounds(int n, int nFineBlk, const EntryKey* __restrict__ keys,
                                                      int* __restrict__ off) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    auto blockOf = [&](int q) { return q >= n || keys[q] >= (EntryKey)nFineBlk ? nFineBlk : (int)keys[q]; };
    const int b = blockOf(j), prev = j == 0 ? -1 : blockOf(j - 1);
    for (int k = prev + 1; k <= b; ++k) off[k] = j;  // blocks (prev, b] start here
}

// push records of coarse node x (a run start in the sorted additional keys):
// targets x, gn[x], ... below total
// (keys relative to kb: node = key + kb; push keys written the same way)
__global__ __launch_bounds__(256) void k_push_count(int nA, int begin1, int tc, const unsigned* __restrict__ aKeys,
                                                    unsigned kb, const int* __restrict__ gn, int* __restrict__ pCnt) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > nA) return;
    int c = 0;
    if (j < nA) {
        const unsigned x = aKeys[j] + kb;
        if (x >= (unsigned)begin1 && (j == 0 || aKeys[j - 1] != aKeys[j]))
            for (int t = (int)x; t < tc; t = gn[t]) ++c;
    }
    pCnt[j] = c;
}

__global__ __launch_bounds__(256) void k_push_write(int nA, int begin1, int tc, const unsigned* __restrict__ aKeys,
                                                    unsigned kb, const int* __restrict__ gn,
                                                    const int* __restrict__ pOff, unsigned* __restrict__ pKeys,
                                                    int* __restrict__ pIds) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nA) return;
    const unsigned x = aKeys[j] + kb;
    if (x < (unsigned)begin1 || (j > 0 && aKeys[j - 1] == aKeys[j])) return;
    int w = pOff[j];
    for (int t = (int)x; t < tc; t = gn[t], ++w) {
        pKeys[w] = (unsigned)t - kb;
        pIds[w] = (int)x;  // the pushed value: additional row x (row-major)
    }
}

// ---------------------------------------------------------------------------
// CSR Hessian (deterministic, reference order)
// ---------------------------------------------------------------------------

// Level-0 assembly, one 64-lane workgroup per level-0 block; per vertex
// (.cpp:1257-1297): diag + additional on its diagonal, every same-bank CSR
// neighbour into its row, the running sum od(v) = diag + additional + those
// neighbour blocks (the vertex's part of its level-1 diagonal, .cpp:1275-1282),
// and the count of its coarse edge records.  The block's 96x96 tile is built
// in LDS (vertex n adds only into its own rows 3n..3n+2, as in the
// reference's owner loop) and written out whole
// with coalesced stores, so the fine part of the dense buffer needs no memset
// and no read-modify-write of scattered 3x3 entries (k_level0 moved 5 GB per
// launch at 1M for 1.2 GB of blocks as a thread-per-vertex kernel).  The tile
// starts from zeros; contact pair terms are added afterwards (see
// k_collision_hessian).  Measured alternatives: no LDS, the wave stores the
// zero block, drains, then each lane stores its 3x3 entries straight to HBM --
// 749 vs 338 us at 1M (the 12-byte scattered stores are partial-line writes);
// persistent workgroups (4 per CU) looping over blocks -- 355 us.
// Contact block entries of this block (sorted, each entry's records in
// stencil order) are added to the zero tile first, lane e < 9 owning
// component e of every entry -- the reference adds PrepareCollisionHessian's
// terms before PrepareHessian's (.cpp:88-97).
struct FineContacts {
    const EntryKey* keys;  // sorted block-entry keys row * 32 + (col & 31) (RecKey)
    const int* ids;                  // record index -> 9 column-major floats in val
    const float* val;
    const int* off;                  // per level-0 block: first record (nFineBlk + 1)
    int B;
};

__global__ __launch_bounds__(64) void k_level0_block(int nV, int L, const int* __restrict__ s2o,
                                                     const int* __restrict__ nbrNum, const int* __restrict__ nbr,
                                                     const float* __restrict__ diag9,
                                                     const float* __restrict__ off9, const int* __restrict__ ranges,
                                                     const float* __restrict__ additional,
                                                     float* __restrict__ dense, float* __restrict__ od,
                                                     int* __restrict__ recCnt, FineContacts fc, int fb0, int fb1) {
    __shared__ __attribute__((aligned(16))) float tile[kDenseFloats];
    const int lane = threadIdx.x;
    const size_t blk = blockIdx.x;
    // a sharded Prepare builds only its own blocks' tiles; od and the record
    // counts (the coarse assembly's inputs) come from every block
    const bool tiles = (int)blk >= fb0 && (int)blk < fb1;  // workgroup-uniform
    float4* gblk = reinterpret_cast<float4*>(dense + blk * kDenseFloats);
    float4* t4 = reinterpret_cast<float4*>(tile);
    if (tiles)
        for (int q = lane; q < kDenseFloats / 4; q += 64) t4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (tiles && fc.off && lane < 9) {
        const int r = lane / 3, c = lane % 3;
        const int j1 = fc.off[blk + 1];
        for (int j = fc.off[blk]; j < j1; ++j) {
            const EntryKey k = fc.keys[j];
            const unsigned row = (unsigned)(k >> fc.B), col = (unsigned)(k & ((1ull << fc.B) - 1));
            float* e = tile + (3 * (row & 31) + r) * 96 + 3 * (col & 31) + c;
            *e = __fadd_rn(*e, fc.val[9 * (size_t)fc.ids[j] + c * 3 + r]);
        }
    }
    __syncthreads();
    const int n = lane;
    const int v = (int)blk * 32 + n;
    if (n < 32 && v < nV) {
        const int o = s2o[v];
        float acc[9];
        const float* d = diag9 + 9 * (size_t)o;
        const float* ad = additional + 9 * (size_t)v;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) acc[r * 3 + c] = __fadd_rn(d[c * 3 + r], ad[r * 3 + c]);  // .cpp:1270
        float* e = tile + (3 * n) * 96 + 3 * n;  // .cpp:1271
        if (tiles)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) e[r * 96 + c] = __fadd_rn(e[r * 96 + c], acc[r * 3 + c]);
        const int num = nbrNum[v];
        const size_t base = (size_t)ranges[o];
        int cnt = 0;
        // neighbours in chunks of 4 with every load of the chunk issued first
        // (the loop is latency-bound: one wave per block, 32 active lanes)
        for (int k0 = 1; k0 < num; k0 += 4) {
            unsigned ot[4];
            float mm[4][9];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = k0 + j;
                ot[j] = k < num ? (unsigned)nbr[(size_t)k * nV + v] : 0xffffffffu;
                const float* m = off9 + 9 * (base + (k < num ? k - 1 : 0));
#pragma unroll
                for (int q = 0; q < 9; ++q) mm[j][q] = m[q];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (k0 + j >= num) break;
                if ((ot[j] >> 5) == ((unsigned)v >> 5)) {  // same bank: level 0
                    float* t = tile + (3 * n) * 96 + 3 * (ot[j] & 31);
                    if (tiles)
                        for (int r = 0; r < 3; ++r)
                            for (int c = 0; c < 3; ++c) t[r * 96 + c] = __fadd_rn(t[r * 96 + c], mm[j][c * 3 + r]);
                    for (int r = 0; r < 3; ++r)
                        for (int c = 0; c < 3; ++c) acc[r * 3 + c] = __fadd_rn(acc[r * 3 + c], mm[j][c * 3 + r]);
                } else {
                    cnt++;  // a coarse edge record (k_records finds its level; level >= L: a dead record)
                }
            }
        }
        for (int q = 0; q < 9; ++q) od[9 * (size_t)v + q] = acc[q];
        recCnt[v] = cnt;
    }
    __syncthreads();
    if (tiles)
        for (int q = lane; q < kDenseFloats / 4; q += 64) gblk[q] = t4[q];
}

// od(v) and the coarse record count of every vertex, one thread per vertex:
// k_level0_block's per-vertex sums without the tile (the fused variant builds
// the tiles inside k_factor_fused).  od = diag + additional, then the
// same-bank neighbour blocks in ELL order (.cpp:1270-1282).
__global__ __launch_bounds__(256) void k_od(FineAsm a, float* __restrict__ od, int* __restrict__ recCnt, int v0,
                                            int v1) {
    const int v = v0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= v1) return;
    const int o = a.s2o[v];
    float acc[9];
    const float* d = a.diag9 + 9 * (size_t)o;
    const float* ad = a.additional + 9 * (size_t)v;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) acc[r * 3 + c] = __fadd_rn(d[c * 3 + r], ad[r * 3 + c]);
    const int num = a.nbrNum[v];
    const size_t base = (size_t)a.ranges[o];
    int cnt = 0;
    for (int k0 = 1; k0 < num; k0 += 4) {  // every load of a chunk first; cross-bank blocks are not read
        bool same[4];
        float mm[4][9];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            const unsigned ot = k < num ? (unsigned)a.nbr[(size_t)k * a.nV + v] : 0xffffffffu;
            same[j] = k < num && (ot >> 5) == ((unsigned)v >> 5);
            cnt += k < num && !same[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float* m = a.off9 + 9 * (base + k0 + j - 1);
#pragma unroll
            for (int q = 0; q < 9; ++q) mm[j][q] = same[j] ? m[q] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (same[j])
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) acc[r * 3 + c] = __fadd_rn(acc[r * 3 + c], mm[j][c * 3 + r]);
    }
    for (int q = 0; q < 9; ++q) od[9 * (size_t)v + q] = acc[q];
    recCnt[v] = cnt;
}

// k_od with G lanes per vertex (G >= the largest neighbour count): lane j
// loads ELL slot 1 + j's block (when it is a same-bank neighbour) so every
// load of a vertex is in flight at once -- the thread-per-vertex form waits a
// dependent chain per 4 slots (217 us at 1M + contacts, ~1.3 TB/s).  The
// blocks go through LDS, then lane q of the vertex's group folds entry q over
// the slots in ELL order (the same left fold, skipping cross-bank slots:
// bitwise equal to k_od).
template <int G>
__global__ __launch_bounds__(256) void k_od_lanes(FineAsm a, float* __restrict__ od, int* __restrict__ recCnt, int v0,
                                                  int v1) {
    constexpr int VPW = 64 / G;  // vertices per wave
    // lane j folds entries j and j + G: all nine only when G >= 8
    static_assert(G >= 8 && 2 * G >= 9 && 64 % G == 0, "k_od_lanes: 8, 16, 32 or 64 lanes per vertex");
    __shared__ float stg[4][64][10];  // [wave][lane][entry], padded row
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = v0 + t / G, j = t % G, g0 = lane & ~(G - 1);
    const bool vin = v < v1;
    const int vc = vin ? v : 0;
    // every load issued as early as its address allows: the s2o -> ranges ->
    // off9 chain, and beside it nbr, the vertex's diagonal (after s2o) and
    // additional rows, which the folding lanes need after the barrier (a
    // fourth dependent round trip when they were loaded there; beside the
    // fused kernel this kernel runs on the reserved CUs and is bound by those
    // round trips)
    const int o = vin ? a.s2o[v] : 0;
    const int num = vin ? a.nbrNum[v] : 0;
    const int k = 1 + j;
    const unsigned ot = vin && k < num ? (unsigned)a.nbr[(size_t)k * a.nV + v] : 0xffffffffu;
    // lane j folds entries j (and j + G when G = 8: lane 0 also folds entry 8)
    float dd[2], aa[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = j + G * i, r = q / 3, c = q % 3;
        const bool fold = q < 9;
        dd[i] = fold ? a.diag9[9 * (size_t)o + c * 3 + r] : 0.f;
        aa[i] = fold ? a.additional[9 * (size_t)vc + r * 3 + c] : 0.f;
    }
    const bool has = vin && k < num;
    const bool same = has && (ot >> 5) == ((unsigned)v >> 5);
    const unsigned long long bs = __ballot(has && !same);
    if (vin && j == 0) recCnt[v] = __popcll((bs >> g0) & (G == 64 ? ~0ull : ((1ull << G) - 1)));
    float m[9];
    if (same) {
        const float* src = a.off9 + 9 * ((size_t)a.ranges[o] + k - 1);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) m[r * 3 + c] = src[c * 3 + r];
    } else {
#pragma unroll
        for (int q = 0; q < 9; ++q) m[q] = 0.f;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) stg[w][lane][q] = m[q];
    stg[w][lane][9] = same ? 1.f : 0.f;
    __syncthreads();
    if (!vin) return;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = j + G * i;
        if (q >= 9) break;
        float acc = __fadd_rn(dd[i], aa[i]);
        for (int s = 0; s < G && 1 + s < num; ++s)
            if (stg[w][g0 + s][9] != 0.f) acc = __fadd_rn(acc, stg[w][g0 + s][q]);
        od[9 * (size_t)v + q] = acc;
    }
    (void)VPW;
}

// Entry keys.  A record's row and column nodes always share a bank (the
// climb stops at the first level where they do), so an entry is its row id
// relative to begin1 and the column's lane: key = (row - begin1) * 32 +
// (col & 31), B + 5 bits (B = bit width of the node count above begin1: 16 at
// 1M, 18 at 4M) instead of 2B -- the stable radix sort runs 3 passes instead
// of 4 (1M) and 5 (4M), over 32-bit keys (half the bytes per pass of the
// 64-bit ones).  A dead record's key has all B + 5 bits set, above every live
// key.  Contact block entries use the same form with begin1 = 0.
struct RecKey {
    int begin1, B;
    static constexpr int kLaneBits = 5;
    __host__ __device__ int bits() const { return B + kLaneBits; }
    __host__ __device__ EntryKey dead() const { return bits() >= 32 ? ~0u : (1u << bits()) - 1; }
    __device__ EntryKey pack(unsigned row, unsigned col) const { return ((row - begin1) << kLaneBits) | (col & 31u); }
    __device__ unsigned row(EntryKey k) const { return (k >> kLaneBits) + begin1; }
    __device__ unsigned col(EntryKey k) const { return (row(k) & ~31u) | (k & 31u); }
};

// one thread per vertex (neighbour counts <= 8: a 2-D cloth has ~2 cross-bank
// neighbours per vertex, and G lanes per vertex measured 78 vs 70 us at 1M)
// vertices [v0, v1) only: a sharded Prepare's own (the rows of every record of
// a vertex are its ancestors, so its own rows' records are its own vertices')
__global__ __launch_bounds__(256) void k_records_vertex(int nV, int L, RecKey rk, const int* __restrict__ s2o,
                                                 const int* __restrict__ nbrNum, const int* __restrict__ nbr,
                                                 const int* __restrict__ gn, const int* __restrict__ ranges,
                                                 const int* __restrict__ recOff, EdgeRec* __restrict__ rec,
                                                 EntryKey* __restrict__ keys, int* __restrict__ mats, int v0, int v1) {
    const int v = v0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= v1) return;
    const int o = s2o[v];
    const int num = nbrNum[v];
    const int base = ranges[o];
    int w = recOff[v];
    for (int k = 1; k < num; ++k) {
        unsigned my = (unsigned)v, ot = (unsigned)nbr[(size_t)k * nV + v];
        if ((my >> 5) == (ot >> 5)) continue;  // level 0: in the block (k_level0_block)
        const int level = climb(gn, L, my, ot);
        if (level >= L) {  // no common bank below L (.cpp:1286): a dead record, sorted last
            rec[w] = EdgeRec{L, -1, -1, base + k - 1};
            keys[w] = rk.dead();
        } else {
            rec[w] = EdgeRec{level, (int)my, (int)ot, base + k - 1};
            keys[w] = rk.pack(my, ot);
        }
        mats[w] = base + k - 1;  // sort payload: records of one entry stay in (u, k) order (stable sort)
        ++w;
    }
}

// G lanes per vertex (G >= the largest neighbour count; lane j takes ELL slot
// k = j + 1): a vertex's cross-bank neighbours are found by one ballot and
// each lane writes its record at recOff[v] + (rank among the vertex's
// cross-bank lanes), the (u, k) order of the thread-per-vertex form, whose
// serial loop of level climbs cost 1.17 ms for the 4M tet lattice (697 us
// this way).  Used when a vertex can have more than 8 neighbours.
template <int G>
__device__ __forceinline__ int group_rank(bool pred, unsigned long long& groupMask) {
    const int lane = threadIdx.x & 63, g0 = lane & ~(G - 1);
    const unsigned long long b = __ballot(pred);
    groupMask = G == 64 ? b : (b >> g0) & ((1ull << G) - 1);
    return __popcll(groupMask & ((1ull << (lane - g0)) - 1));
}

template <int G>
__global__ __launch_bounds__(256) void k_records(int nV, int L, RecKey rk, const int* __restrict__ s2o,
                                                 const int* __restrict__ nbrNum, const int* __restrict__ nbr,
                                                 const int* __restrict__ gn, const int* __restrict__ ranges,
                                                 const int* __restrict__ recOff, EdgeRec* __restrict__ rec,
                                                 EntryKey* __restrict__ keys, int* __restrict__ mats, int v0, int v1) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = v0 + t / G, k = 1 + t % G;
    const bool has = v < v1 && k < nbrNum[v];
    unsigned my = (unsigned)v, ot = has ? (unsigned)nbr[(size_t)k * nV + v] : (unsigned)v;
    const bool cross = has && (my >> 5) != (ot >> 5);  // same bank: level 0 (k_level0_block)
    unsigned long long grp;
    const int rank = group_rank<G>(cross, grp);
    if (!cross) return;
    const int base = ranges[s2o[v]];
    const int w = recOff[v] + rank;
    const int level = climb(gn, L, my, ot);
    if (level >= L) {  // no common bank below L (.cpp:1286): a dead record, sorted last
        rec[w] = EdgeRec{L, -1, -1, base + k - 1};
        keys[w] = rk.dead();
    } else {
        rec[w] = EdgeRec{level, (int)my, (int)ot, base + k - 1};
        keys[w] = rk.pack(my, ot);
    }
    mats[w] = base + k - 1;  // sort payload: records of one entry stay in (u, k) order (stable sort)
}

// The (row, col) runs of the stably sorted record keys are folded strictly
// left, so a run's fold is one dependent chain; what is parallel is its loads.
// Run lengths are very uneven (cloth 1M, 4 levels: ~10 records per level-1
// entry, hundreds per level-3 entry), and a thread walking a long run pays two
// dependent load latencies per record (mats, then off9) -- the longest runs set
// the kernel time.  So:
//   short runs (< kLongRun): one lane each; records are loaded kFoldBatch at
//                 a time (all loads issued, then the adds in order).
//   long runs:    the wave, one run after the other: 64 records per step are
//                 loaded by the lanes into LDS, then lanes 0..8 each fold one
//                 of the nine entries over them in order.
// (Collecting the long runs into a list with a counter was measured first: ~60k
// atomics on one address serialised and cost ~300 us.)
constexpr int kLongRun = 16, kFoldBatch = 8;
#ifndef MAS_LONG_STEP
#define MAS_LONG_STEP 256
#endif
constexpr int kLongStep = MAS_LONG_STEP, kLongK = kLongStep / 64, kLongStride = kLongStep + 1;  // long-run steps (below)

// Fold targets: where the 3x3 of a key lives and its row stride.
struct DenseEntry {  // block entry (row node, column node) of the dense buffer
    float* dense;
    RecKey rk;
    static constexpr int kStride = 96;
    static constexpr bool kFromZero = false;
    __device__ bool live(EntryKey) const { return true; }
    __device__ float* at(EntryKey k, int) const { return entry(dense, rk.row(k), rk.col(k)); }
};
struct DenseDiag {  // the diagonal entry of node key + kb
    float* dense;
    unsigned kb;
    static constexpr int kStride = 96;
    static constexpr bool kFromZero = false;
    __device__ bool live(unsigned) const { return true; }
    __device__ float* at(unsigned k, int) const { return entry(dense, k + kb, k + kb); }
};
struct NodeRow {  // a row-major 9-float row per node (additional)
    float* base;
    static constexpr int kStride = 3;
    static constexpr bool kFromZero = false;
    __device__ bool live(unsigned) const { return true; }
    __device__ float* at(unsigned k, int) const { return base + 9 * (size_t)k; }
};

// One wave per 64 sorted positions: the lanes find the runs starting there;
// each short-run lane folds its own run, then the wave folds the long runs one
// after the other.  (Separate kernels for the two kinds measured 106 + 78 us
// at 1M: each re-read the keys to find its runs.)  Each run is folded onto
// the target's current value in sorted (= stable, insertion) order; a record's
// 3x3 is vals[9 id ...], column-major (off9, contact values) or row-major
// (additional rows).  `dead` marks records to skip.
template <class Tgt, bool kColMajor, class Key>
__global__ __launch_bounds__(64) void k_fold_runs(int n, Key dead, const Key* __restrict__ keys,
                                                  const int* __restrict__ mats, const float* __restrict__ vals,
                                                  Tgt tgt) {
    __shared__ float T[9 * kLongStride];  // T[q * kLongStride + record]: component q (row-major)
    constexpr int S = Tgt::kStride;
    auto comp = [](int r, int c) { return kColMajor ? c * 3 + r : r * 3 + c; };
    const int lane = threadIdx.x;
    const int i = blockIdx.x * 64 + lane;
    bool isStart = false, isLong = false;
    Key key = 0;
    if (i < n) {
        key = keys[i];
        isStart = key != dead && tgt.live(key) && (i == 0 || keys[i - 1] != key);
        // sorted: a run starting at i has >= kLongRun records iff position i + kLongRun - 1 has its key
        isLong = isStart && i + kLongRun - 1 < n && keys[i + kLongRun - 1] == key;
    }
    if (isStart && !isLong) {  // short run: this lane, loads batched kFoldBatch at a time
        float* e = tgt.at(key, i);
        float acc[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) acc[r * 3 + c] = Tgt::kFromZero ? 0.f : e[r * S + c];
        for (int j0 = i; j0 < i + kLongRun; j0 += kFoldBatch) {
            bool in[kFoldBatch];
            float m[kFoldBatch][9];
#pragma unroll
            for (int t = 0; t < kFoldBatch; ++t) {
                const int j = j0 + t;
                in[t] = j < n && keys[j] == key;
                const float* src = vals + 9 * (size_t)(in[t] ? mats[j] : mats[i]);
#pragma unroll
                for (int q = 0; q < 9; ++q) m[t][q] = src[q];
            }
#pragma unroll
            for (int t = 0; t < kFoldBatch; ++t)
                if (in[t])
                    for (int r = 0; r < 3; ++r)
                        for (int c = 0; c < 3; ++c) acc[r * 3 + c] = __fadd_rn(acc[r * 3 + c], m[t][comp(r, c)]);
            if (!in[kFoldBatch - 1]) break;
        }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) e[r * S + c] = acc[r * 3 + c];
    }
    // long runs: the whole wave, kLongStep records per step (kLongK per lane,
    // coalesced) staged in LDS, lanes 0..8 each folding one of the nine
    // entries over them in order.  Software-pipelined: while a step is folded,
    // the values of the next step and the keys / record ids of the one after
    // it are in flight, so a step costs its fold, not the three dependent
    // load latencies (keys -> ids -> values) it took when each 64-record step
    // waited for its own loads (~4.5 us per step; the push and contact-entry
    // folds' runs of ~1 000 records set a world-8 rank's Prepare chain).
    const int r = lane / 3, c = lane % 3;
    for (unsigned long long starts = __ballot(isLong); starts; starts &= starts - 1) {
        const int start = blockIdx.x * 64 + __ffsll((long long)starts) - 1;
        const Key lkey = keys[start];
        float* e = tgt.at(lkey, start);
        float acc = lane < 9 && !Tgt::kFromZero ? e[r * S + c] : 0.f;
        auto loadKM = [&](int p0, bool (&in)[kLongK], int (&mt)[kLongK]) {
#pragma unroll
            for (int k = 0; k < kLongK; ++k) {
                const int pos = p0 + 64 * k + lane;
                in[k] = pos < n && keys[pos] == lkey;
                mt[k] = pos < n ? mats[pos] : 0;
            }
        };
        auto loadV = [&](const int (&mt)[kLongK], float (&v)[kLongK][9]) {
#pragma unroll
            for (int k = 0; k < kLongK; ++k) {
                const float* src = vals + 9 * (size_t)mt[k];
#pragma unroll
                for (int q = 0; q < 9; ++q) v[k][q] = src[q];
            }
        };
        bool inA[kLongK], inB[kLongK];
        int mA[kLongK], mB[kLongK];
        float vA[kLongK][9];
        loadKM(start, inA, mA);
        loadV(mA, vA);
        loadKM(start + kLongStep, inB, mB);
        for (int p0 = start;; p0 += kLongStep) {
            int cnt = 0;  // the run is contiguous: positions p0 .. p0 + cnt - 1
#pragma unroll
            for (int k = 0; k < kLongK; ++k) cnt += __popcll(__ballot(inA[k]));
#pragma unroll
            for (int k = 0; k < kLongK; ++k)
                if (inA[k])
#pragma unroll
                    for (int q = 0; q < 9; ++q) T[q * kLongStride + 64 * k + lane] = vA[k][q];
            float vB[kLongK][9];
            bool inC[kLongK];
            int mC[kLongK];
            if (cnt == kLongStep) {  // the next step's values, the one after's keys and ids
                loadV(mB, vB);
                loadKM(p0 + 2 * kLongStep, inC, mC);
            }
            __syncthreads();
            if (lane < 9) {
                const float* col = T + comp(r, c) * kLongStride;
                for (int k = 0; k < cnt; ++k) acc = __fadd_rn(acc, col[k]);
            }
            __syncthreads();
            if (cnt < kLongStep) break;
#pragma unroll
            for (int k = 0; k < kLongK; ++k) {
                inA[k] = inB[k];
                inB[k] = inC[k];
                mB[k] = mC[k];
#pragma unroll
                for (int q = 0; q < 9; ++q) vA[k][q] = vB[k][q];
            }
        }
        if (lane < 9) e[r * S + c] = acc;
    }
}

// level-1 diagonal: one thread per level-0 bank, members in lane order.  The
// bank's vertices mostly share one level-1 node, so the running entry stays in
// registers and is written back only when the parent changes (the same left
// fold, without a dependent read-modify-write of HBM per vertex).
// The bank's parents and od rows are loaded 8 vertices at a time, all loads
// of a batch issued before its adds (one dependent round trip per batch
// instead of one per vertex: beside the fused kernel this kernel runs on the
// reserved CUs and was bound by those round trips).
__global__ __launch_bounds__(256) void k_diag1(int nV, const int* __restrict__ gn, const float* __restrict__ od,
                                               float* __restrict__ dense, int w0, int w1) {
    constexpr int kB = 8;
    const int w = w0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= w1 || w * 32 >= nV) return;
    const int end = min(w * 32 + 32, nV);
    unsigned cur = (unsigned)gn[w * 32];
    float acc[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) acc[r * 3 + c] = entry(dense, cur, cur)[r * 96 + c];
    for (int u0 = w * 32; u0 < end; u0 += kB) {
        unsigned pb[kB];
        float ob[kB][9];
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            const int u = min(u0 + i, end - 1);  // clamped: the tail's extra rows are not added
            pb[i] = (unsigned)gn[u];
            const float* a = od + 9 * (size_t)u;
#pragma unroll
            for (int e = 0; e < 9; ++e) ob[i][e] = a[e];
        }
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            if (u0 + i >= end) break;
            if (pb[i] != cur) {
                float* e = entry(dense, cur, cur);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) e[r * 96 + c] = acc[r * 3 + c];
                cur = pb[i];
                e = entry(dense, cur, cur);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) acc[r * 3 + c] = e[r * 96 + c];
            }
#pragma unroll
            for (int e = 0; e < 9; ++e) acc[e] = __fadd_rn(acc[e], ob[i][e]);
        }
    }
    float* e = entry(dense, cur, cur);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) e[r * 96 + c] = acc[r * 3 + c];
}

// Stable grouping boundaries: off[key] = first sorted position of key.
__global__ __launch_bounds__(256) void k_bounds(int n, const int* __restrict__ sortedKeys, int nKeys,
                                                int* __restrict__ off) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k = sortedKeys[i];
    if (i == 0 || sortedKeys[i - 1] != k) off[k] = i;
    if (i == n - 1) off[nKeys] = n;
}

// diagTable fold for level l >= 2, one thread per level-l node P.
// diagTable fold (.cpp:1299-1343), parallelised over the terms but folded
// strictly left in the reference's order.  For level l the ordered term list
// of node P is: for each member vertex u in ascending order, u's edge records
// with lam == l-1 (in (u, k) order) and, for l == 2, od(u); then (l >= 3) the
// level-(l-1) tables of the children in id order.  k_term_count / scan /
// k_term_write flatten the vertex part into one index array (>= 0: off9
// matrix, < 0: od of vertex -t-1); k_table_fold folds it with one wave per
// node: the wave stages 256 terms at a time in LDS (coalesced loads, 4 terms
// in flight per lane) and lanes 0..8 each fold one of the nine entries.
__global__ __launch_bounds__(256) void k_term_count(int l, int nV, const int* __restrict__ vlist,
                                                    const int* __restrict__ recOff, const EdgeRec* __restrict__ rec,
                                                    int* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nV) return;
    if (i == nV) { cnt[i] = 0; return; }
    const int u = vlist[i];
    int c = (l == 2) ? 1 : 0;
    for (int j = recOff[u]; j < recOff[u + 1]; ++j) c += (rec[j].lam == l - 1);
    cnt[i] = c;
}

__global__ __launch_bounds__(256) void k_term_write(int l, int nV, const int* __restrict__ vlist,
                                                    const int* __restrict__ recOff, const EdgeRec* __restrict__ rec,
                                                    const int* __restrict__ termOff, int* __restrict__ terms) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nV) return;
    const int u = vlist[i];
    int o = termOff[i];
    for (int j = recOff[u]; j < recOff[u + 1]; ++j) {
        const EdgeRec r = rec[j];
        if (r.lam == l - 1) terms[o++] = r.mat;
    }
    if (l == 2) terms[o] = -(u + 1);
}

// k_term_write with G lanes per member vertex (lane j: the vertex's j-th
// record; positions by ballot rank), for vertices with more than 8
// neighbours: 490 -> 324 us per level for the 4M tet lattice, slower than the
// thread per vertex at 1M cloth (29 vs 16 us).  (The same form of
// k_term_count was slower at both sizes.)
template <int G>
__global__ __launch_bounds__(256) void k_term_write_lanes(int l, int nV, const int* __restrict__ vlist,
                                                          const int* __restrict__ recOff,
                                                          const EdgeRec* __restrict__ rec,
                                                          const int* __restrict__ termOff, int* __restrict__ terms) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = t / G, j = t % G;
    bool hit = false;
    int u = 0, mat = 0;
    if (i < nV) {
        u = vlist[i];
        const int r = recOff[u] + j;
        if (r < recOff[u + 1]) {
            const EdgeRec e = rec[r];
            hit = e.lam == l - 1;
            mat = e.mat;
        }
    }
    unsigned long long grp;
    const int rank = group_rank<G>(hit, grp);
    if (i >= nV) return;
    const int o = termOff[i];
    if (hit) terms[o + rank] = mat;
    if (l == 2 && j == 0) terms[o + __popcll(grp)] = -(u + 1);
}

// Terms per staged chunk of k_table_fold (a compile-time A/B knob): 256
// against 512 / 1024 / 128, world-8 rank at 1M + contacts 1.29 -> 1.24 ms,
// 4M tet rank 3.70 -> 3.6 (the 9.4 KB of LDS per node leaves room for more
// nodes per CU; 1024 was slower everywhere, 128 the same as 256;
// profiles/round5/ab/table_fold_chunk/)
#ifndef MAS_FOLD_CHUNK
#define MAS_FOLD_CHUNK 256
#endif
// Levels with few nodes (a shard's level 3: 4 nodes at 1M) are one node's
// dependent chain of ~10k terms; there a 256-term chunk's fold (~1 000
// cycles) is shorter than the HBM latency the two-deep pipeline hides, so
// they fold 1 024-term chunks (k_table_fold<kFoldChunkFew>, 37 KB of LDS).
constexpr int kFoldChunkFew = 1024, kFoldFewNodes = 64;

template <int kFoldChunk>
__global__ __launch_bounds__(64) void k_table_fold(int l, int count, int begin, int beginPrev,
                                                   const int* __restrict__ vlist, const int* __restrict__ voff,
                                                   const int* __restrict__ termOff, const int* __restrict__ terms,
                                                   const int* __restrict__ cstPrev2, const int* __restrict__ gn,
                                                   const float* __restrict__ off9, const float* __restrict__ od,
                                                   float* __restrict__ tab, float* __restrict__ dense, int local0) {
    constexpr int kFoldStride = kFoldChunk + 4;
    __shared__ __attribute__((aligned(16))) float st[9 * kFoldStride];
    const int local = local0 + blockIdx.x;
    const int lane = threadIdx.x;
    const int P = begin + local;
    const int vb = voff[local], ve = voff[local + 1];
    const int tb = termOff[vb], te = termOff[ve];
    // lane q < 9 folds entry q = (row, col) = (q / 3, q % 3); off9 is column-major
    const int q = lane < 9 ? lane : 0;
    float acc = 0.f;
    // Software-pipelined two chunks deep: while lanes 0..8 fold chunk i from
    // LDS, the term matrices of chunk i+1 (whose term ids arrived during the
    // previous fold) and the term ids of chunk i+2 are in flight, so no HBM
    // latency is exposed per chunk (the first form waited two dependent
    // latencies per 256 terms: 220 us for the ~10k-term chains of the 32
    // level-3 nodes at 1M).  Loads are unconditional (indices clamped into the
    // chunk; the fold never reads past n).  LDS is entry-major with a padded
    // stride, so a folding lane reads 4 terms per ds_read_b128 and lanes 0..8
    // hit distinct banks.  One wave per workgroup: its LDS operations run in
    // program order and one buffer suffices.
    constexpr int kPer = kFoldChunk / 64;
    float reg[kPer][9];
    int tk[kPer];
    auto loadIds = [&](int base) {
        const int last = min(kFoldChunk, te - base) - 1;
#pragma unroll
        for (int m = 0; m < kPer; ++m) tk[m] = terms[base + min(m * 64 + lane, last)];
    };
    auto loadMats = [&]() {
#pragma unroll
        for (int m = 0; m < kPer; ++m) {
            const int t = tk[m];
            const bool colMajor = t >= 0;
            const float* src = colMajor ? off9 + 9 * (size_t)t : od + 9 * (size_t)(-t - 1);
#pragma unroll
            for (int e = 0; e < 9; ++e) reg[m][e] = src[colMajor ? (e % 3) * 3 + e / 3 : e];
        }
    };
    if (tb < te) {
        loadIds(tb);
        loadMats();
        if (tb + kFoldChunk < te) loadIds(tb + kFoldChunk);
    }
    for (int base = tb; base < te; base += kFoldChunk) {
        const int n = min(kFoldChunk, te - base);
#pragma unroll
        for (int m = 0; m < kPer; ++m)
#pragma unroll
            for (int e = 0; e < 9; ++e) st[e * kFoldStride + m * 64 + lane] = reg[m][e];
        __syncthreads();
        if (base + kFoldChunk < te) {
            loadMats();
            if (base + 2 * kFoldChunk < te) loadIds(base + 2 * kFoldChunk);
        }
        if (lane < 9) {
            const float* col = st + q * kFoldStride;
            int k = 0;
            for (; k + 8 <= n; k += 8) {
                const float4 x0 = *reinterpret_cast<const float4*>(col + k);
                const float4 x1 = *reinterpret_cast<const float4*>(col + k + 4);
                acc = __fadd_rn(acc, x0.x);
                acc = __fadd_rn(acc, x0.y);
                acc = __fadd_rn(acc, x0.z);
                acc = __fadd_rn(acc, x0.w);
                acc = __fadd_rn(acc, x1.x);
                acc = __fadd_rn(acc, x1.y);
                acc = __fadd_rn(acc, x1.z);
                acc = __fadd_rn(acc, x1.w);
            }
            for (; k < n; ++k) acc = __fadd_rn(acc, col[k]);
        }
        __syncthreads();
    }
    bool present = te > tb;
    if (l >= 3 && ve > vb) {  // pushes of the level-(l-1) tables, children in id order (.cpp:1333-1341)
        const int childLocal = cstPrev2[vlist[vb]];  // level-(l-1) local id of the first member
        const int bankBase = beginPrev + (childLocal & ~31);
        // the bank's 32 parent ids and all 288 table floats are loaded at once
        // (a dependent load per child cost ~32 HBM latencies per node)
        const unsigned long long kids = __ballot(lane < 32 && gn[bankBase + (lane & 31)] == P) & 0xffffffffull;
        for (int x = lane; x < 32 * 9; x += 64) st[x] = tab[9 * (size_t)bankBase + x];
        __syncthreads();
        for (unsigned long long m = kids; m; m &= m - 1) {
            const int j = __ffsll((long long)m) - 1;  // children in id order
            if (lane < 9) acc = __fadd_rn(acc, st[9 * j + q]);
        }
        present = present || kids != 0;
    }
    if (lane < 9) {
        tab[9 * (size_t)P + q] = acc;
        if (present) {
            float* d = entry(dense, (unsigned)P, (unsigned)P) + (q / 3) * 96 + q % 3;
            *d = __fadd_rn(*d, acc);
        }
    }
}

static void table_fold(int cnt, int l, int count, int begin, int beginPrev, const int* vlist, const int* voff,
                       const int* termOff, const int* terms, const int* cstPrev2, const int* gn, const float* off9,
                       const float* od, float* tab, float* dense, int local0, hipStream_t s) {
    if (cnt <= kFoldFewNodes)
        k_table_fold<kFoldChunkFew><<<cnt, 64, 0, s>>>(l, count, begin, beginPrev, vlist, voff, termOff, terms,
                                                       cstPrev2, gn, off9, od, tab, dense, local0);
    else
        k_table_fold<MAS_FOLD_CHUNK><<<cnt, 64, 0, s>>>(l, count, begin, beginPrev, vlist, voff, termOff, terms,
                                                        cstPrev2, gn, off9, od, tab, dense, local0);
}

template <class T>
static int exclusive_scan(mas_context* h, const T* in, T* out, int n, hipStream_t s, const char* what) {
    if constexpr (std::is_same_v<T, int>)
        if (h->sortImpl) return rs_exclusive_scan(h, in, out, n, s, what);
    size_t tmp = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, n, s);
    int rc = ensure(h, h->cubTemp, tmp);
    if (rc) return rc;
    return hip_check(h, hipcub::DeviceScan::ExclusiveSum(h->cubTemp.p, tmp, in, out, n, s), what);
}

int sort_pairs_u32(mas_context* h, const unsigned* kin, unsigned* kout, const int* vin, int* vout, int n, int bits,
                   hipStream_t s, const char* what) {
    return sort_pairs(h, kin, kout, vin, vout, n, bits, s, what);
}

// Fused variant: k_factor_fused over the prepared level-0 blocks on
// prepStream, after everything this stream has queued (its inputs: additional
// and the prefolded level-0 contact entries); run_factor joins
// (measured: a CU-masked side stream, stream priorities and a persistent
// fused grid all lost to this plain form).
int prep_stream_init(mas_context* h) {
    int rc = MAS_OK;
    if (!h->prepStream) {
        // The fused kernel's queue may leave prepCuReserve CUs (env
        // MAS_PREP_CU_RESERVE, opt-in since round 6: a CU-masked queue in a
        // process beside another GPU process stalled its applies, mas_internal.h)
        // to the caller's stream: without that the coarse
        // assembly gets no slot while the fused kernel's 32 768 waves hold
        // every CU, and the two run one after the other.  The reserved CUs are
        // spread over the mask so that every XCD loses the same number whether
        // the bits map to XCDs by bit % 8 or by bit / 32.
        const int reserve = h->prepCuReserve;
        hipDeviceProp_t prop{};
        if (reserve > 0 && hipGetDeviceProperties(&prop, h->device) == hipSuccess &&
            prop.multiProcessorCount % 32 == 0 && reserve % 8 == 0 && reserve <= prop.multiProcessorCount / 2) {
            const int n = prop.multiProcessorCount, words = n / 32, per = n / 8;
            std::vector<uint32_t> mask(words, 0xffffffffu);
            for (int j = 0; j < reserve; ++j) {
                const int x = j % 8, y = j / 8;
                const int bit = per * x + (8 * (y % (per / 8)) + x + y / (per / 8)) % per;
                mask[bit / 32] &= ~(1u << (bit % 32));
            }
            rc = hip_check(h, hipExtStreamCreateWithCUMask(&h->prepStream, words, mask.data()), "prepare stream");
        } else {
            rc = hip_check(h, hipStreamCreateWithFlags(&h->prepStream, hipStreamNonBlocking), "prepare stream");
        }
        if (rc) return rc;
    }
    if (!h->evPrepFork &&
        ((rc = hip_check(h, hipEventCreateWithFlags(&h->evPrepFork, hipEventDisableTiming), "event")) ||
         (rc = hip_check(h, hipEventCreateWithFlags(&h->evPrepJoin, hipEventDisableTiming), "event")) ||
         (rc = hip_check(h, hipEventCreate(&h->evFine[0]), "event")) ||
         (rc = hip_check(h, hipEventCreate(&h->evFine[1]), "event")) ||
         (rc = hip_check(h, hipEventCreateWithFlags(&h->evAdd0, hipEventDisableTiming), "event"))))
        return rc;
    return rc;
}

static int fork_fused(mas_context* h, const FineAsm& fa, hipStream_t s) {
    int rc;
    if ((rc = prep_stream_init(h))) return rc;
    // MAS_PREP_SERIAL=1 (A/B): the same kernel in line on the caller's stream
    static const bool serial = std::getenv("MAS_PREP_SERIAL") && std::atoi(std::getenv("MAS_PREP_SERIAL"));
    hipStream_t ps = serial ? s : h->prepStream;
    if ((rc = hip_check(h, hipEventRecord(h->evPrepFork, s), "fork")) ||
        (rc = hip_check(h, hipStreamWaitEvent(ps, h->evPrepFork, 0), "fork wait")) ||
        (rc = hip_check(h, hipEventRecord(h->evFine[0], ps), "record")) ||
        (rc = launch_factor_fused(h, fa, h->fineBlk0, h->fineBlk1, ps)) ||
        (rc = hip_check(h, hipEventRecord(h->evFine[1], ps), "record")) ||
        (rc = hip_check(h, hipEventRecord(h->evPrepJoin, ps), "join")))
        return rc;
    return MAS_OK;
}

// The contact part of the assembly in the reference's single-thread order
// (see "contacts" above): on return the coarse blocks hold the contact block
// entries and the additional pushes, `additional` holds every node's contact
// row, and fc points k_level0_block at the fine block entries.
static int run_contacts(mas_context* h, hipStream_t s, FineContacts& fc, FineAsm& fa, bool& forked) {
    const int n = h->nStencil, L = h->L, tc = h->totalClusters, begin1 = L > 1 ? h->levelSize[3] : tc;
    const int B = std::max(1, bit_width((unsigned)(tc - 1)));
    const int* gn = P<int>(h->goingNext);
    const DevStencil* st = P<DevStencil>(h->stencils);
    int rc;
    if (B + RecKey::kLaneBits > 32) return fail(h, MAS_ERR_ARG, "contact entry keys: more than 2^27 nodes");
    if ((rc = ensure(h, h->cdCnt, (size_t)(n + 1) * 4)) || (rc = ensure(h, h->cdOff, (size_t)(n + 1) * 4)) ||
        (rc = ensure(h, h->caCnt, (size_t)(n + 1) * 4)) || (rc = ensure(h, h->caOff, (size_t)(n + 1) * 4)) ||
        (!h->earlyPlanned && (rc = ensure(h, h->cFineOff, (size_t)(h->nFineBlk + 1) * 4))))  // prepStream's otherwise
        return rc;
    const bool skip0 = h->earlyPlanned;  // level-0 records built by run_level0_early (its worker may still be queueing)
    // keys relative to kb: with only coarse records (skip0) every row, node and
    // push target is >= begin_1, so the sorts need the bits of the coarse node
    // count (16 at 1M) instead of all nodes' (21): one pass less per sort
    const unsigned kb = skip0 ? (unsigned)begin1 : 0u;
    const int Bk = skip0 ? std::max(1, bit_width((unsigned)std::max(tc - begin1 - 1, 0))) : B;
    const int4* anc = P<int4>(h->coarseTables);
    k_contact_count<<<cdiv(n + 1, 256), 256, 0, s>>>(st, n, anc, L, P<int>(h->cdCnt), P<int>(h->caCnt), skip0, h->own);
    if ((rc = exclusive_scan(h, P<int>(h->cdCnt), P<int>(h->cdOff), n + 1, s, "contact scan")) ||
        (rc = exclusive_scan(h, P<int>(h->caCnt), P<int>(h->caOff), n + 1, s, "contact scan")))
        return rc;
    int tot[2] = {0, 0};
    if ((rc = read_back(h, s, {P<int>(h->cdOff) + n, P<int>(h->caOff) + n}, tot))) return rc;
    const int nD = tot[0], nA = tot[1];
    const size_t d1 = nD > 0 ? nD : 1, a1 = nA > 0 ? nA : 1;
    if ((rc = ensure(h, h->cdKeys, d1 * 4)) || (rc = ensure(h, h->cdKeysS, d1 * 4)) ||
        (rc = ensure(h, h->cdIds, d1 * 4)) || (rc = ensure(h, h->cdIdsS, d1 * 4)) ||
        (rc = ensure(h, h->cdVal, d1 * 36)) || (rc = ensure(h, h->cdEnt, d1 * 4)) || (rc = ensure(h, h->caKeys, a1 * 4)) ||
        (rc = ensure(h, h->caKeysS, a1 * 4)) || (rc = ensure(h, h->caIds, a1 * 4)) ||
        (rc = ensure(h, h->caIdsS, a1 * 4)) || (rc = ensure(h, h->caVal, a1 * 36)) ||
        (rc = ensure(h, h->cpCnt, (a1 + 1) * 4)) || (rc = ensure(h, h->cpOff, (a1 + 1) * 4)))
        return rc;
    k_contact_write<<<cdiv(n, 256), 256, 0, s>>>(st, n, anc, L, P<int>(h->cdOff), P<int>(h->caOff),
                                                 P<EntryKey>(h->cdKeys), P<int>(h->cdIds),
                                                 P<float>(h->cdVal), P<int>(h->cdEnt), P<unsigned>(h->caKeys),
                                                 P<int>(h->caIds), P<float>(h->caVal), skip0, kb, h->own);
    if ((rc = sort_pairs(h, P<EntryKey>(h->cdKeys), P<EntryKey>(h->cdKeysS), P<int>(h->cdIds),
                         P<int>(h->cdIdsS), nD, Bk + RecKey::kLaneBits, s, "contact entry sort")) ||
        (rc = sort_pairs(h, P<unsigned>(h->caKeys), P<unsigned>(h->caKeysS), P<int>(h->caIds), P<int>(h->caIdsS), nA,
                         Bk, s, "contact row sort")))
        return rc;
    float* dense = dense_base(h);
    // fine entries: k_level0_block; coarse entries: folded onto the zeroed coarse blocks
    if (!skip0)
        k_contact_fine_bounds<<<cdiv(nD + 1, 256), 256, 0, s>>>(nD, RecKey::kLaneBits, begin1, h->nFineBlk,
                                                            P<EntryKey>(h->cdKeysS), P<int>(h->cFineOff));
    // additional rows (level 0 and coarse), folded from zero
    if (nA > 0)
        k_fold_runs<NodeRow, true, unsigned><<<cdiv(nA, 64), 64, 0, s>>>(
            nA, 0xffffffffu, P<unsigned>(h->caKeysS), P<int>(h->caIdsS), P<float>(h->caVal),
            NodeRow{P<float>(h->additional) + 9 * (size_t)kb});
    fc = FineContacts{P<EntryKey>(h->cdKeysS), P<int>(h->cdIdsS), P<float>(h->cdVal), P<int>(h->cFineOff),
                      RecKey::kLaneBits};
    if (h->factorVariant >= 4 && !skip0) {
        if (nD > 0) {
            // the level-0 records lead the entry-sorted array (rows < begin1),
            // each entry's in stencil order: the fused kernel adds them per block
            fa.coff = P<int>(h->cFineOff);
            fa.cids = P<int>(h->cdIdsS);
            fa.cent = P<int>(h->cdEnt);
            fa.cvals = P<float>(h->cdVal);
        }
        // the level-0 blocks need nothing below (pushes and coarse entries):
        // they start now, before the push count's host round trip
        if ((rc = fork_fused(h, fa, s))) return rc;
        forked = true;
    }
    k_push_count<<<cdiv(nA + 1, 256), 256, 0, s>>>(nA, begin1, tc, P<unsigned>(h->caKeysS), kb, gn,
                                                   P<int>(h->cpCnt));
    if ((rc = exclusive_scan(h, P<int>(h->cpCnt), P<int>(h->cpOff), nA + 1, s, "push scan"))) return rc;
    int pf[2] = {0, 0};  // push count, first coarse block-entry record (0: no level-0 records here)
    if (skip0) {
        if ((rc = read_back(h, s, {P<int>(h->cpOff) + nA}, pf))) return rc;
    } else if ((rc = read_back(h, s, {P<int>(h->cpOff) + nA, P<int>(h->cFineOff) + h->nFineBlk}, pf))) {
        return rc;
    }
    const int nP = pf[0], fineEnd = pf[1];
    const RecKey rk{(int)kb, Bk};
    if (nD > fineEnd)
        k_fold_runs<DenseEntry, true, EntryKey><<<cdiv(nD - fineEnd, 64), 64, 0, s>>>(
            nD - fineEnd, ~0u, P<EntryKey>(h->cdKeysS) + fineEnd, P<int>(h->cdIdsS) + fineEnd,
            P<float>(h->cdVal), DenseEntry{dense, rk});
    if (nP > 0) {
        if ((rc = ensure(h, h->cpKeys, (size_t)nP * 4)) || (rc = ensure(h, h->cpKeysS, (size_t)nP * 4)) ||
            (rc = ensure(h, h->cpIds, (size_t)nP * 4)) || (rc = ensure(h, h->cpIdsS, (size_t)nP * 4)))
            return rc;
        k_push_write<<<cdiv(nA, 256), 256, 0, s>>>(nA, begin1, tc, P<unsigned>(h->caKeysS), kb, gn,
                                                   P<int>(h->cpOff), P<unsigned>(h->cpKeys), P<int>(h->cpIds));
        if ((rc = sort_pairs(h, P<unsigned>(h->cpKeys), P<unsigned>(h->cpKeysS), P<int>(h->cpIds), P<int>(h->cpIdsS),
                             nP, Bk, s, "push sort")))
            return rc;
        // .cpp:1236-1252: diag(target) += additional[x], x ascending (row-major rows)
        k_fold_runs<DenseDiag, false, unsigned><<<cdiv(nP, 64), 64, 0, s>>>(
            nP, 0xffffffffu, P<unsigned>(h->cpKeysS), P<int>(h->cpIdsS), P<float>(h->additional),
            DenseDiag{dense, kb});
    }
    return hip_check(h, hipGetLastError(), "contact kernels");
}

// The level-0 blocks need only level-0 data -- the sorted vertices' CSR rows,
// the level-0 contact entries and additional rows -- not the coarse levels.
// So right after the stencils the caller's stream forks prepStream, which
// builds the level-0 contact records (k_contact0_*: no level ids, no host
// read: sizes are bounded by the stencil count and the tails carry the
// sentinel key), sorts and folds them exactly as run_contacts does for rows
// < begin_1, and starts the fused assemble + factor kernel, while the caller's
// stream builds the levels, the coarse contact records (run_contacts skips the
// level-0 ones) and the coarse assembly on the CUs the fused kernel's queue
// leaves free (prep_stream_init).  Same records in the same order: every
// block bitwise as before.
// od and the coarse record counts (k_od / k_od_lanes): level-0 data only.
// Lanes per vertex: the largest neighbour count (ELL slot 0 is the vertex
// itself), a power of two.
// vertices [v0, v1) (a sharded Prepare with the coarse split: its own)
static void launch_od(mas_context* h, const FineAsm& fa, hipStream_t s, int v0, int v1) {
    const long long n = v1 - v0;
    const int val = h->maxNbr - 1;
    float* od = P<float>(h->od);
    int* cnt = P<int>(h->recCnt);
    if (n <= 0) return;
    if (val <= 8) k_od_lanes<8><<<cdiv(n * 8, 256), 256, 0, s>>>(fa, od, cnt, v0, v1);
    else if (val <= 16) k_od_lanes<16><<<cdiv(n * 16, 256), 256, 0, s>>>(fa, od, cnt, v0, v1);
    else if (val <= 32) k_od_lanes<32><<<cdiv(n * 32, 256), 256, 0, s>>>(fa, od, cnt, v0, v1);
    else k_od<<<cdiv(n, 256), 256, 0, s>>>(fa, od, cnt, v0, v1);
}

// od and the record counts in the early path (see run_level0_early)
// od and the record counts in the early path: by default for a sharded Prepare
// and for an unsharded one of 2 048 .. 32 768 level-0 blocks, where the
// coarse assembly then starts its chain without the od pass (round 6, beside
// the chunked fused kernel, steady state, ms: 1M + contacts 2.571 -> 2.450,
// 1M cloth 1.913 -> 1.876, 256k 0.571 -> 0.547; 4M tet 8.27 -> 8.57, so not
// there; profiles/round6/prepare/r6y, r6z)
bool early_od(const mas_context* h) {
    if (h->earlyOd >= 0) return h->earlyOd > 0;
    return h->prepWorld > 1 || (h->nFineBlk >= 2048 && h->nFineBlk <= 32768);
}

bool early_fused_wanted(const mas_context* h) {
    const int nv32 = h->nFineBlk * 32;
    return h->factorVariant >= 4 && !h->cfg.keep_blocks && nv32 > 0 &&
           bit_width((unsigned)(nv32 - 1)) + 1 + RecKey::kLaneBits <= 32;  // level-0 keys fit (else the late path)
}

// The early path's buffers that the caller's thread reads as well, sized by
// the caller before the worker starts (run_prepare): the level-0 inverses go
// straight into inv -- room for them now and for a coarse share like the
// previous Prepare's (run_assemble grows it, keeping the level-0 part, if the
// hierarchy needs more) -- add0, and od / the record counts when early_od.
int early_buffers(mas_context* h) {
    const size_t blockBytes = (size_t)kBlockFloats * 4;
    const size_t want = (size_t)std::max(h->nBlkPrev, h->nFineBlk + h->nFineBlk / 8 + 64) * blockBytes;
    int rc;
    if (h->inv.bytes < (size_t)h->nFineBlk * blockBytes && (rc = ensure(h, h->inv, want))) return rc;
    if ((rc = ensure(h, h->add0, (size_t)h->nFineBlk * 32 * 36))) return rc;
    if (early_od(h) && ((rc = ensure(h, h->od, (size_t)h->nV * 36)) ||
                        (rc = ensure(h, h->recCnt, (size_t)(h->nV + 1) * 4))))
        return rc;
    return MAS_OK;
}

int run_level0_early(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, hipStream_t s) {
    h->earlyFused = false;
    if (!early_fused_wanted(h)) return MAS_OK;
    int rc;
    if ((rc = prep_stream_init(h))) return rc;
    static const bool serial = std::getenv("MAS_PREP_SERIAL") && std::atoi(std::getenv("MAS_PREP_SERIAL"));
    hipStream_t ps = serial ? s : h->prepStream;
    const int nV = h->nV, n = h->nStencil, nv32 = h->nFineBlk * 32;
    if ((rc = early_buffers(h))) return rc;  // sized by run_prepare already: no allocation here
    // evPrepFork was recorded on s right after the stencils (run_prepare), before
    // the level kernels: prepStream waits for the stencils only
    if ((rc = hip_check(h, hipStreamWaitEvent(ps, h->evPrepFork, 0), "fork wait"))) return rc;
    FineAsm fa{nV, h->maxNbr, P<int>(h->s2o), P<int>(h->nbrNum), P<int>(h->nbr), d_diag9, d_off9, d_ranges,
               P<float>(h->add0), nullptr, nullptr, nullptr, nullptr, nullptr};
    if (n > 0) {
        // record bounds: 2 C(5, 2) = 20 block entries per EF stencil, 2 C(4, 2) = 12 per EE / VF
        // stencil (the sort runs over all of them); kA0 rows per stencil
        const size_t ubD = (size_t)h->nStencilEF * 20 + (size_t)(n - h->nStencilEF) * 12, ubA = (size_t)n * kA0;
        if (ubD > 0x7fffffff) return fail(h, MAS_ERR_ARG, "too many contact stencils");
        if ((rc = ensure(h, h->c0Cnt, (size_t)(n + 1) * 4)) || (rc = ensure(h, h->c0Off, (size_t)(n + 1) * 4)) ||
            (rc = ensure(h, h->c0Keys, ubD * 4)) || (rc = ensure(h, h->c0KeysS, ubD * 4)) ||
            (rc = ensure(h, h->c0Ids, ubD * 4)) || (rc = ensure(h, h->c0IdsS, ubD * 4)) ||
            (rc = ensure(h, h->c0Val, ubD * 36)) || (rc = ensure(h, h->c0Ent, ubD * 4)) ||
            (rc = ensure(h, h->a0Keys, ubA * 4)) || (rc = ensure(h, h->a0KeysS, ubA * 4)) ||
            (rc = ensure(h, h->a0Ids, ubA * 4)) || (rc = ensure(h, h->a0IdsS, ubA * 4)) ||
            (rc = ensure(h, h->a0Val, ubA * 36)) || (rc = ensure(h, h->cFineOff, (size_t)(h->nFineBlk + 1) * 4)))
            return rc;
        // add0 zeroed, sentinel keys past the records (their ids index record
        // 0: never folded, a sentinel is dead, but no index is left
        // undefined), and the per-stencil counts: one launch
        const DevStencil* st = P<DevStencil>(h->stencils);
        k_contact0_init<<<std::max(cdiv(n + 1, 256), 1024), 256, 0, ps>>>(
            st, n, P<int>(h->c0Cnt), P<float4>(h->add0), (size_t)nv32 * 9 / 4, P<EntryKey>(h->c0Keys),
            P<int>(h->c0Ids), ubD, P<unsigned>(h->a0Keys), P<int>(h->a0Ids), ubA);
        // prepStream's own sort / scan scratch (rs_*(..., side = true)), whatever MAS_SORT selects
        if ((rc = rs_exclusive_scan(h, P<int>(h->c0Cnt), P<int>(h->c0Off), n + 1, ps, "level-0 contact scan", true)))
            return rc;
        k_contact0_write<<<cdiv(n, 256), 256, 0, ps>>>(st, n, P<int>(h->c0Off), P<EntryKey>(h->c0Keys),
                                                       P<int>(h->c0Ids), P<float>(h->c0Val), P<int>(h->c0Ent),
                                                       P<unsigned>(h->a0Keys), P<int>(h->a0Ids), P<float>(h->a0Val));
        // block-entry records by level-0 block (stable: stencil order inside a
        // block, so inside every entry), one bit above the largest block id
        // so the sentinel (all ones) sorts last instead of tying with one;
        // additional rows by vertex, the same way
        const int bb = bit_width((unsigned)h->nFineBlk);
        const int vb = std::max(1, bit_width((unsigned)(nv32 - 1))) + 1;
        if ((rc = rs_sort_pairs(h, P<EntryKey>(h->c0Keys), P<EntryKey>(h->c0KeysS), P<int>(h->c0Ids),
                                P<int>(h->c0IdsS), (int)ubD, bb, ps, "level-0 contact record sort", true)) ||
            (rc = rs_sort_pairs(h, P<unsigned>(h->a0Keys), P<unsigned>(h->a0KeysS), P<int>(h->a0Ids),
                                P<int>(h->a0IdsS), (int)ubA, vb, ps, "level-0 contact row sort", true)))
            return rc;
        k_block_bounds<<<cdiv(ubD + 1, 256), 256, 0, ps>>>((int)ubD, h->nFineBlk, P<EntryKey>(h->c0KeysS),
                                                          P<int>(h->cFineOff));
        k_fold_runs<NodeRow, true, unsigned><<<cdiv(ubA, 64), 64, 0, ps>>>(
            (int)ubA, 0xffffffffu, P<unsigned>(h->a0KeysS), P<int>(h->a0IdsS), P<float>(h->a0Val),
            NodeRow{P<float>(h->add0)});
        fa.coff = P<int>(h->cFineOff);
        fa.cids = P<int>(h->c0IdsS);
        fa.cent = P<int>(h->c0Ent);
        fa.cvals = P<float>(h->c0Val);
    } else {  // no contacts: add0 zeroed only
        k_contact0_init<<<1024, 256, 0, ps>>>(nullptr, -1, nullptr, P<float4>(h->add0), (size_t)nv32 * 9 / 4, nullptr,
                                              nullptr, 0, nullptr, nullptr, 0);
    }
    // earlyOd (env MAS_EARLY_OD; default for a sharded Prepare): od and the
    // record counts need only level-0 data too and can run here, ahead of the
    // fused kernel, instead of on the caller's reserved CUs.  Unsharded that
    // delays the fused kernel, the longer path; a shard's fused kernel is 1/world
    // of the blocks and the replicated coarse chain is the longer path, which
    // then no longer carries od: world-8 rank at 1M + contacts 1.40-1.43 ->
    // 1.37-1.39 ms (profiles/round4/prepare/shard_sweep/)
    // A sharded Prepare (world > 1, L >= 2): od of its own vertices only --
    // all the coarse split needs (coarse_split.hip); when the split turns out
    // to cut a subtree, run_assemble adds the others'.  Record counts of the
    // other vertices are zero then (no records of theirs are built).
    h->odDone = false;
    if (early_od(h)) {
        const bool own = h->prepWorld > 1 && h->L > 1;
        h->odV0 = own ? 32 * h->fineBlk0 : 0;
        h->odV1 = own ? std::min(32 * h->fineBlk1, nV) : nV;
        if ((rc = hip_check(h, hipMemsetAsync(P<int>(h->recCnt) + (own ? 0 : nV), 0, own ? (size_t)(nV + 1) * 4 : 4, ps),
                            "memset recCnt")))
            return rc;
        launch_od(h, fa, ps, h->odV0, h->odV1);
        h->odDone = true;
    }
    if ((rc = hip_check(h, hipEventRecord(h->evAdd0, ps), "add0 ready"))) return rc;
    h->earlyFused = true;
    h->earlyFa = fa;
    return h->fusedAfterLevels ? MAS_OK : launch_level0_fused(h, nullptr);
}

// the fused kernel on prepStream; s (not null): after everything s has queued
// (the level build, MAS_FUSED_AFTER_LEVELS)
int launch_level0_fused(mas_context* h, hipStream_t s) {
    static const bool serial = std::getenv("MAS_PREP_SERIAL") && std::atoi(std::getenv("MAS_PREP_SERIAL"));
    int rc;
    hipStream_t ps = serial && s ? s : h->prepStream;
    if (s && ps != s &&
        ((rc = hip_check(h, hipEventRecord(h->evPrepFork, s), "fork")) ||
         (rc = hip_check(h, hipStreamWaitEvent(ps, h->evPrepFork, 0), "fork wait"))))
        return rc;
    if ((rc = hip_check(h, hipEventRecord(h->evFine[0], ps), "record")) ||
        (rc = launch_factor_fused(h, h->earlyFa, h->fineBlk0, h->fineBlk1, ps)) ||
        (rc = hip_check(h, hipEventRecord(h->evFine[1], ps), "record")) ||
        (rc = hip_check(h, hipEventRecord(h->evPrepJoin, ps), "join")))
        return rc;
    return MAS_OK;
}

int run_assemble(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, hipStream_t s) {
    const int nV = h->nV, L = h->L, tc = h->totalClusters;
    int rc;
    const bool fused = h->factorVariant >= 4;
    // the fused factor never stores level-0 blocks unless asked to keep them
    h->denseFine = !fused || h->cfg.keep_blocks;
    const int nStored = h->denseFine ? h->nBlk : h->nBlk - h->nFineBlk;
    const size_t denseBytes = (size_t)std::max(nStored, 1) * kDenseFloats * 4;
    if (h->earlyPlanned && h->inv.bytes < (size_t)h->nBlk * kBlockFloats * 4) {
        // the fused kernel is writing the level-0 inverses into inv: let it
        // finish, then grow inv keeping them (first Prepare of a hierarchy
        // with more coarse blocks than run_level0_early reserved)
        Buffer grown;
        if ((rc = finish_early(h)) || (rc = hip_check(h, hipStreamSynchronize(h->prepStream), "prepare stream")) ||
            (rc = hip_check(h, hipMalloc(&grown.p, (size_t)h->nBlk * kBlockFloats * 4), "hipMalloc inv")))
            return rc;
        grown.bytes = (size_t)h->nBlk * kBlockFloats * 4;
        if ((rc = hip_check(h, hipMemcpyAsync(grown.p, h->inv.p, (size_t)h->nFineBlk * kBlockFloats * 4,
                                              hipMemcpyDeviceToDevice, s), "keep level-0 inverses")) ||
            (rc = hip_check(h, hipStreamSynchronize(s), "grow inv")))
            return rc;
        hipFree(h->inv.p);
        h->inv = grown;
    }
    if ((rc = ensure(h, h->dense, denseBytes)) || (rc = ensure(h, h->inv, (size_t)h->nBlk * kBlockFloats * 4)) ||
        (rc = ensure(h, h->additional, (size_t)(tc + 1) * 36)) ||
        (rc = ensure(h, h->od, (size_t)nV * 36)) || (rc = ensure(h, h->recCnt, (size_t)(nV + 1) * 4)) ||
        (rc = ensure(h, h->recOff, (size_t)(nV + 1) * 4)) || (rc = ensure(h, h->tab, (size_t)(tc + 1) * 36)))
        return rc;
    // level-0 blocks are written whole (or never stored): zero only the coarse blocks
    const size_t zeroFrom = h->denseFine ? (size_t)h->nFineBlk * kDenseFloats * 4 : 0;
    const size_t coarseBytes = (size_t)(h->nBlk - h->nFineBlk) * kDenseFloats * 4;
    if ((coarseBytes > 0 &&
         (rc = hip_check(h, hipMemsetAsync(static_cast<char*>(h->dense.p) + zeroFrom, 0, coarseBytes, s),
                         "memset dense"))) ||
        (rc = hip_check(h, hipMemsetAsync(h->additional.p, 0, (size_t)(tc + 1) * 36, s), "memset additional")) ||
        (!(h->earlyPlanned && early_od(h)) &&  // else od / record counts come from the early path
         (rc = hip_check(h, hipMemsetAsync(h->recCnt.p, 0, (size_t)(nV + 1) * 4, s), "memset recCnt"))))
        return rc;
    float* dense = dense_base(h);
    float* add = P<float>(h->additional);
    const int* gn = P<int>(h->goingNext);
    FineContacts fc{};
    // level-0 additional rows: add0 when run_level0_early built them (its
    // pointer is read only after the worker is joined: the worker allocates it)
    FineAsm fa{nV, h->maxNbr, P<int>(h->s2o), P<int>(h->nbrNum), P<int>(h->nbr), d_diag9, d_off9, d_ranges,
               h->earlyPlanned ? nullptr : add, nullptr, nullptr, nullptr, nullptr,
               h->cfg.keep_blocks ? dense : nullptr};
    bool forked = false;
    if (h->nStencil && (rc = run_contacts(h, s, fc, fa, forked))) return rc;
    // With the records cached, their fold (off-diagonal coarse entries only:
    // a record's nodes differ at its level) needs nothing od, k_diag1 or the
    // table folds (diagonal entries) produce: it can run on a side stream
    // beside them, after the contacts' records (added first, as the
    // reference), joining before the coarse factor.  A sharded Prepare, whose
    // critical path is this chain: world-8 rank at 1M + contacts 1.33-1.36 ->
    // 1.28-1.29 ms; unsharded, where the fused level-0 kernel is as long, the
    // side fold slows that kernel (1.83 -> 1.90 ms) and Prepare 2.35-2.37 ->
    // 2.36-2.41 (profiles/round5/ab/fold_side/), so it stays in line there.
    const bool sideWanted = h->foldSide > 0 || (h->foldSide < 0 && h->prepWorld > 1);
    // the cached records are the own vertices' of a shard (coarse split) or everyone's
    const long long shardKey = h->splitClean ? ((long long)h->prepRank << 32) + h->prepWorld : 0;
    const bool recsValid = h->hierCache && h->recHierId == h->hierId && !h->rangesChanged && h->recShardKey == shardKey;
    const bool sideFold = L > 1 && sideWanted && recsValid && h->nRecCached > 0;
    if (sideFold) {
        if (!h->foldStream && ((rc = hip_check(h, hipStreamCreateWithFlags(&h->foldStream, hipStreamNonBlocking),
                                               "fold stream")) ||
                               (rc = hip_check(h, hipEventCreateWithFlags(&h->evFoldFork, hipEventDisableTiming),
                                               "fold event")) ||
                               (rc = hip_check(h, hipEventCreateWithFlags(&h->evFoldJoin, hipEventDisableTiming),
                                               "fold event")) ||
                               (rc = hip_check(h, hipEventCreateWithFlags(&h->evDiag1, hipEventDisableTiming),
                                               "fold event")) ||
                               (rc = hip_check(h, hipEventCreateWithFlags(&h->evPreJoin, hipEventDisableTiming),
                                               "fold event"))))
            return rc;
        const RecKey rk0{h->levelSize[3], bit_width((unsigned)(tc - h->levelSize[3]))};
        if ((rc = hip_check(h, hipEventRecord(h->evFoldFork, s), "fold fork")) ||
            (rc = hip_check(h, hipStreamWaitEvent(h->foldStream, h->evFoldFork, 0), "fold fork wait")))
            return rc;
        k_fold_runs<DenseEntry, true, EntryKey><<<cdiv(h->nRecCached, 64), 64, 0, h->foldStream>>>(
            h->nRecCached, rk0.dead(), P<EntryKey>(h->recKeysSorted), P<int>(h->recIdsSorted), d_off9,
            DenseEntry{dense, rk0});
        if ((rc = hip_check(h, hipEventRecord(h->evFoldJoin, h->foldStream), "fold join"))) return rc;
    }
    if (fused) {
        // the level-0 blocks assemble and factor on prepStream while this
        // stream assembles the coarse levels (run_factor joins); the early
        // path's worker has queued its part by now (its state is read below)
        if ((rc = finish_early(h))) return rc;
        if (h->earlyPlanned) fa.additional = P<float>(h->add0);
        if (h->earlyFused) {
            // add0 (and od, earlyOd) from the early path (run_level0_early)
            if ((rc = hip_check(h, hipStreamWaitEvent(s, h->evAdd0, 0), "wait add0"))) return rc;
        } else if (!forked && (rc = fork_fused(h, fa, s))) {
            return rc;
        }
        // od: the rows this Prepare assembles need it for their vertices
        // (a sharded Prepare with the coarse split: its own; else all)
        const int v0 = h->splitClean ? h->own.lo[0] : 0, v1 = h->splitClean ? h->own.hi[0] : nV;
        if (!h->odDone) {
            launch_od(h, fa, s, v0, v1);
        } else {  // the early path covered [odV0, odV1)
            launch_od(h, fa, s, v0, std::min(v1, h->odV0));
            launch_od(h, fa, s, std::max(v0, h->odV1), v1);
        }
    } else {
        k_level0_block<<<h->nFineBlk, 64, 0, s>>>(nV, L, P<int>(h->s2o), P<int>(h->nbrNum), P<int>(h->nbr), d_diag9,
                                                  d_off9, d_ranges, add, dense, P<float>(h->od), P<int>(h->recCnt),
                                                  fc, h->fineBlk0, h->fineBlk1);
    }
    if (L == 1) return hip_check(h, hipGetLastError(), "assembly kernels");

    // Coarse edge records, their stable sort and the diagTable term lists
    // depend only on the hierarchy and the CSR structure, not on any value: a
    // Prepare whose hierarchy is the one they were built for (and whose CSR
    // ranges equal the ones they index off9 with) reuses them and only folds.
    const bool cached = recsValid;
    h->recHierId = ~0ull;  // valid again only once rebuilt below
    // the banks / nodes per level this Prepare folds (a shard's own, or all)
    const int bank0 = h->splitClean ? h->own.lo[0] / 32 : 0;
    const int bank1 = h->splitClean ? cdiv(h->own.hi[0], 32) : h->nFineBlk;
    auto nodeRange = [&](int l, int& local0, int& cnt) {
        const int begin = h->levelSize[2 * l + 1], count = h->levelSize[2 * l];
        local0 = h->splitClean ? h->own.lo[l] - begin : 0;
        cnt = h->splitClean ? h->own.hi[l] - h->own.lo[l] : count;
    };
    EdgeRec* rec = P<EdgeRec>(h->rec);
    const RecKey rk{h->levelSize[3], bit_width((unsigned)(tc - h->levelSize[3]))};
    if (rk.bits() > 32) return fail(h, MAS_ERR_ARG, "record keys: more than 2^27 coarse nodes");
    // lanes per vertex: the largest neighbour count (slot 0 is the vertex), rounded to a power of two
    const int valence = h->maxNbr - 1;
    const int lanesPerVertex = valence <= 8 ? 8 : valence <= 16 ? 16 : valence <= 32 ? 32 : 64;
    if (valence > 64) return fail(h, MAS_ERR_ARG, "more than 64 neighbours per vertex");
    if (cached) {
        const int nRec = h->nRecCached;
        if (nRec > 0 && !sideFold)
            k_fold_runs<DenseEntry, true, EntryKey><<<cdiv(nRec, 64), 64, 0, s>>>(
                nRec, rk.dead(), P<EntryKey>(h->recKeysSorted), P<int>(h->recIdsSorted), d_off9,
                DenseEntry{dense, rk});
        if (bank1 > bank0)
            k_diag1<<<cdiv(bank1 - bank0, 256), 256, 0, s>>>(nV, gn, P<float>(h->od), dense, bank0, bank1);
        // The coarse split's level-1 blocks that only this rank has rows in are
        // complete now (contacts, the records' fold, k_diag1: the table folds
        // write level >= 2 diagonals only), so their factor runs on the side
        // stream beside the table folds, whose level-3 fold is one node's
        // dependent chain (~0.1 ms at 1M) however the rows are split
        if (sideFold && h->splitPlanned && h->splitPre.size() == 2 && L > 2) {
            if ((rc = hip_check(h, hipEventRecord(h->evDiag1, s), "diag1 done")) ||
                (rc = hip_check(h, hipStreamWaitEvent(h->foldStream, h->evDiag1, 0), "pre-factor wait")) ||
                (rc = factor_blocks(h, h->splitPre[0], h->splitPre[1], h->foldStream)) ||
                (rc = hip_check(h, hipEventRecord(h->evPreJoin, h->foldStream), "pre-factor join")))
                return rc;
            h->preFactored = true;
        }
        for (int l = 2; l < L; ++l) {
            const int count = h->levelSize[2 * l], begin = h->levelSize[2 * l + 1];
            const int beginPrev = h->levelSize[2 * (l - 1) + 1];
            int local0 = 0, cnt = 0;
            nodeRange(l, local0, cnt);
            if (cnt > 0)
                table_fold(cnt, l, count, begin, beginPrev, P<int>(h->vlistL[l]), P<int>(h->voffL[l]),
                           P<int>(h->termOffL[l]), P<int>(h->termsL[l]), P<int>(h->cst) + (size_t)(l - 2) * nV, gn,
                           d_off9, P<float>(h->od), P<float>(h->tab), dense, local0, s);
        }
        h->recHierId = h->hierId;
        h->recShardKey = shardKey;
        if (sideFold && (rc = hip_check(h, hipStreamWaitEvent(s, h->evFoldJoin, 0), "fold join wait"))) return rc;
        return hip_check(h, hipGetLastError(), "assembly kernels");
    }

    // coarse edge records in (u, k) order
    if ((rc = exclusive_scan(h, P<int>(h->recCnt), P<int>(h->recOff), nV + 1, s, "record scan"))) return rc;
    int nRec = 0;
    if ((rc = read_back(h, s, {P<int>(h->recOff) + nV}, &nRec))) return rc;
    const size_t nr = nRec > 0 ? nRec : 1;
    if ((rc = ensure(h, h->rec, nr * sizeof(EdgeRec))) || (rc = ensure(h, h->recKeys, nr * 4)) ||
        (rc = ensure(h, h->recKeysSorted, nr * 4)) || (rc = ensure(h, h->recIds, nr * 4)) ||
        (rc = ensure(h, h->recIdsSorted, nr * 4)) || (rc = ensure(h, h->recRanges, (size_t)(nV + 1) * 4)))
        return rc;
    rec = P<EdgeRec>(h->rec);
    // the ranges these records index off9 with (k_hier_check compares the next Prepare's)
    if ((rc = hip_check(h, hipMemcpyAsync(h->recRanges.p, d_ranges, (size_t)(nV + 1) * 4, hipMemcpyDeviceToDevice, s),
                        "keep ranges")))
        return rc;
    // the vertices whose records are built (their counts are zero elsewhere)
    const int rv0 = h->splitClean ? h->own.lo[0] : 0, rv1 = h->splitClean ? h->own.hi[0] : nV;
    auto recordLaunch = [&](auto gtag) {
        constexpr int G = decltype(gtag)::value;
        k_records<G><<<cdiv((long long)(rv1 - rv0) * G, 256), 256, 0, s>>>(
            nV, L, rk, P<int>(h->s2o), P<int>(h->nbrNum), P<int>(h->nbr), gn, d_ranges, P<int>(h->recOff), rec,
            P<EntryKey>(h->recKeys), P<int>(h->recIds), rv0, rv1);
    };
    switch (lanesPerVertex) {
        case 8:
            if (rv1 > rv0)
                k_records_vertex<<<cdiv(rv1 - rv0, 256), 256, 0, s>>>(
                    nV, L, rk, P<int>(h->s2o), P<int>(h->nbrNum), P<int>(h->nbr), gn, d_ranges, P<int>(h->recOff), rec,
                    P<EntryKey>(h->recKeys), P<int>(h->recIds), rv0, rv1);
            break;
        case 16: recordLaunch(std::integral_constant<int, 16>{}); break;
        case 32: recordLaunch(std::integral_constant<int, 32>{}); break;
        default: recordLaunch(std::integral_constant<int, 64>{}); break;
    }
    if (nRec > 0) {
        if ((rc = sort_pairs(h, P<EntryKey>(h->recKeys), P<EntryKey>(h->recKeysSorted),
                             P<int>(h->recIds), P<int>(h->recIdsSorted), nRec, rk.bits(), s, "record sort")))
            return rc;
        k_fold_runs<DenseEntry, true, EntryKey><<<cdiv(nRec, 64), 64, 0, s>>>(
            nRec, rk.dead(), P<EntryKey>(h->recKeysSorted), P<int>(h->recIdsSorted), d_off9,
            DenseEntry{dense, rk});
    }
    if (bank1 > bank0)
        k_diag1<<<cdiv(bank1 - bank0, 256), 256, 0, s>>>(nV, gn, P<float>(h->od), dense, bank0, bank1);

    // diagTable folds, levels 2..L-1 (term lists kept per level for the next Prepare)
    if ((rc = ensure(h, h->vkeys, (size_t)nV * 4)) || (rc = ensure(h, h->termCnt, (size_t)(nV + 1) * 4))) return rc;
    for (int l = 2; l < L; ++l) {
        const int count = h->levelSize[2 * l], begin = h->levelSize[2 * l + 1];
        const int beginPrev = h->levelSize[2 * (l - 1) + 1];
        const int* cstPrev = P<int>(h->cst) + (size_t)(l - 1) * nV;  // level-l local id per vertex
        const int* cstPrev2 = P<int>(h->cst) + (size_t)(l - 2) * nV; // level-(l-1) local id per vertex
        if ((rc = ensure(h, h->vlistL[l], (size_t)nV * 4)) || (rc = ensure(h, h->voffL[l], (size_t)(nV + 1) * 4)) ||
            (rc = ensure(h, h->termOffL[l], (size_t)(nV + 1) * 4)) ||
            (rc = ensure(h, h->termsL[l], ((size_t)nRec + nV) * 4)))
            return rc;
        int* vlist = P<int>(h->vlistL[l]);
        int* voff = P<int>(h->voffL[l]);
        int* termOff = P<int>(h->termOffL[l]);
        int* terms = P<int>(h->termsL[l]);
        // keys are level-l local ids < count: sort only their bits
        const int vbits = std::max(1, bit_width((unsigned)std::max(count - 1, 0)));
        if ((rc = sort_pairs(h, reinterpret_cast<const unsigned*>(cstPrev), P<unsigned>(h->vkeys), P<int>(h->iota),
                             vlist, nV, vbits, s, "vertex-list sort")))
            return rc;
        k_bounds<<<cdiv(nV, 256), 256, 0, s>>>(nV, P<int>(h->vkeys), count, voff);
        k_term_count<<<cdiv(nV + 1, 256), 256, 0, s>>>(l, nV, vlist, P<int>(h->recOff), rec, P<int>(h->termCnt));
        if ((rc = exclusive_scan(h, P<int>(h->termCnt), termOff, nV + 1, s, "term scan"))) return rc;
        switch (lanesPerVertex) {
            case 8:
                k_term_write<<<cdiv(nV, 256), 256, 0, s>>>(l, nV, vlist, P<int>(h->recOff), rec, termOff, terms);
                break;
            case 16:
                k_term_write_lanes<16><<<cdiv(nV * 16, 256), 256, 0, s>>>(l, nV, vlist, P<int>(h->recOff), rec,
                                                                          termOff, terms);
                break;
            case 32:
                k_term_write_lanes<32><<<cdiv(nV * 32, 256), 256, 0, s>>>(l, nV, vlist, P<int>(h->recOff), rec,
                                                                          termOff, terms);
                break;
            default:
                k_term_write_lanes<64><<<cdiv(nV * 64, 256), 256, 0, s>>>(l, nV, vlist, P<int>(h->recOff), rec,
                                                                          termOff, terms);
                break;
        }
        int local0 = 0, cnt = 0;
        nodeRange(l, local0, cnt);
        if (cnt > 0)
            table_fold(cnt, l, count, begin, beginPrev, vlist, voff, termOff, terms, cstPrev2, gn, d_off9,
                       P<float>(h->od), P<float>(h->tab), dense, local0, s);
    }
    h->nRecCached = nRec;
    h->recHierId = h->hierId;
    h->recShardKey = shardKey;
    return hip_check(h, hipGetLastError(), "assembly kernels");
}

}  // namespace mas

int mas_dev_contact_terms(mas_handle h, const float* dir3, const float* stiff, const float* w5, float* out, int n) {
    using namespace mas;
    if (!h || n < 0 || (n > 0 && (!dir3 || !stiff || !w5 || !out))) return MAS_ERR_ARG;
    if (n == 0) return MAS_OK;
    hipSetDevice(h->device);
    Buffer b;
    const size_t inF = (size_t)n * 9, outF = (size_t)n * 234;
    int rc = hip_check(h, hipMalloc(&b.p, (inF + outF) * 4), "hipMalloc");
    if (rc) return rc;
    float* d = static_cast<float*>(b.p);
    hipStream_t s = h->stream;
    if (!(rc = hip_check(h, hipMemcpyAsync(d, dir3, (size_t)n * 12, hipMemcpyHostToDevice, s), "H2D")) &&
        !(rc = hip_check(h, hipMemcpyAsync(d + 3 * n, stiff, (size_t)n * 4, hipMemcpyHostToDevice, s), "H2D")) &&
        !(rc = hip_check(h, hipMemcpyAsync(d + 4 * n, w5, (size_t)n * 20, hipMemcpyHostToDevice, s), "H2D"))) {
        k_contact_terms<<<cdiv(n, 64), 64, 0, s>>>(d, d + 3 * n, d + 4 * n, n, d + inF);
        if (!(rc = hip_check(h, hipGetLastError(), "contact terms")))
            rc = hip_check(h, hipMemcpyAsync(out, d + inF, outF * 4, hipMemcpyDeviceToHost, s), "D2H");
    }
    hipStreamSynchronize(s);
    hipFree(b.p);
    return rc;
}
