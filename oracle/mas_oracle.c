/*
 * mas_oracle.c -- CPU restatement of the reference MAS preconditioner
 * (V-Sekai/preconditioner-for-cloth-and-deformable-body-simulation,
 * SeSchwarzPreconditioner.cpp).  TEST INFRASTRUCTURE ONLY -- see mas_oracle.h.
 *
 * Parity: PARTIALLY PINNED.  Morton codes, Clamp and the value layouts are
 * pinned against the reference's own unmodified headers (oracle/ref_headers.cpp,
 * tests/test_ref_pinned.py); level sizes / block counts against reference runs
 * recorded in SURVEY.md; the .cpp's floating-point phases are unpinned (the
 * .cpp needs MSVC headers and a source patch) and checked by numpy fp64
 * identities.
 *
 * Policy on the reference's defects:
 *   B-1 sort only on the first Allocate (reproduced; orc_allocate re-sorts only
 *       on its first call).
 *   B-2 VF weight reads the 4 bytes after Float2 (reproduced unless fixVfBary).
 *   B-3 EE/VF sets indexed with the set-local index (fixed; identical for
 *       single-type inputs).
 *   B-4 buffers sized from the actual cluster count (fixed).
 *   B-5 PrefixSumLx block prefix uses a correct scan (fixed; identical where
 *       the bug is latent, i.e. every level <= 33 792 nodes).
 *   B-6 only min(L,4)-1 coarse levels are prolonged (reproduced); L > 5 rejected.
 *   B-9 Morton ties broken by vertex index (stable); std::sort leaves them
 *       unspecified.
 *   B-10 all order-sensitive float sums run serially in index order
 *       (== CPU_THREAD_NUM=1); hash-map pushes of PrepareHessian are done in
 *       node-id order.
 * Floating point: compiled with -ffp-contract=off; every place the reference
 * uses _mm256_fmadd_ps is an explicit fmaf().  The scalar remainder of
 * LDLtInverse512 (.cpp:1489 `acc += a*b*r`) is evaluated as fmaf(r, a*b, acc),
 * i.e. the contracted form clang produces for the reference.
 */
#include "mas_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BANK 32
#define TRI_SZ 4704 /* (1 + 96) * 96 / 2 + 16 * 3, .cpp:165,1349 */
#define MAXL 8

typedef struct {
    int n;         /* verextNumPerStencil */
    int nFirst;    /* vertexNumOfFirstPrimitive */
    int index[5];
    float weight[5];
    float stiff;
    float dir[4];
} orc_stencil; /* Stencil, SeCollisionElements.h:60-69 */

struct orc_state {
    int nV, nE, nF;
    int natLevels, L, capacity, nThreads;
    int frameIndex;
    float lower[4], upper[4];
    uint64_t* morton;
    int *s2o, *o2s;
    int maxNbr;
    int *nbrNum, *nbr, *nbrNumRemain, *nbrRemain;
    int *edges4, *faces4;
    /* stencils */
    int nStencil, maxStencil;
    orc_stencil* stencils;
    int* stencilIdx; /* [n][5] Int5 */
    /* level maps */
    int* cst; /* m_CoarseSpaceTables [L][nV] */
    unsigned *fineMask, *nextMask;
    int* prefixOrig;
    int* nextPrefix;
    int* goingNext;
    int goingCap;
    int levelSize[2 * (MAXL + 1)];
    int totalClusters;
    int* coarseTables; /* [nV][4] */
    /* assembly */
    float* h32; /* [32][h32Cols][9] */
    int h32Cols;
    float* additional; /* [h32Cols + 1][9] */
    float* inv;        /* [nBlk][TRI_SZ] */
    int invBlocks;
    /* apply */
    float *mappedR, *mappedZ;
    int rzCap;
};

/* ------------------------------------------------------------------ */
/* small helpers                                                       */
/* ------------------------------------------------------------------ */

static inline int ceil32(int x) { return (x + 31) / 32 * 32; }
static inline float se_min(float a, float b) { return a < b ? a : b; } /* SE_MIN, SePreDefine.h:37 */
static inline float se_max(float a, float b) { return a > b ? a : b; } /* SE_MAX, SePreDefine.h:38 */
/* Math::Clamp = Min(Max(lo, a), hi), SeMath.h:103.  NaN -> hi (B-8). */
static inline float se_clamp(float a, float lo, float hi) { return se_min(se_max(lo, a), hi); }

/* exported for the reference-pinned tests (tests/test_ref_pinned.py) */
float orc_clamp(float a, float lo, float hi) { return se_clamp(a, lo, hi); }
float orc_min(float a, float b) { return se_min(a, b); }
float orc_max(float a, float b) { return se_max(a, b); }
static inline int popc32(unsigned v) { return __builtin_popcount(v); }
static inline int ffs32(unsigned v) { return v ? __builtin_ctz(v) + 1 : 0; } /* Intrinsic::Ffs */
static inline unsigned lanemask_lt(unsigned lane) { return (1u << lane) - 1u; } /* SeIntrinsic.h:154 */

static inline float* H32(orc_state* s, int row, int col) {
    return s->h32 + ((size_t)row * s->h32Cols + col) * 9;
}
static inline void m3_add(float* dst, const float* a) {
    for (int i = 0; i < 9; ++i) dst[i] += a[i];
}

static void* xcalloc(size_t n, size_t sz) {
    void* p = calloc(n ? n : 1, sz);
    if (!p) {
        fprintf(stderr, "mas_oracle: out of memory (%zu x %zu)\n", n, sz);
        abort();
    }
    return p;
}

/* ------------------------------------------------------------------ */
/* Morton code, SeMorton.h:75-101                                      */
/* ------------------------------------------------------------------ */

static uint64_t expand_bits(uint64_t bits) { /* SeMorton.h:94-101 */
    bits = (bits | (bits << 32)) & 0xFFFF00000000FFFFull;
    bits = (bits | (bits << 16)) & 0x00FF0000FF0000FFull;
    bits = (bits | (bits << 8)) & 0xF00F00F00F00F00Full;
    bits = (bits | (bits << 4)) & 0x30C30C30C30C30C3ull;
    return (bits | (bits << 2)) & 0x9249249249249249ull;
}

uint64_t orc_morton_encode(float x, float y, float z) { /* SeMorton.h:75-86 */
    x = se_clamp(x * 2097152.0f, 0.0f, 2097151.0f);
    y = se_clamp(y * 2097152.0f, 0.0f, 2097151.0f);
    z = se_clamp(z * 2097152.0f, 0.0f, 2097151.0f);
    uint64_t xx = expand_bits((uint64_t)x);
    uint64_t yy = expand_bits((uint64_t)y);
    uint64_t zz = expand_bits((uint64_t)z);
    return (xx << 2) + (yy << 1) + zz;
}

/* ------------------------------------------------------------------ */
/* create / destroy                                                    */
/* ------------------------------------------------------------------ */

/* ComputeLevelNums, .cpp:112-135 */
static void compute_level_nums(orc_state* s) {
    const int bankSize = 32;
    int totalSz = 0, nLevel = 1;
    int levelSz = (s->nV + bankSize - 1) / bankSize * bankSize;
    totalSz += levelSz;
    while (levelSz > 32) {
        levelSz /= 32;
        nLevel++;
        levelSz = (levelSz + bankSize - 1) / bankSize * bankSize;
        totalSz += levelSz;
    }
    s->natLevels = nLevel;
    s->capacity = (int)(totalSz * 1.5f);
}

orc_state* orc_create(int nV, int nE, int nF, int maxLevels, int nThreads) {
    if (nV <= 0) return NULL;
    orc_state* s = (orc_state*)xcalloc(1, sizeof(orc_state));
    s->nV = nV;
    s->nE = nE;
    s->nF = nF;
    s->nThreads = nThreads > 0 ? nThreads : 1;
    compute_level_nums(s);
    s->L = s->natLevels;
    if (maxLevels > 0 && maxLevels < s->L) s->L = maxLevels;
    if (s->L > 5) { /* B-6: Int4 coarseTables overflows at L >= 6 */
        free(s);
        return NULL;
    }
    int nv32 = ceil32(nV);
    s->morton = (uint64_t*)xcalloc(nV, sizeof(uint64_t));
    s->s2o = (int*)xcalloc(nV, sizeof(int));
    s->o2s = (int*)xcalloc(nV, sizeof(int));
    s->nbrNum = (int*)xcalloc(nV, sizeof(int));
    s->nbrNumRemain = (int*)xcalloc(nV, sizeof(int));
    s->cst = (int*)xcalloc((size_t)s->L * nV, sizeof(int));
    s->fineMask = (unsigned*)xcalloc(nv32, sizeof(unsigned));
    s->nextMask = (unsigned*)xcalloc(nv32, sizeof(unsigned));
    s->prefixOrig = (int*)xcalloc(nv32 / 32 + 1, sizeof(int));
    s->nextPrefix = (int*)xcalloc(nv32 / 32 + 1, sizeof(int));
    s->goingCap = (s->L + 1) * nv32 + 64;
    s->goingNext = (int*)xcalloc(s->goingCap, sizeof(int));
    s->coarseTables = (int*)xcalloc((size_t)nV * 4, sizeof(int));
    s->maxStencil = nV * 32; /* .cpp:187-188 */
    return s;
}

void orc_set_threads(orc_state* s, int nThreads) { s->nThreads = nThreads > 0 ? nThreads : 1; }

void orc_destroy(orc_state* s) {
    if (!s) return;
    free(s->morton); free(s->s2o); free(s->o2s);
    free(s->nbrNum); free(s->nbr); free(s->nbrNumRemain); free(s->nbrRemain);
    free(s->edges4); free(s->faces4);
    free(s->stencils); free(s->stencilIdx);
    free(s->cst); free(s->fineMask); free(s->nextMask); free(s->prefixOrig); free(s->nextPrefix);
    free(s->goingNext); free(s->coarseTables);
    free(s->h32); free(s->additional); free(s->inv);
    free(s->mappedR); free(s->mappedZ);
    free(s);
}

/* ------------------------------------------------------------------ */
/* Allocate phase, .cpp:38-65, 193-285                                 */
/* ------------------------------------------------------------------ */

static const uint64_t* g_sort_keys; /* qsort comparator context */
static int cmp_morton(const void* a, const void* b) {
    int i = *(const int*)a, j = *(const int*)b;
    uint64_t ki = g_sort_keys[i], kj = g_sort_keys[j];
    if (ki < kj) return -1;
    if (ki > kj) return 1;
    return (i > j) - (i < j); /* B-9: ties by index */
}

int orc_allocate(orc_state* s, const float* pos4, const int* starts, const int* idx,
                 const int* edges4, const int* faces4) {
    const int nV = s->nV;
    if (!pos4 || !starts || !idx) return -1;
    if (edges4 && s->nE > 0) {
        free(s->edges4);
        s->edges4 = (int*)xcalloc((size_t)s->nE * 4, sizeof(int));
        memcpy(s->edges4, edges4, (size_t)s->nE * 16);
    }
    if (faces4 && s->nF > 0) {
        free(s->faces4);
        s->faces4 = (int*)xcalloc((size_t)s->nF * 4, sizeof(int));
        memcpy(s->faces4, faces4, (size_t)s->nF * 16);
    }
    if (s->frameIndex == 0) {
        /* DoAlllocation, .cpp:175-185: maxNeighbours = max valence + 1 */
        int maxN = 0;
        for (int v = 0; v < nV; ++v) {
            int deg = starts[v + 1] - starts[v] + 1;
            if (deg > maxN) maxN = deg;
        }
        s->maxNbr = maxN;
        free(s->nbr);
        free(s->nbrRemain);
        s->nbr = (int*)xcalloc((size_t)maxN * nV, sizeof(int));
        s->nbrRemain = (int*)xcalloc((size_t)maxN * nV, sizeof(int));
    }
    if (s->frameIndex % 17 != 0) return 0; /* B-1: .cpp:49-52 */

    /* ComputeTotalAABB/ComputeAABB, .cpp:193-211; SeAabbSimd.h:51,76-79 */
    float lo[4] = {FLT_MAX, FLT_MAX, FLT_MAX, 0.f}, hi[4] = {-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f};
    for (int v = 0; v < nV; ++v) {
        for (int c = 0; c < 4; ++c) {
            float p = pos4[4 * (size_t)v + c];
            lo[c] = lo[c] < p ? lo[c] : p; /* _mm_min_ps */
            hi[c] = hi[c] > p ? hi[c] : p; /* _mm_max_ps */
        }
    }
    memcpy(s->lower, lo, sizeof lo);
    memcpy(s->upper, hi, sizeof hi);
    float ext[3] = {hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]}; /* Extent(), SeAabbSimd.h:91-94 */

    /* FillSortingData, .cpp:219-235 */
#pragma omp parallel for num_threads(s->nThreads)
    for (int v = 0; v < nV; ++v) {
        const float* p = pos4 + 4 * (size_t)v;
        float tx = (p[0] - lo[0]) / ext[0];
        float ty = (p[1] - lo[1]) / ext[1];
        float tz = (p[2] - lo[2]) / ext[2];
        s->morton[v] = orc_morton_encode(tx, ty, tz);
        s->s2o[v] = v;
    }
    /* DoingSort, .cpp:238-243 (stable tie-break, B-9) */
    g_sort_keys = s->morton;
    qsort(s->s2o, nV, sizeof(int), cmp_morton);
    /* ComputeInverseMapper, .cpp:245-255 */
    for (int v = 0; v < nV; ++v) s->o2s[s->s2o[v]] = v;
    /* MapHessianTable, .cpp:258-285: ELL table [k][vid], slot 0 = self */
    for (int v = 0; v < nV; ++v) {
        int o = s->s2o[v];
        int deg = starts[o + 1] - starts[o];
        s->nbrNum[v] = deg + 1;
        s->nbr[v] = v;
        for (int k = 1; k < deg + 1; ++k) s->nbr[(size_t)k * nV + v] = s->o2s[idx[starts[o] + k - 1]];
    }
    s->frameIndex++;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Prepare: collision stencils, .cpp:287-413                           */
/* ------------------------------------------------------------------ */

static void prepare_collision_stencils(orc_state* s, const void* ef, const void* ee, const void* vf,
                                       const unsigned* efC, const unsigned* eeC, const unsigned* vfC,
                                       int fixVfBary) {
    int efNum = efC ? (int)efC[s->nE] : 0;
    int eeNum = eeC ? (int)eeC[s->nE] : 0;
    int vfNum = vfC ? (int)vfC[s->nV] : 0;
    int total = efNum + eeNum + vfNum;
    if (total > s->maxStencil) {
        total = s->maxStencil;
        printf("stencil size %d exceed max stencils num  %d\n", total, s->maxStencil); /* B-11 */
    }
    free(s->stencils);
    free(s->stencilIdx);
    s->stencils = (orc_stencil*)xcalloc(total, sizeof(orc_stencil));
    s->stencilIdx = (int*)xcalloc((size_t)total * 5, sizeof(int));
    int n = 0;
    const unsigned char* efb = (const unsigned char*)ef;
    const unsigned char* eeb = (const unsigned char*)ee;
    const unsigned char* vfb = (const unsigned char*)vf;
    for (int i = 0; i < total; ++i) {
        orc_stencil st;
        memset(&st, 0, sizeof st);
        if (i < efNum) { /* .cpp:326-354; EfSet {eId@0,fId@4,stiff@8,bary@12[3],normal@32} */
            const unsigned char* p = efb + 48 * (size_t)i;
            int eId, fId;
            float stiff, b[3];
            memcpy(&eId, p + 0, 4);
            memcpy(&fId, p + 4, 4);
            if (eId < 0 || fId < 0) continue;
            memcpy(&stiff, p + 8, 4);
            memcpy(b, p + 12, 12);
            memcpy(st.dir, p + 32, 16);
            const int* e = s->edges4 + 4 * (size_t)eId;
            const int* f = s->faces4 + 4 * (size_t)fId;
            st.n = 5;
            st.nFirst = 2;
            st.index[0] = e[0]; st.index[1] = e[1];
            st.index[2] = f[0]; st.index[3] = f[1]; st.index[4] = f[2];
            st.weight[0] = b[0];
            st.weight[1] = 1.f - b[0];
            st.weight[2] = -b[1];
            st.weight[3] = -b[2];
            st.weight[4] = -(1.f - b[1] - b[2]);
            st.stiff = stiff;
        } else if (i < efNum + eeNum) { /* .cpp:355-380; B-3 fixed: set-local index */
            const unsigned char* p = eeb + 48 * (size_t)(i - efNum);
            int e0, e1;
            float stiff, b[2];
            memcpy(&e0, p + 0, 4);
            memcpy(&e1, p + 4, 4);
            if (e1 < 0 || e0 < 0) continue;
            memcpy(&stiff, p + 8, 4);
            memcpy(b, p + 16, 8);
            memcpy(st.dir, p + 32, 16);
            const int* a = s->edges4 + 4 * (size_t)e0;
            const int* c = s->edges4 + 4 * (size_t)e1;
            st.n = 4;
            st.nFirst = 2;
            st.index[0] = a[0]; st.index[1] = a[1];
            st.index[2] = c[0]; st.index[3] = c[1];
            st.weight[0] = b[0];
            st.weight[1] = 1.f - b[0];
            st.weight[2] = -b[1];
            st.weight[3] = -(1.f - b[1]);
            st.stiff = stiff;
        } else { /* .cpp:381-405; VfSet {vId@0,fId@4,stiff@8,bary@16[2],normal@32} */
            const unsigned char* p = vfb + 48 * (size_t)(i - efNum - eeNum);
            int vId, fId;
            float stiff, b[2], b2;
            memcpy(&vId, p + 0, 4);
            memcpy(&fId, p + 4, 4);
            if (vId < 0 || fId < 0) continue;
            memcpy(&stiff, p + 8, 4);
            memcpy(b, p + 16, 8);
            memcpy(&b2, p + 24, 4); /* B-2: m_bary[2] reads the padding after Float2 */
            memcpy(st.dir, p + 32, 16);
            const int* f = s->faces4 + 4 * (size_t)fId;
            st.n = 4;
            st.nFirst = 3;
            st.index[0] = f[0]; st.index[1] = f[1]; st.index[2] = f[2];
            st.index[3] = vId;
            st.weight[0] = -b[0];
            st.weight[1] = -b[1];
            st.weight[2] = fixVfBary ? -(1.f - b[0] - b[1]) : -(1.f - b2);
            st.weight[3] = 1.f;
            st.stiff = stiff;
        }
        s->stencils[n++] = st; /* slot = AtomicAdd(&m_stencilNum,1), single-thread order */
    }
    s->nStencil = n;
    /* MapCollisionStencilIndices, .cpp:287-302 */
    for (int i = 0; i < n; ++i)
        for (int vi = 0; vi < s->stencils[i].n; ++vi)
            s->stencilIdx[5 * (size_t)i + vi] = s->o2s[s->stencils[i].index[vi]];
}

/* ------------------------------------------------------------------ */
/* Prepare: ReorderRealtime, .cpp:415-1162                             */
/* ------------------------------------------------------------------ */

/* BuildConnectMaskL0, .cpp:447-511 */
static void build_connect_mask_l0(orc_state* s) {
    const int nV = s->nV;
    for (int v = 0; v < nV; ++v) {
        int warp = v / 32, lane = v % 32;
        int num = s->nbrNumRemain[v];
        unsigned msk = 1u << lane;
        int nk = 0;
        for (int k = 0; k < num; ++k) {
            int u = s->nbrRemain[(size_t)k * nV + v];
            if (u / 32 == warp)
                msk |= 1u << (u % 32);
            else
                s->nbrRemain[(size_t)(nk++) * nV + v] = u;
        }
        s->nbrNumRemain[v] = nk;
        s->fineMask[v] = msk;
    }
}

/* BuildCollisionConnection, .cpp:514-563 */
static void build_collision_connection(orc_state* s, unsigned* pConnect, const int* pCoarse) {
    for (int i = 0; i < s->nStencil; ++i) {
        const orc_stencil* st = &s->stencils[i];
        int idx[5];
        unsigned msk[5] = {0, 0, 0, 0, 0};
        for (int it = 0; it < 5; ++it) idx[it] = s->stencilIdx[5 * (size_t)i + it];
        if (pCoarse)
            for (int it = 0; it < st->n; ++it) idx[it] = pCoarse[idx[it]];
        for (int a = 0; a < st->n; ++a)
            for (int b = a + 1; b < st->n; ++b) {
                unsigned my = (unsigned)idx[a], ot = (unsigned)idx[b];
                if (my == ot) continue;
                if (my / BANK == ot / BANK && a < st->nFirst && b >= st->nFirst) {
                    msk[a] |= 1u << (ot % BANK);
                    msk[b] |= 1u << (my % BANK);
                }
            }
        for (int it = 0; it < st->n; ++it)
            if (msk[it]) pConnect[idx[it]] |= msk[it];
    }
}

/* Per-warp bit-BFS closure shared by PreparePrefixSumL0 (.cpp:590-625) and
 * NextLevelCluster (.cpp:917-954). */
static unsigned bfs_closure(const unsigned* cache, unsigned lane, unsigned msk) {
    unsigned visited = 1u << lane;
    while (msk != 0xFFFFFFFFu) {
        unsigned todo = visited ^ msk;
        if (!todo) break;
        unsigned next = (unsigned)ffs32(todo) - 1u;
        visited |= 1u << next;
        msk |= cache[next];
    }
    return msk;
}

/* PreparePrefixSumL0, .cpp:565-628 */
static void prepare_prefix_sum_l0(orc_state* s) {
    const int nV = s->nV, nWarps = (nV + 31) / 32;
    for (int w = 0; w < nWarps; ++w) {
        unsigned cache[32] = {0};
        for (int l = 0; l < 32 && w * 32 + l < nV; ++l) cache[l] = s->fineMask[w * 32 + l];
        int cnt = 0;
        for (unsigned l = 0; l < 32 && (int)(w * 32 + l) < nV; ++l) {
            unsigned m = bfs_closure(cache, l, cache[l]);
            s->fineMask[w * 32 + l] = m;
            if (popc32(m & lanemask_lt(l)) == 0) cnt++;
        }
        s->prefixOrig[w] = cnt;
    }
}

/* Cluster-id assignment of BuildLevel1 (.cpp:630-740) and PrefixSumLx
 * (.cpp:963-1072, B-5 fixed: plain exclusive scan over banks).  masks[0..n)
 * are component masks per 32-node bank, counts[] their leader counts.
 * ids[i] = bankPrefix + rank of the lowest lane of i's component. */
static int assign_cluster_ids(const unsigned* masks, const int* counts, int n, int* ids) {
    int nBanks = (n + 31) / 32, prefix = 0;
    for (int w = 0; w < nBanks; ++w) {
        unsigned elected = 0;
        for (unsigned l = 0; l < 32 && (int)(w * 32 + l) < n; ++l)
            if (popc32(masks[w * 32 + l] & lanemask_lt(l)) == 0) elected |= 1u << l;
        for (unsigned l = 0; l < 32 && (int)(w * 32 + l) < n; ++l) {
            unsigned lead = (unsigned)ffs32(masks[w * 32 + l]) - 1u;
            ids[w * 32 + l] = prefix + popc32(elected & lanemask_lt(lead));
        }
        prefix += counts[w];
    }
    return prefix;
}

/* BuildConnectMaskLx, .cpp:743-871.  The per-component OR (isFullWarp /
 * cacheMsk / elected-lane path) yields, for every level-l node, the OR of the
 * same-bank bits of all its member vertices' remaining neighbours; every member
 * of a level-0 component maps to the same coarse node, so OR-ing per vertex is
 * the same set operation. */
static void build_connect_mask_lx(orc_state* s, int level) {
    const int nV = s->nV;
    const int* prev = s->cst + (size_t)(level - 1) * nV;
    for (int v = 0; v < nV; ++v) {
        unsigned cv = (unsigned)prev[v];
        unsigned msk = 0;
        unsigned kn = (unsigned)s->nbrNumRemain[v], nk = 0;
        for (unsigned k = 0; k < kn; ++k) {
            unsigned u = (unsigned)s->nbrRemain[(size_t)k * nV + v];
            unsigned cu = (unsigned)prev[u];
            if (cv / BANK == cu / BANK)
                msk |= 1u << (cu % BANK);
            else
                s->nbrRemain[(size_t)(nk++) * nV + v] = (int)u;
        }
        s->nbrNumRemain[v] = (int)nk;
        if (msk) s->nextMask[cv] |= msk;
    }
}

/* NextLevelCluster, .cpp:873-961 */
static void next_level_cluster(orc_state* s, int level) {
    const int levelNum = s->levelSize[2 * level];
    const int nBanks = (levelNum + 31) / 32;
    for (int w = 0; w < nBanks; ++w) {
        unsigned cache[32] = {0};
        for (unsigned l = 0; l < 32; ++l) {
            int c = w * 32 + (int)l;
            cache[l] = (1u << l) | (c < levelNum ? s->nextMask[c] : 0u);
        }
        int cnt = 0;
        for (unsigned l = 0; l < 32 && (int)(w * 32 + l) < levelNum; ++l) {
            unsigned m = bfs_closure(cache, l, cache[l]);
            s->nextMask[w * 32 + l] = m;
            if (popc32(m & lanemask_lt(l)) == 0) cnt++;
        }
        s->nextPrefix[w] = cnt;
    }
}

static int reorder_realtime(orc_state* s) {
    const int nV = s->nV, L = s->L, nv32 = ceil32(nV);
    memset(s->levelSize, 0, sizeof s->levelSize);
    /* level 0 -> 1 */
    build_connect_mask_l0(s);
    build_collision_connection(s, s->fineMask, NULL);
    prepare_prefix_sum_l0(s);
    { /* BuildLevel1, .cpp:630-740 */
        int total = assign_cluster_ids(s->fineMask, s->prefixOrig, nV, s->cst);
        for (int v = 0; v < nV; ++v) s->goingNext[v] = s->cst[v] + nv32;
        s->levelSize[2] = total;
        s->levelSize[3] = nv32;
    }
    int* ids = (int*)xcalloc(nv32, sizeof(int));
    for (int level = 1; level < L; ++level) { /* .cpp:427-440 */
        memset(s->nextMask, 0, (size_t)nv32 * sizeof(unsigned));
        build_connect_mask_lx(s, level);
        build_collision_connection(s, s->nextMask, s->cst + (size_t)(level - 1) * nV);
        next_level_cluster(s, level);
        /* PrefixSumLx, .cpp:963-1072 */
        const int levelNum = s->levelSize[2 * level];
        const int levelBegin = s->levelSize[2 * level + 1];
        int total = assign_cluster_ids(s->nextMask, s->nextPrefix, levelNum, ids);
        if (levelBegin + ceil32(levelNum) > s->goingCap) {
            free(ids);
            return -3;
        }
        for (int c = 0; c < levelNum; ++c) {
            s->nextMask[c] = (unsigned)ids[c];
            s->goingNext[c + levelBegin] = ids[c] + levelBegin + ceil32(levelNum);
        }
        s->levelSize[2 * (level + 1)] = total;
        s->levelSize[2 * (level + 1) + 1] = levelBegin + ceil32(levelNum);
        /* ComputeNextLevel, .cpp:1074-1084 */
        const int* prev = s->cst + (size_t)(level - 1) * nV;
        int* cur = s->cst + (size_t)level * nV;
        for (int v = 0; v < nV; ++v) cur[v] = (int)s->nextMask[prev[v]];
    }
    free(ids);
    s->totalClusters = s->levelSize[2 * L + 1]; /* TotalNodes, .cpp:1086-1090 */
    /* AggregationKernel, .cpp:1092-1162 (m_denseLevel is never read; omitted) */
    for (int v = 0; v < nV; ++v) {
        int cur = v;
        for (int l = 0; l < 4; ++l) s->coarseTables[4 * (size_t)v + l] = 0;
        for (int l = 0; l < L - 1; ++l) {
            cur = s->goingNext[cur];
            s->coarseTables[4 * (size_t)v + l] = cur;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Prepare: Hessian assembly, .cpp:1164-1345                           */
/* ------------------------------------------------------------------ */

/* The contact terms of one stencil (.cpp:1208-1223), column-major 3x3:
 *   contact_outer   hessian = OuterProduct(d, d * stiff)   SeMatrix.h:352-363,
 *                   SeVector.h:250 (d * stiff lane by lane)
 *   contact_self    hessian * Math::Square(w)              SeMath.h:98, SeMatrix.h:741
 *   contact_pair    w_a * w_b * hessian                    SeMatrix.h:977 (scalar * mat = mat * scalar)
 *   contact_double  t * 2.0f                               .cpp:1190
 * Shared by prepare_collision_hessian and orc_contact_terms (the fixture check
 * against the reference's own headers, tests/test_ref_pinned.py). */
static void contact_outer(const float* dir, float stiff, float* h) {
    const float ds[3] = {dir[0] * stiff, dir[1] * stiff, dir[2] * stiff};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) h[c * 3 + r] = dir[r] * ds[c];
}
static void contact_self(const float* h, float w, float* t) {
    const float w2 = w * w;
    for (int e = 0; e < 9; ++e) t[e] = h[e] * w2;
}
static void contact_pair(const float* h, float wa, float wb, float* t) {
    const float ww = wa * wb;
    for (int e = 0; e < 9; ++e) t[e] = ww * h[e];
}
static void contact_double(const float* t, float* t2) {
    for (int e = 0; e < 9; ++e) t2[e] = t[e] * 2.0f;
}

void orc_contact_terms(const float* dir3, float stiff, const float* w5, float* out) {
    contact_outer(dir3, stiff, out);
    for (int it = 0; it < 5; ++it) contact_self(out, w5[it], out + 9 + 9 * it);
    for (int a = 0, p = 0; a < 5; ++a)
        for (int b = a + 1; b < 5; ++b, ++p) {
            contact_pair(out, w5[a], w5[b], out + 54 + 9 * p);
            contact_double(out + 54 + 9 * p, out + 144 + 9 * p);
        }
}

/* AdditionalSchwarzHessian2, .cpp:1164-1199 */
static void additional_schwarz_hessian2(orc_state* s, const float* h, int v1, int v2) {
    int level = 0;
    unsigned my = (unsigned)v1, ot = (unsigned)v2;
    const int L = s->L;
    while (my / BANK != ot / BANK && level < L) {
        my = (unsigned)s->goingNext[my];
        ot = (unsigned)s->goingNext[ot];
        level++;
    }
    if (level >= L) return;
    m3_add(H32(s, ot % BANK, my), h);
    m3_add(H32(s, my % BANK, ot), h);
    if (level < L - 1) {
        my = (unsigned)s->goingNext[my];
        ot = (unsigned)s->goingNext[ot];
        if (my == ot) {
            float h2[9];
            contact_double(h, h2);
            m3_add(s->additional + 9 * (size_t)my, h2);
        } else {
            m3_add(s->additional + 9 * (size_t)my, h);
            m3_add(s->additional + 9 * (size_t)ot, h);
        }
    }
}

/* PrepareCollisionHessian, .cpp:1201-1227 */
static void prepare_collision_hessian(orc_state* s) {
    for (int i = 0; i < s->nStencil; ++i) {
        const orc_stencil* st = &s->stencils[i];
        const int* idx = s->stencilIdx + 5 * (size_t)i;
        float h[9]; /* OuterProduct(d, d*stiff), SeMatrix.h:352-363; column-major */
        contact_outer(st->dir, st->stiff, h);
        for (int it = 0; it < st->n; ++it) {
            float t[9];
            contact_self(h, st->weight[it], t);
            m3_add(s->additional + 9 * (size_t)idx[it], t);
        }
        for (int a = 0; a < st->n; ++a)
            for (int b = a + 1; b < st->n; ++b) {
                float t[9];
                contact_pair(h, st->weight[a], st->weight[b], t);
                additional_schwarz_hessian2(s, t, idx[a], idx[b]);
            }
    }
}

/* PrepareHessian, .cpp:1229-1345 */
static void prepare_hessian(orc_state* s, const float* diag9, const float* off9, const int* ranges) {
    const int nV = s->nV, L = s->L, nVC = ceil32(nV), tc = s->totalClusters;
    /* coarse additional terms -> own diagonal and every ancestor, .cpp:1236-1252 */
    for (int vid = nVC; vid < tc; ++vid) {
        const float* od = s->additional + 9 * (size_t)vid;
        int my = vid;
        m3_add(H32(s, my % BANK, my), od);
        for (;;) {
            my = s->goingNext[my];
            if (my >= tc) break;
            m3_add(H32(s, my % BANK, my), od);
        }
    }
    /* diagTable[level] of .cpp:1257 as dense per-node arrays */
    float* table = (float*)xcalloc((size_t)(tc + 1) * 9, sizeof(float));
    unsigned char* present = (unsigned char*)xcalloc(tc + 1, 1);
    for (int vid = 0; vid < nV; ++vid) {
        const int vo = s->s2o[vid];
        const int oldNum = s->nbrNum[vid];
        float od[9];
        for (int e = 0; e < 9; ++e) od[e] = diag9[9 * (size_t)vo + e] + s->additional[9 * (size_t)vid + e];
        m3_add(H32(s, vid % BANK, vid), od);
        for (int k = 1; k < oldNum; ++k) {
            const unsigned nb = (unsigned)s->nbr[(size_t)k * nV + vid];
            const float* mat = off9 + 9 * (size_t)(ranges[vo] + k - 1);
            int level = 0;
            unsigned my = (unsigned)vid, ot = nb;
            while (my / BANK != ot / BANK && level < L) {
                level++;
                my = (unsigned)s->goingNext[my];
                ot = (unsigned)s->goingNext[ot];
            }
            if (level >= L) continue;
            m3_add(H32(s, ot % BANK, my), mat);
            if (level == 0) {
                m3_add(od, mat);
            } else if (level + 1 < L) {
                my = (unsigned)s->goingNext[my];
                m3_add(table + 9 * (size_t)my, mat);
                present[my] = 1;
            }
        }
        if (1 < L) {
            int p = s->goingNext[vid];
            m3_add(H32(s, p % BANK, p), od);
            if (2 < L) {
                p = s->goingNext[p];
                m3_add(table + 9 * (size_t)p, od);
                present[p] = 1;
            }
        }
    }
    /* push the level tables upward, .cpp:1326-1343 (node-id order) */
    for (int lv = 2; lv < L; ++lv) {
        const int beg = s->levelSize[2 * lv + 1], end = beg + ceil32(s->levelSize[2 * lv]);
        for (int my = beg; my < end; ++my) {
            if (!present[my]) continue;
            const float* val = table + 9 * (size_t)my;
            m3_add(H32(s, my % BANK, my), val);
            if (lv + 1 < L) {
                int p = s->goingNext[my];
                m3_add(table + 9 * (size_t)p, val);
                present[p] = 1;
            }
        }
    }
    free(table);
    free(present);
}

/* Assemble the dense 96x96 block (.cpp:1357-1377). */
static void load_block(const orc_state* s, int blk, float* A /* [96][96] */) {
    for (int x = 0; x < 32; ++x)
        for (int y = 0; y < 32; ++y) {
            const float* t = s->h32 + ((size_t)y * s->h32Cols + x + blk * 32) * 9;
            int ident = (x == y && t[0] == 0.0f);
            for (int ii = 0; ii < 3; ++ii)
                for (int jj = 0; jj < 3; ++jj)
                    A[(x * 3 + ii) * 96 + y * 3 + jj] = ident ? (ii == jj ? 1.f : 0.f) : t[jj * 3 + ii];
        }
}

/* LDLtInverse512 for one block (.cpp:1357-1495, WIN32 path) */
static void ldlt_inverse_block(const orc_state* s, int blk, float* out /* TRI_SZ */) {
    float A[96][96];
    float diagonal[96];
    load_block(s, blk, &A[0][0]);
    for (int x = 0; x < 96; ++x) { /* elimination, .cpp:1395-1415 */
        float dg = A[x][x];
        float line[96];
        memcpy(line, A[x], sizeof line);
        for (int y = x + 1; y < 96; ++y) {
            if (A[y][x] == 0.0f) continue;
            float r = -A[y][x] / dg;
            for (int c = 0; c < 96; ++c) A[y][c] = fmaf(r, line[c], A[y][c]);
            A[y][x] = r;
        }
    }
    for (int y = 0; y < 96; ++y) { /* .cpp:1419-1433 */
        diagonal[95 - y] = A[y][y];
        A[y][y] = 1.0f;
        for (int x = y + 1; x < (96 < y + 9 ? 96 : y + 9); ++x) A[y][x] = 0.0f;
    }
    for (int i = 0; i < 96; ++i) diagonal[i] = 1.0f / diagonal[i];
    int off = 0;
    for (int it = 0; it < 12; ++it) { /* diagonal, .cpp:1437-1449 */
        int lc = 96 - it * 8;
        for (int j = 0; j < 8; ++j) {
            float acc = 0.f;
            for (int l = 0; l < lc; ++l) {
                float a = A[95 - l][it * 8 + j];
                acc = fmaf(diagonal[l], a * a, acc);
            }
            out[off + it * 8 + j] = acc;
        }
    }
    off += 96;
    for (int it = 0; it < 12; ++it) { /* diagonal strips, .cpp:1451-1469 */
        int xBg = it * 8;
        for (int scan = xBg + 1; scan <= 96 - 8; ++scan) {
            int lc = 96 - scan;
            for (int j = 0; j < 8; ++j) {
                float acc = 0.f;
                for (int l = 0; l < lc; ++l) {
                    float a = A[95 - l][xBg + j], b = A[95 - l][scan + j];
                    acc = fmaf(diagonal[l], a * b, acc);
                }
                out[off + j] = acc;
            }
            off += 8;
        }
    }
    for (int it = 0; it < 12; ++it) /* remainder, .cpp:1475-1495 */
        for (int lane = 0; lane < 7; ++lane) {
            int xBg = it * 8 + lane;
            for (int h = 96 - 7 + lane; h < 96; ++h) {
                int lc = 96 - h;
                float acc = 0.f;
                for (int l = 0; l < lc; ++l) {
                    float a = A[95 - l][xBg], b = A[95 - l][h];
                    acc = fmaf(diagonal[l], a * b, acc);
                }
                out[off++] = acc;
            }
        }
    for (; off < TRI_SZ; ++off) out[off] = 0.f;
}

int orc_prepare(orc_state* s, const float* diag9, const float* off9, const int* ranges,
                const void* ef, const void* ee, const void* vf,
                const unsigned* efC, const unsigned* eeC, const unsigned* vfC, int fixVfBary) {
    const int nV = s->nV;
    if (!diag9 || !off9 || !ranges) return -1;
    if (s->frameIndex == 0) return -4; /* Allocate first */
    /* .cpp:74-75 */
    memcpy(s->nbrRemain, s->nbr, (size_t)s->maxNbr * nV * sizeof(int));
    memcpy(s->nbrNumRemain, s->nbrNum, (size_t)nV * sizeof(int));
    prepare_collision_stencils(s, ef, ee, vf, efC, eeC, vfC, fixVfBary);
    int rc = reorder_realtime(s);
    if (rc) return rc;
    /* B-4: size the dense buffers from the actual cluster count */
    const int tc = s->totalClusters;
    free(s->h32);
    free(s->additional);
    s->h32Cols = tc;
    s->h32 = (float*)xcalloc((size_t)32 * tc * 9, sizeof(float)); /* MemsetZero, .cpp:88 */
    s->additional = (float*)xcalloc((size_t)(tc + 1) * 9, sizeof(float)); /* .cpp:89 */
    prepare_collision_hessian(s);
    prepare_hessian(s, diag9, off9, ranges);
    /* LDLtInverse512, .cpp:1347-1546 */
    const int nBlk = tc / 32;
    free(s->inv);
    s->inv = (float*)xcalloc((size_t)nBlk * TRI_SZ, sizeof(float));
    s->invBlocks = nBlk;
#pragma omp parallel for num_threads(s->nThreads) schedule(dynamic, 4)
    for (int b = 0; b < nBlk; ++b) ldlt_inverse_block(s, b, s->inv + (size_t)b * TRI_SZ);
    /* apply buffers (reference: m_totalSz entries, .cpp:150-151) */
    int cap = s->capacity > tc ? s->capacity : tc;
    if (cap > s->rzCap) {
        free(s->mappedR);
        free(s->mappedZ);
        s->mappedR = (float*)xcalloc((size_t)cap * 4, sizeof(float));
        s->mappedZ = (float*)xcalloc((size_t)cap * 4, sizeof(float));
        s->rzCap = cap;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Apply, .cpp:100-110, 1548-1719                                      */
/* ------------------------------------------------------------------ */

/* SchwarzLocalXSym for one block (.cpp:1612-1693, WIN32 path) */
static void schwarz_local_block(const float* m, const float* R, float* Z) {
    float rhs[96], out[96];
    for (int l = 0; l < 32; ++l)
        for (int c = 0; c < 3; ++c) rhs[l * 3 + c] = R[4 * l + c];
    for (int i = 0; i < 96; ++i) out[i] = m[i] * rhs[i];
    int off = 96;
    for (int it = 0; it < 11; ++it) {
        int xBg = it * 8;
        float sr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int scan = xBg + 1; scan <= 96 - 8; ++scan) {
            const float* mtx = m + off;
            off += 8;
            for (int j = 0; j < 8; ++j) {
                sr[j] = fmaf(mtx[j], rhs[scan + j], sr[j]);
                out[scan + j] = fmaf(mtx[j], rhs[xBg + j], out[scan + j]);
            }
        }
        for (int j = 0; j < 8; ++j) out[xBg + j] = out[xBg + j] + sr[j];
    }
    for (int it = 0; it < 12; ++it)
        for (int lane = 0; lane < 7; ++lane) {
            int xBg = it * 8 + lane;
            float srhs = rhs[xBg], sres = 0.f;
            for (int h = 96 - 7 + lane; h < 96; ++h) {
                float v = m[off++];
                if (v != 0.f) {
                    sres += v * rhs[h];
                    out[h] += v * srhs;
                }
            }
            out[xBg] += sres;
        }
    for (int l = 0; l < 32; ++l) {
        Z[4 * l + 0] = out[l * 3 + 0];
        Z[4 * l + 1] = out[l * 3 + 1];
        Z[4 * l + 2] = out[l * 3 + 2];
        Z[4 * l + 3] = 0.f;
    }
}

int orc_apply(orc_state* s, float* z4, const float* r4) {
    const int nV = s->nV, L = s->L;
    if (!s->inv) return -4;
    float* R = s->mappedR;
    float* Z = s->mappedZ;
    memset(Z, 0, (size_t)s->rzCap * 16); /* .cpp:102-103 */
    memset(R, 0, (size_t)s->rzCap * 16);
    /* BuildResidualHierarchy, .cpp:1548-1598 */
    const int nb = (nV + 31) / 32;
#pragma omp parallel for num_threads(s->nThreads)
    for (int b = 0; b < nb; ++b) {
        for (int lane = 0; lane < 32; ++lane) {
            int v = lane + b * 32;
            if (v >= nV) break;
            const float* r = r4 + 4 * (size_t)s->s2o[v];
            for (int c = 0; c < 4; ++c) R[4 * (size_t)v + c] = r[c];
            if (1 < L) {
                float* dst = R + 4 * (size_t)s->goingNext[v]; /* level-1 parents are warp-local */
                for (int c = 0; c < 4; ++c) dst[c] += r[c];
            }
        }
    }
    if (L > 2) {
        const int bg = s->levelSize[3], n1 = s->levelSize[2];
        for (int vid = bg; vid < bg + n1; ++vid) {
            const float* r = R + 4 * (size_t)vid;
            int nx = vid;
            for (int lv = 2; lv < L; ++lv) {
                nx = s->goingNext[nx];
                for (int c = 0; c < 4; ++c) R[4 * (size_t)nx + c] += r[c];
            }
        }
    }
    /* SchwarzLocalXSym, .cpp:1600-1696 */
    const int nBlk = s->invBlocks;
#pragma omp parallel for num_threads(s->nThreads) schedule(static)
    for (int b = 0; b < nBlk; ++b)
        schwarz_local_block(s->inv + (size_t)b * TRI_SZ, R + (size_t)b * 128, Z + (size_t)b * 128);
    /* CollectFinalZ, .cpp:1698-1719 */
    const int np = (L < 4 ? L : 4);
#pragma omp parallel for num_threads(s->nThreads)
    for (int v = 0; v < nV; ++v) {
        float acc[4];
        for (int c = 0; c < 4; ++c) acc[c] = Z[4 * (size_t)v + c];
        for (int l = 1; l < np; ++l) {
            const float* zz = Z + 4 * (size_t)s->coarseTables[4 * (size_t)v + l - 1];
            for (int c = 0; c < 4; ++c) acc[c] += zz[c];
        }
        memcpy(z4 + 4 * (size_t)s->s2o[v], acc, 16);
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* introspection                                                       */
/* ------------------------------------------------------------------ */

int orc_num_levels(const orc_state* s) { return s->L; }
int orc_natural_levels(const orc_state* s) { return s->natLevels; }
int orc_total_clusters(const orc_state* s) { return s->totalClusters; }
int orc_capacity(const orc_state* s) { return s->capacity; }
int orc_max_neighbors(const orc_state* s) { return s->maxNbr; }
int orc_num_stencils(const orc_state* s) { return s->nStencil; }
void orc_level_size(const orc_state* s, int* out) { memcpy(out, s->levelSize, sizeof(int) * 2 * (s->L + 1)); }
void orc_aabb(const orc_state* s, float* lo, float* hi) {
    memcpy(lo, s->lower, 16);
    memcpy(hi, s->upper, 16);
}
const uint64_t* orc_morton(const orc_state* s) { return s->morton; }
const int* orc_s2o(const orc_state* s) { return s->s2o; }
const int* orc_o2s(const orc_state* s) { return s->o2s; }
const int* orc_nbr_num(const orc_state* s) { return s->nbrNum; }
const int* orc_nbr(const orc_state* s) { return s->nbr; }
const int* orc_coarse_space_tables(const orc_state* s) { return s->cst; }
const int* orc_going_next(const orc_state* s) { return s->goingNext; }
const float* orc_mapped_r(const orc_state* s) { return s->mappedR; }
const int* orc_coarse_tables(const orc_state* s) { return s->coarseTables; }
const unsigned* orc_fine_connect_mask(const orc_state* s) { return s->fineMask; }
const int* orc_stencil_index_mapped(const orc_state* s) { return s->stencilIdx; }
const float* orc_inv_packed(const orc_state* s) { return s->inv; }

int orc_block_matrix(const orc_state* s, int blk, float* A96) {
    if (!s->h32 || blk < 0 || blk >= s->totalClusters / 32) return -1;
    load_block(s, blk, A96);
    return 0;
}

int orc_block_inverse(const orc_state* s, int blk, float* B) {
    if (!s->inv || blk < 0 || blk >= s->invBlocks) return -1;
    const float* m = s->inv + (size_t)blk * TRI_SZ;
    memset(B, 0, 96 * 96 * sizeof(float));
    for (int i = 0; i < 96; ++i) B[i * 96 + i] = m[i];
    int off = 96;
    for (int it = 0; it < 12; ++it) {
        int xBg = it * 8;
        for (int scan = xBg + 1; scan <= 96 - 8; ++scan) {
            for (int l = 0; l < 8; ++l) {
                B[(scan + l) * 96 + xBg + l] = m[off + l];
                B[(xBg + l) * 96 + scan + l] = m[off + l];
            }
            off += 8;
        }
    }
    for (int it = 0; it < 12; ++it)
        for (int lane = 0; lane < 7; ++lane) {
            int xBg = it * 8 + lane;
            for (int h = 96 - 7 + lane; h < 96; ++h) {
                B[h * 96 + xBg] = m[off];
                B[xBg * 96 + h] = m[off];
                off++;
            }
        }
    return 0;
}
