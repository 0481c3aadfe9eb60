/*
 * mas_oracle.h -- CPU restatement of the reference MAS preconditioner.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (libmas_amd.so) never links it.
 *
 * Parity status: PARTIALLY PINNED.  The reference's .cpp cannot be built in
 * this image without stand-ins for MSVC headers and a source patch (DESIGN.md
 * section 2), and it ships no tests or golden vectors.  Its headers do build
 * unmodified: Morton codes, Math::Clamp and the value layouts are pinned against
 * them (oracle/ref_headers.cpp -> tests/golden/ref_headers.json,
 * ref_morton.npz).  Level sizes, active block counts and PCG iteration counts
 * are pinned against reference runs recorded in SURVEY.md
 * (tests/golden/known_answers.json); the floating-point phases are unpinned and
 * checked by independent numpy fp64 identities (Galerkin coarse blocks, exact
 * local solves).
 *
 * Every function cites the reference file:line it restates.  Buffer layouts
 * follow the reference: float4 vectors (SeVec3fSimd, 16 B), 3x3 blocks as 9
 * floats column-major (SeMatrix3f, SeMatrix.h:650-682), the packed symmetric
 * inverse with stride 4704 floats per 32-node block (.cpp:1349,1435-1495).
 */
#ifndef MAS_ORACLE_H
#define MAS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_state orc_state;

/* maxLevels: 0 = the reference's natural level count (ComputeLevelNums,
 * .cpp:112-135); otherwise min(natural, maxLevels) -- this is the SURVEY
 * harness override of m_numLevel.
 * nThreads: OpenMP threads for the embarrassingly parallel phases (apply
 * blocks, factor blocks, Morton encode).  Order-sensitive float sums always
 * run serially (== reference at CPU_THREAD_NUM=1). */
orc_state* orc_create(int nV, int nE, int nF, int maxLevels, int nThreads);
void orc_destroy(orc_state* s);
void orc_set_threads(orc_state* s, int nThreads);

/* AllocatePrecoditioner (.cpp:38-65).  pos4: [nV][4] floats (w ignored).
 * CSR adjacency starts[nV+1], idx[starts[nV]] (no self).  edges4/faces4:
 * [nE][4], [nF][4] ints (m_edges/m_faces, only needed for contacts; may be
 * NULL when there are none).  Returns 0 or a negative error. */
int orc_allocate(orc_state* s, const float* pos4, const int* starts, const int* idx,
                 const int* edges4, const int* faces4);

/* PreparePreconditioner (.cpp:67-98).  diag9[nV][9], off9[nnz][9]
 * (column-major 3x3), ranges[nV+1].  ef/ee/vf point to 48-byte EfSet/EeSet/VfSet
 * records (SeCollisionElements.h:33-58); counts arrays hold the total at
 * [nE] / [nE] / [nV] (.cpp:306-308).  Any contact pointer may be NULL if its
 * count is zero.  fixVfBary: 0 = parity mode (B-2, read the 4 bytes after the
 * Float2), 1 = documented formula -(1-b0-b1). */
int orc_prepare(orc_state* s, const float* diag9, const float* off9, const int* ranges,
                const void* ef, const void* ee, const void* vf,
                const unsigned* efC, const unsigned* eeC, const unsigned* vfC, int fixVfBary);

/* Preconditioning (.cpp:100-110): z4[nV][4] = M^-1 r4[nV][4]. */
int orc_apply(orc_state* s, float* z4, const float* r4);

/* ---- introspection (parity checks) ---- */
int orc_num_levels(const orc_state* s);
int orc_natural_levels(const orc_state* s);
int orc_total_clusters(const orc_state* s);
int orc_capacity(const orc_state* s);           /* reference m_totalSz (1.5x rule) */
int orc_max_neighbors(const orc_state* s);
int orc_num_stencils(const orc_state* s);
void orc_level_size(const orc_state* s, int* out); /* (L+1) pairs (x,y) */
void orc_aabb(const orc_state* s, float* lower4, float* upper4);
const uint64_t* orc_morton(const orc_state* s);   /* [nV], by original id */
const int* orc_s2o(const orc_state* s);           /* m_MapperSortedGetOriginal */
const int* orc_o2s(const orc_state* s);           /* m_mapperOriginalGetSorted */
const int* orc_nbr_num(const orc_state* s);       /* m_mappedNeighborsNum [nV] */
const int* orc_nbr(const orc_state* s);           /* m_mappedNeighbors [maxNbr][nV] */
const int* orc_coarse_space_tables(const orc_state* s); /* [L][nV] */
const int* orc_going_next(const orc_state* s);    /* [totalClusters] */
const int* orc_coarse_tables(const orc_state* s); /* [nV][4] (Int4) */
const unsigned* orc_fine_connect_mask(const orc_state* s); /* [nV] after ReorderRealtime */
const int* orc_stencil_index_mapped(const orc_state* s); /* [nStencil][5] */
/* Assembled dense block A (96x96 row-major, after the zero-diagonal ->
 * identity rule of .cpp:1365-1368) and its unpacked symmetric inverse. */
int orc_block_matrix(const orc_state* s, int blk, float* A96);
int orc_block_inverse(const orc_state* s, int blk, float* inv96);
const float* orc_inv_packed(const orc_state* s);  /* [nBlk][4704] reference packing */
const float* orc_mapped_r(const orc_state* s);    /* m_mappedR [capacity][4] after orc_apply */

/* The reference's Morton encode of one normalised point (SeMorton.h:75-86). */
uint64_t orc_morton_encode(float x, float y, float z);
float orc_clamp(float a, float lo, float hi); /* Math::Clamp, SeMath.h:103 */
float orc_min(float a, float b);              /* Math::Min, SeMath.h:101 */
float orc_max(float a, float b);              /* Math::Max, SeMath.h:102 */
/* The contact Hessian terms of one stencil (.cpp:1208-1223) from direction
 * dir3, stiffness and five weights; out[234], column-major 3x3 each: [0, 9)
 * H = OuterProduct(d, d * stiff), [9 + 9 it] H * Square(w[it]) (it < 5),
 * [54 + 9 p] w[a] * w[b] * H and [144 + 9 p] that times 2.0f, pairs p over
 * a < b < 5 in (a, b) order. */
void orc_contact_terms(const float* dir3, float stiff, const float* w5, float* out);

#ifdef __cplusplus
}
#endif
#endif
