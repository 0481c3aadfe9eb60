/*
 * mas_capi.h -- C ABI of the MI355X-native multilevel additive Schwarz (MAS)
 * preconditioner.  Plain pointers and sizes only; no HIP or torch types.
 *
 * Drop-in boundary.  Each entry point replaces one member of the reference
 * plugin surface (V-Sekai/preconditioner-for-cloth-and-deformable-body-simulation,
 * SeSchwarzPreconditioner.h, namespace SE):
 *
 *   mas_allocate      <- SeSchwarzPreconditioner::AllocatePrecoditioner
 *                        (SeSchwarzPreconditioner.h:56, .cpp:38-65) together
 *                        with the public inputs m_positions / m_edges /
 *                        m_faces / m_neighbours (SeSchwarzPreconditioner.h:44-51)
 *   mas_prepare       <- SeSchwarzPreconditioner::PreparePreconditioner
 *                        (SeSchwarzPreconditioner.h:59-60, .cpp:67-98)
 *   mas_apply         <- SeSchwarzPreconditioner::Preconditioning
 *                        (SeSchwarzPreconditioner.h:63, .cpp:100-110)
 *   mas_apply_device  <- same, on device-resident vectors (the benchmarked path)
 *
 * Memory layouts are the reference's:
 *   vectors  float[4] per vertex (SeVec3fSimd, 16 B, w ignored on input,
 *            written 0 on output)                   SeVectorSimd.h:45-57
 *   3x3      float[9] column-major (SeMatrix3f)     SeMatrix.h:650-682
 *   Int4     int[4]                                 SeVector.h:395
 *   contact  48-byte EfSet / EeSet / VfSet records  SeCollisionElements.h:33-58
 *   counts   unsigned[], only the total at [nE] / [nE] / [nV] is read
 *                                                   .cpp:306-308
 *
 * All functions return MAS_OK (0) or a negative mas_status.  A handle is not
 * thread-safe (neither is the reference object).  Host-pointer functions
 * synchronise the handle's stream before returning; *_device functions are
 * asynchronous on the given stream (NULL = the handle's own stream).
 */
#ifndef MAS_CAPI_H
#define MAS_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mas_stats / mas_pcg_result grew (prepare_fine_ms, factor_formation,
 *    first_pass_iterations, replacements) and gained a reserved tail, so later
 *    additions do not change their size again; mas_config.reference_formation;
 *    MAS_ERR_COMM. */
/* 3: MAS_ERR_NOT_SPD; mas_config.reference_restriction; mas_stats' reserved
 *    tail now carries hier_dirty_level, hier_rebuilt, prepare_fine_start_ms,
 *    nonspd_blocks, wait_timeouts (same sizes). */
/* 4: mas_config.strict_spd (from the reserved tail, same size): a non-SPD
 *    pivot fails Prepare only when set; by default Prepare returns MAS_OK,
 *    counts the blocks in mas_stats.nonspd_blocks and leaves a warning in
 *    mas_last_error, as the reference keeps going.  mas_apply_device reports
 *    an earlier apply's coarse give-up (MAS_ERR_HIP) before queueing. */
/* 5: the sharded coarse assembly (mas_prepare_shard_rows / _complete,
 *    mas_set_prepare_allgather; mas_stats.prepare_complete_ms and coarse_split
 *    from the reserved tail, same size); mas_allgather_loopback;
 *    mas_config.host_register (from the reserved tail, same size): opt-in
 *    page-locking of the caller's host arrays. */
#define MAS_ABI_VERSION 5

typedef enum {
    MAS_OK = 0,
    MAS_ERR_ARG = -1,      /* null / out-of-range argument                       */
    MAS_ERR_HIP = -2,      /* HIP runtime failure (see mas_last_error)           */
    MAS_ERR_CAPACITY = -3, /* a size limit was exceeded (stencils, levels, ...)  */
    MAS_ERR_STATE = -4,    /* call order violated (prepare before allocate, ...)  */
    MAS_ERR_LEVELS = -5,   /* more than 5 levels requested (reference B-6)        */
    MAS_ERR_NOMEM = -6,    /* device allocation failed                           */
    MAS_ERR_NO_DEVICE = -7, /* no HIP device / kernels not loadable               */
    MAS_ERR_COMM = -8,      /* the allgather hook / RCCL failed (see mas_last_error) */
    MAS_ERR_NOT_SPD = -9    /* Prepare with mas_config.strict_spd = 1: a block's LDL^T met a zero,
                               negative or non-finite pivot (mas_stats.nonspd_blocks; mas_last_error
                               names the first block).  The reference divides by such pivots unchecked
                               (.cpp:1406,1431); here the handle stays prepared with the same inverses,
                               but the call fails.  Without strict_spd the call returns MAS_OK */
} mas_status;

typedef struct mas_context* mas_handle;
/* an allgather of `bytes` per rank (see mas_shard_apply_device) */
typedef int (*mas_allgather_fn)(const void* send, void* recv, size_t bytes, void* stream, void* user);

typedef struct {
    int max_levels;    /* 0 = reference rule (ComputeLevelNums .cpp:112-135), else min(natural, max_levels) */
    int resort_period; /* 0 = reference behaviour (sort on first Allocate only, B-1); k>0: re-sort every k calls */
    int fix_vf_bary;   /* 0 = parity with reference release build (B-2); 1 = -(1-b0-b1) */
    int device;        /* HIP device ordinal; -1 = current device */
    int keep_blocks;   /* 1 = Prepare also stores the assembled level-0 blocks (mas_get_block_matrix on
                          them; +2.4 GB of HBM traffic at 1M).  0 = the fused level-0 assemble + factor
                          never writes them; only the coarse blocks are kept */
    int reference_formation; /* 0 = every block's inverse Inv = L^-T D^-1 L^-1 (level 0 and coarse) is
                                formed on the matrix cores (default; within 5e-8 of the reference
                                arithmetic, not bitwise);
                                1 = the reference's own operation order on the vector ALUs
                                (.cpp:1437-1495): every inverse bitwise equal to the reference
                                arithmetic, ~0.15 ms more Prepare at 1M */
    int reference_restriction; /* ABI 3.  0 = the level-3 residual is the sum of its children's level-2
                                  residuals in level-2 id order (default: a 32-add chain; R1 and R2 stay
                                  bitwise the reference's, R3 is the same sum associated by level-2
                                  node, z within 1e-5); 1 = the reference's own association
                                  (BuildResidualHierarchy .cpp:1581-1590: every R1 folded into R3 in
                                  level-1 id order, a 1 024-add chain at 1M): the whole residual
                                  hierarchy bitwise the reference arithmetic, ~6 us more per apply */
    int strict_spd;    /* ABI 4.  0 = as the reference, Prepare keeps going over a zero / negative /
                          non-finite pivot: MAS_OK, mas_stats.nonspd_blocks > 0 and a warning in
                          mas_last_error (an SPD but ill-conditioned Hessian can meet one in fp32);
                          1 = such a Prepare fails with MAS_ERR_NOT_SPD */
    int host_register; /* ABI 5.  0 = the host-pointer entry points copy through the runtime's
                          pageable staging (default); 1 = the caller's host arrays are page-locked
                          (hipHostRegister) when the same (pointer, size) comes back a second time,
                          so the copies run at the pinned rate.  With 1 the caller promises that a
                          registered array stays allocated until it passes another array in that
                          argument or destroys the handle, and that it starts on a page boundary
                          with its allocation covering its last page whole (posix_memalign /
                          mmap rounded to pages); an array that does not start on a page is
                          never registered (its pages may be shared with other allocations) */
    int reserved[7];
} mas_config;

typedef struct {
    int num_verts, num_edges, num_faces;
    int num_levels;          /* levels in use */
    int natural_levels;      /* reference ComputeLevelNums */
    int total_clusters;      /* levelSize[L].y: node ids [0, total_clusters) */
    int num_blocks;          /* total_clusters / 32 */
    int num_fine_blocks;     /* ceil(nV / 32) */
    int max_neighbors;       /* max valence + 1 */
    int num_stencils;
    int level_size[2 * 9];   /* (count, begin) for levels 0..num_levels */
    int64_t inv_bytes;       /* bytes of packed inverses on device */
    int64_t device_bytes;    /* total device memory held by the handle */
} mas_info;

typedef struct {
    /* device time (ms) of the most recent call of each phase */
    double allocate_ms, prepare_ms;
    double prepare_levels_ms, prepare_assemble_ms, prepare_factor_ms;
    int64_t apply_calls;       /* applies since mas_create */
    /* averages over the applies recorded while profiling was on (mas_set_profiling),
       measured with HIP events on the apply stream around each kernel group */
    int64_t profiled_applies;
    double apply_ms_avg;       /* apply start -> apply end on the caller stream */
    double pre_fine_ms_avg;    /* before the fine kernel: the coarse levels */
    double fine_ms_avg;        /* the fine-level kernel: gather + level-0 block solves (+ prolongation) -- dominant */
    double post_fine_ms_avg;   /* after it (0 on the single-GPU path: the prolongation is fused) */
    int64_t apply_mode;        /* coarse levels: 2 = restrictions then all solves, two launches
                                  (default); 0 = one launch per level */
    /* Prepare phases: levels = stencils + aggregation; assemble = contacts + the coarse
       assembly (+ the level-0 assembly when unfused); factor = the rest (coarse factor,
       apply tables; + the level-0 factor when unfused).  The fused level-0 assemble +
       factor (default) runs on its own stream beside assemble/factor: prepare_fine_ms
       is its device time (0 when unfused) */
    double prepare_fine_ms;
    int64_t factor_formation;  /* level-0 inverse formation of the last Prepare: 1 = matrix cores
                                  (v_mfma_f32_32x32x2_f32), 0 = vector ALUs in the reference's order */
    /* incremental level maps (ABI 3): the contact-free hierarchy of the current sort is kept; the last
       Prepare's contact stencils changed level hier_dirty_level of it (num_levels: none -- its levels,
       coarse records, term lists and apply tables were reused; -1: not checked, the cache is off) */
    int64_t hier_dirty_level;
    int64_t hier_rebuilt;      /* the last Prepare ran a level build (first Prepare after a sort, or dirty) */
    double prepare_fine_start_ms; /* the fused level-0 kernel's start, after the Prepare's start */
    int64_t nonspd_blocks;     /* the last Prepare: blocks whose factor met a zero / negative / non-finite pivot */
    int64_t wait_timeouts;     /* since mas_create: bounded device waits of the one-launch coarse form that
                                  gave up (that apply's z is then incomplete), read on the handle's own
                                  stream (no device-wide sync).  The apply that gave up is named by
                                  MAS_ERR_HIP from mas_apply / the PCG solve itself, or for mas_apply_device
                                  from the next mas_apply* / PCG call on the handle */
    double prepare_complete_ms; /* ABI 5: device time of the last mas_prepare_shard_complete (unpack + factor) */
    int64_t coarse_split;      /* ABI 5: the last Prepare's coarse assembly: 0 = every row (unsharded),
                                  1 = sharded, own rows only (the split cuts no subtree), 2 = sharded, every
                                  row (the split cuts a subtree); 1 and 2 exchange rows the same way */
    int64_t reserved[1];       /* zero; room for later fields without a size change */
} mas_stats;

/* lifecycle */
int mas_version(void);
int mas_create(mas_handle* out, const mas_config* cfg /* may be NULL */);
int mas_destroy(mas_handle h);
const char* mas_last_error(mas_handle h);

/* AllocatePrecoditioner + the public input members.
 * pos4[nV][4]; CSR nbr_starts[nV+1], nbr_idx[nbr_starts[nV]] (symmetric, no self);
 * edges4[nE][4], faces4[nF][4] (may be NULL when no EF/EE/VF contacts are used).
 * Host pointers; copied. */
int mas_allocate(mas_handle h, int nV, int nE, int nF, const float* pos4, const int* nbr_starts,
                 const int* nbr_idx, const int* edges4, const int* faces4);

/* PreparePreconditioner with host pointers (copied to the device).
 * diag9[nV][9], off9[nnz][9], ranges[nV+1] (== nbr_starts).  ef/ee/vf may be
 * NULL when their count array is NULL or holds 0. */
int mas_prepare(mas_handle h, const float* diag9, const float* off9, const int* ranges, const void* ef,
                const void* ee, const void* vf, const unsigned* ef_counts, const unsigned* ee_counts,
                const unsigned* vf_counts);

/* PreparePreconditioner with device pointers.  The contact records and their
 * count arrays may be host or device pointers (e.g. the output buffers of a
 * GPU collision-detection pass); only the totals are read back. */
int mas_prepare_device(mas_handle h, const float* d_diag9, const float* d_off9, const int* d_ranges,
                       const void* ef, const void* ee, const void* vf, const unsigned* ef_counts,
                       const unsigned* ee_counts, const unsigned* vf_counts, void* stream);

/* Preconditioning(z, r, dim): host vectors [nV][4]. */
int mas_apply(mas_handle h, float* z4, const float* r4);

/* Preconditioning on device vectors d_z4, d_r4 ([nV][4], 16-B aligned).
 * stream: hipStream_t (NULL = handle stream).  Asynchronous. */
int mas_apply_device(mas_handle h, float* d_z4, const float* d_r4, void* stream);

/* ---- GPU-resident PCG, the caller of the apply ----
 * Solves A x = b with preconditioned conjugate gradients on the device, A the
 * Prepare input in the caller's vertex order (diag9[nV], off9[nnz] column-
 * major 3x3, ranges[nV+1] == nbr_starts, with the neighbour ids given to
 * mas_allocate), preconditioned by this handle's MAS (precondition = 1) or
 * not at all (precondition = 0, plain CG).  x: initial guess in, solution out.
 * Stops when the returned x satisfies ||b - A x||_2 <= tol ||b||_2 (fp64
 * evaluation; the fp32 recursive residual only triggers that check, and r is
 * replaced by b - A x whenever it does) or after max_iters iterations.
 * Vectors are [nV][4] fp32 (w written 0); the solution accumulates in fp64
 * and is rounded once at the end; dot products accumulate in fp64 in a fixed
 * order (deterministic).  The reference has no solver: this is the loop its
 * callers run around Preconditioning. */
typedef struct {
    int iterations;       /* iterations performed */
    int converged;        /* true_rel_residual <= tol */
    double rel_residual;  /* ||r||_2 / ||b||_2 as last tested (true residual after a replacement) */
    double true_rel_residual; /* ||b - A x||_2 / ||b||_2 of the returned x, fp64 evaluation */
    double solve_ms;      /* device time from the initial residual to the stop */
    int first_pass_iterations; /* iterations until the recursive residual first met tol (0: never) --
                                  what an fp64 PCG would report; the rest drive the fp32 x below tol */
    int replacements;     /* residual replacements (r = b - A x) performed */
    int reserved[8];      /* zero; room for later fields without a size change */
} mas_pcg_result;
int mas_pcg_solve_device(mas_handle h, const float* d_diag9, const float* d_off9, const int* d_ranges,
                         float* d_x4, const float* d_b4, int max_iters, float tol, int precondition,
                         mas_pcg_result* out, void* stream);
/* The same with host arrays (copied in and out; synchronous). */
int mas_pcg_solve(mas_handle h, const float* diag9, const float* off9, const int* ranges, float* x4,
                  const float* b4, int max_iters, float tol, int precondition, mas_pcg_result* out);
/* Record HIP events around the apply kernels of every mas_apply_device call
 * (up to 4096 applies) and reset the averages in mas_stats. */
int mas_set_profiling(mas_handle h, int enable);
/* ABI 4.  Duration of the level-0 kernel of mas_apply_device alone (gather,
 * block solves, prolongation from the coarse Z of the last apply): n
 * back-to-back launches on `stream` between two HIP events, synchronised;
 * *ms_per_launch = their average.  A timing marker between two kernels holds
 * the second one back by several microseconds, so the per-apply events of
 * mas_set_profiling overstate this kernel; back-to-back launches do not (the
 * roofline source of bench.py).  d_z4 is written as by an apply. */
int mas_profile_fine(mas_handle h, float* d_z4, const float* d_r4, int n, void* stream, double* ms_per_launch);
/* ABI 4.  The same for the coarse levels of mas_apply_device (the launch(es)
 * before the level-0 kernel, in the form the apply uses): n back-to-back
 * applies' coarse work, *ms_per_launch = their average.  Writes the coarse
 * R / Z of the handle (the next apply recomputes them); z is not touched.
 * MAS_ERR_STATE for a shard-prepared handle or at L < 2. */
int mas_profile_coarse(mas_handle h, const float* d_r4, int n, void* stream, double* ms_per_launch);

/* ---- Morton-range sharding across `world` ranks (one process per GPU) ----
 * Rank g owns a contiguous range of level-0 blocks (equal split).  Clusters
 * never leave a level-0 bank, so its level-1 nodes form a contiguous segment
 * [l1_begin, l1_end).  Per apply:
 *   1. mas_apply_shard_restrict: R1 of the own segment -> d_seg[seg_max] float4
 *   2. the caller allgathers every rank's d_seg into d_gathered[world][seg_max]
 *      (RCCL over xGMI; torch.distributed all_gather_into_tensor)
 *   3. mas_apply_shard_finish: coarse levels (own level-1 blocks, all blocks of
 *      levels >= 2) and the own level-0 blocks; writes z for own vertices only.
 * The union of the ranks' z entries is bitwise equal to mas_apply_device. */
typedef struct {
    int rank, world;
    int fine_block_begin, fine_block_end; /* own level-0 blocks */
    int vert_begin, vert_end;             /* own Morton-sorted vertices */
    int l1_begin, l1_end;                 /* own level-1 nodes (level-1 local ids) */
    int seg_max;                          /* padded segment length (max over ranks) */
} mas_shard;

/* Host-only planner (no device needed): nbanks = ceil(nV/32); l1_first[b] =
 * first level-1 local id of level-0 bank b (b < nbanks), l1_first[nbanks] = n1. */
int mas_shard_plan(int nV, const int* l1_first, int rank, int world, mas_shard* out);
/* Sharded Prepare: every later Prepare of this handle assembles
 * and factors only the level-0 blocks of shard `rank` of `world` (the same
 * equal split of blocks as mas_shard_plan) and every coarse block; the level
 * maps and the coarse assembly stay whole (they need every vertex).  Such a
 * handle serves the sharded apply of that shard only; the single-GPU apply,
 * the PCG driver and mas_save_blob then fail with MAS_ERR_STATE.  (0, 1)
 * restores the whole Prepare. */
int mas_set_prepare_shard(mas_handle h, int rank, int world);
/* ABI 5.  The sharded coarse assembly.  A
 * sharded Prepare (world > 1, L >= 2) assembles only the coarse rows whose
 * subtree lies in its Morton range (every row when the equal split cuts a
 * subtree: mas_stats.coarse_split = 2), factors the level-1 blocks only it has
 * rows in, and leaves the rows other ranks need in one device segment:
 *   mas_prepare_shard_rows      -> that segment and its size (the same on
 *                                  every rank: the largest rank's, padded)
 *   caller: allgather the segments into d_gathered[world][seg_bytes]
 *   mas_prepare_shard_complete  -> unpack the other ranks' rows, factor the
 *                                  shared level-1 blocks and every level >= 2
 *                                  block; synchronous; then the handle serves
 *                                  the sharded apply (before it: MAS_ERR_STATE).
 * Every inverse the rank's sharded apply reads is then bitwise the unsharded
 * Prepare's.  The exchange runs inside mas_prepare instead (nothing pending)
 * when the handle has an RCCL communicator of the same rank / world
 * (mas_rccl_init before the Prepare) or an allgather hook registered here
 * (fn NULL: none). */
int mas_set_prepare_allgather(mas_handle h, mas_allgather_fn fn, void* user);
int mas_prepare_shard_rows(mas_handle h, void** d_seg, size_t* seg_bytes);
int mas_prepare_shard_complete(mas_handle h, const void* d_gathered, void* stream);
/* The same plan for a prepared handle. */
int mas_shard_setup(mas_handle h, int rank, int world, mas_shard* out);
int mas_apply_shard_restrict(mas_handle h, int rank, int world, const float* d_r4, float* d_seg4, void* stream);
int mas_apply_shard_finish(mas_handle h, int rank, int world, const float* d_gathered4, const float* d_r4,
                           float* d_z4, void* stream);
/* Overlapped form of step 3.  The level-0 block solves need no
 * exchanged data, so they can run while the allgather is in flight:
 *   3a. mas_apply_shard_fine: own level-0 blocks, z = Z0 for own vertices (no
 *       coarse terms); enqueue it right after the allgather is started;
 *   3b. mas_apply_shard_complete (after the allgather): the coarse levels from
 *       d_gathered, then z += Z1 + Z2 + Z3 for own vertices (CollectFinalZ order).
 * 3a then 3b is bitwise equal to mas_apply_shard_finish. */
int mas_apply_shard_fine(mas_handle h, int rank, int world, const float* d_r4, float* d_z4, void* stream);
int mas_apply_shard_complete(mas_handle h, int rank, int world, const float* d_gathered4, float* d_z4,
                             void* stream);

/* ---- one-call sharded apply with the collective inside the library ----
 * The whole per-rank Preconditioning of a Morton-range shard behind the
 * reference's apply (SeSchwarzPreconditioner.h:63), so a C/C++ simulator that
 * links the library can shard without Python: restrict the own level-1
 * segment, allgather the segments, solve.  By default every step, the
 * collective included, is enqueued on `stream` (a cross-stream hop costs
 * more on MI355X than the overlap it would buy; env
 * MAS_SHARD_MODE=1 / 2 runs the collective on the handle's communication
 * stream beside the level-0 solves instead).  z is written for the rank's own
 * vertices only; the union over ranks is bitwise equal to mas_apply_device.
 * The segment buffers belong to the handle.
 *
 * mas_allgather_fn: enqueue on `stream` (a hipStream_t) an allgather of
 * `bytes` from `send` into `recv` (world x bytes, rank-major) and return 0, or
 * nonzero on failure (reported as MAS_ERR_COMM).  It is called from the
 * calling thread during mas_shard_apply_device; `user` is passed through.
 * allgather may be NULL only when world == 1. */
/* (mas_allgather_fn is declared next to mas_handle above) */
int mas_shard_apply_device(mas_handle h, int rank, int world, mas_allgather_fn allgather, void* user, float* d_z4,
                           const float* d_r4, void* stream);
/* ABI 5.  A one-process stand-in for the collective (tests, per-rank timing
 * on one GPU): copies `send` into slot *(const int*)user of `recv` on
 * `stream`; the other slots are left unchanged.  Pass it as `allgather` with
 * user = &rank. */
int mas_allgather_loopback(const void* send, void* recv, size_t bytes, void* stream, void* user);

/* The same over RCCL (xGMI) with a communicator the handle owns.  RCCL is
 * loaded at run time (librccl.so.1; the one already in the process if any).
 * mas_rccl_unique_id: rank 0 creates the 128-byte id and the caller
 * broadcasts it (any out-of-band channel); every rank then calls
 * mas_rccl_init with it on its own device.  mas_shard_apply_rccl uses the
 * communicator's rank and size. */
int mas_rccl_unique_id(void* id128);
int mas_rccl_init(mas_handle h, const void* id128, int rank, int world);
int mas_shard_apply_rccl(mas_handle h, float* d_z4, const float* d_r4, void* stream);

/* ---- fixture / wire format ----
 * A prepared handle as one versioned, checksummed blob (header "MASBLOB",
 * version 1, FNV-1a 64 over the payload): level sizes, Morton codes, both
 * permutations, CoarseSpaceTables, goingNext, coarseTables, fine connect
 * masks, the apply maps and the packed inverses (630 MB at 1M).  Loading it
 * into any handle makes that handle prepared without Allocate/Prepare inputs
 * (warm start, cross-box golden comparison); mas_apply*, mas_shard_*,
 * mas_get_maps and mas_get_block_inverse work on it, a new Prepare needs
 * mas_allocate first.  Host buffers. */
int mas_blob_size(mas_handle h, size_t* out_bytes);
int mas_save_blob(mas_handle h, void* dst, size_t capacity, size_t* written);
int mas_load_blob(mas_handle h, const void* src, size_t size);
/* Checks a blob without a device or handle: header, checksum, section sizes
 * and that every index map stays inside the level table (FNV-1a detects
 * corruption, not tampering; mas_load_blob runs the same checks first).
 * MAS_OK or MAS_ERR_ARG. */
int mas_blob_validate(const void* src, size_t size);
/* introspection / parity */
int mas_get_info(mas_handle h, mas_info* out);
int mas_get_stats(mas_handle h, mas_stats* out);
/* Level maps, host outputs; any pointer may be NULL.
 * morton[nV] (by original id), s2o[nV], o2s[nV],
 * coarse_space_tables[L*nV], going_next[total_clusters], coarse_tables[nV*4],
 * fine_connect_mask[nV]. */
int mas_get_maps(mas_handle h, uint64_t* morton, int* s2o, int* o2s, int* coarse_space_tables,
                 int* going_next, int* coarse_tables, unsigned* fine_connect_mask);
/* ELL neighbour table [max_neighbors][nV] and counts [nV] (MapHessianTable). */
int mas_get_neighbors(mas_handle h, int* nbr_num, int* nbr);
/* Dense assembled block (96x96 row-major, zero-diagonal -> identity applied)
 * and its inverse unpacked to 96x96. */
int mas_get_block_matrix(mas_handle h, int blk, float* out96x96);
int mas_get_block_inverse(mas_handle h, int blk, float* out96x96);
/* ABI 5.  Blocks [blk0, blk0 + nblk)'s inverses as stored (4 656 floats each,
 * the packed layout of csrc/layout.h), for bitwise comparisons. */
int mas_get_packed_inverses(mas_handle h, int blk0, int nblk, float* out);
/* The residual hierarchy of the most recent single-GPU apply
 * (BuildResidualHierarchy .cpp:1548-1598) as out4[total_clusters - begin_1][4]
 * over coarse node ids begin_1 .. total_clusters-1.  Only levels
 * 1 .. min(L-1, 3) are computed: at L = 5 the level-4 entries are 0 (that
 * level is never prolonged, CollectFinalZ .cpp:1706-1717, so it is skipped),
 * where the reference's m_mappedR holds the sums.  Level 3 is the sum of the
 * level-2 residuals unless mas_config.reference_restriction = 1. */
int mas_get_coarse_residual(mas_handle h, float* out4);
/* Diagnostics of Prepare's building blocks on device buffers (tests): the
 * stable pair sort by the low `bits` key bits and the int exclusive scan, on
 * the handle's stream, synchronised before return.  impl 1 = the library's
 * look-back-free kernels (rsort.hip), 0 = rocprim/hipcub. */
int mas_dev_sort_pairs(mas_handle h, const unsigned* d_keys_in, unsigned* d_keys_out, const int* d_vals_in,
                       int* d_vals_out, int n, int bits, int impl);
int mas_dev_exclusive_scan(mas_handle h, const int* d_in, int* d_out, int n, int impl);
/* The contact Hessian terms the assembly kernels use (.cpp:1190,1208-1223),
 * for n stencils given by direction dir3[n][3], stiffness stiff[n] and five
 * weights w5[n][5] (host arrays): out[n][234], column-major 3x3 each --
 * OuterProduct(d, d * stiff), H * Square(w[it]) for it < 5, and per pair
 * a < b < 5 w[a] * w[b] * H, then the same times 2.0f (tests pin them against
 * the reference's own headers). */
int mas_dev_contact_terms(mas_handle h, const float* dir3, const float* stiff, const float* w5, float* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MAS_CAPI_H */
