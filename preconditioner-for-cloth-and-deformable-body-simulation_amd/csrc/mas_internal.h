// mas_internal.h -- device-side state of one MAS preconditioner handle.
//
// Data layout in HBM (DESIGN.md "Data layout"):
//   * node ids follow the reference numbering: level 0 =
//     Morton-sorted vertices [0, ceil32(nV)), level l >= 1 at
//     [begin_l, begin_l + ceil32(n_l)), total_clusters = begin_L.  A 32-node
//     "bank" is one Schwarz subdomain block; block b = nodes [32b, 32b+32).
//   * vmap[v] (int4, per sorted vertex) = {s2o[v], a1, a2, a3}: the original
//     id and the global ids of the level-1..3 ancestors -- everything the fine
//     apply kernel needs about a vertex in one 16-byte load.
//   * inv: per block 4656 fp32 (18 624 B, the reference's packed size) in the
//     node-pair-rotation layout described in layout.h.
//   * Rc / Zc: coarse residual / solution, float4 per node id >= begin_1.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mas_capi.h"

namespace mas {

constexpr int kBank = 32;
constexpr int kBlockFloats = 4656;      // (96*97)/2 packed symmetric 96x96
constexpr int kBlockF4 = kBlockFloats / 4;  // 1164 float4 per block
constexpr int kMaxLevels = 5;             // reference B-6
constexpr int kDenseFloats = 96 * 96;
constexpr int kProfRing = 4096;          // applies recorded while profiling
constexpr int kCoarseOccBlocks = 4096;   // level-1 blocks from which the coarse launches use their occupancy forms

// Stencil, SeCollisionElements.h:60-69 (device copy; direction xyz only).
struct DevStencil {
    int n, nFirst;
    int idx[5];     // sorted (mapped) vertex ids, MapCollisionStencilIndices .cpp:287-302
    float w[5];
    float stiff;
    float dir[3];
};

// Level 3 (k_coarse.hip): node T's R is folded from R1 over T's
// level-1 descendants in id order, list slots T * stride .. + stride (zero /
// -1 padded); idx[slot] is a position in src (Rc, or the gathered segments of
// a sharded apply), or src is already in list order (deepR1, idx null).
struct DeepArgs {
    const int* idx;
    const float4* src;
    int lv3Begin, stride;
    int* cnt;           // per level-3 block: node arrivals (the last one solves the block)
};

// Level-0 assembly inputs of the fused assemble + factor kernel (k_factor.hip)
// and the od kernel (k_assemble.hip): the CSR Hessian in the sorted vertex
// order's ELL neighbour table, the contact rows (`additional`), and the
// level-0 blocks' contact block-entry records, grouped by block with every
// entry's records in stencil order (a stable sort by block, or by entry).
struct FineAsm {
    int nV, maxNbr;
    const int* s2o;
    const int* nbrNum;
    const int* nbr;
    const float* diag9;
    const float* off9;
    const int* ranges;
    const float* additional;
    const int* coff;                  // per level-0 block: its records [coff[b], coff[b + 1]) (null: no contacts)
    const int* cids;                  // sorted position -> record id
    const int* cent;                  // per record id: (row & 31) * 32 + (col & 31) inside its block
    const float* cvals;               // per record id: the 3x3, column-major
    float* keep;                      // dense base: also store the assembled blocks (null: not kept)
};

// The node rows a sharded Prepare assembles (coarse_split.hip): level l owns
// the global ids [lo[l], hi[l]) (level 0: sorted vertices); level l's ids
// start at begin[l] (begin[l] = INT_MAX for l >= L).  Unsharded: everything.
struct OwnNodes {
    int lo[5], hi[5];
    int begin[5];
    __host__ __device__ bool own(unsigned x) const {
        int l = 0;
#pragma unroll
        for (int k = 1; k < 5; ++k) l += (long long)x >= (long long)begin[k];
        return (int)x >= lo[l] && (int)x < hi[l];
    }
};

// A run of consecutive node rows of the coarse exchange: rows [node0, node0 +
// count) of the dense blocks at rows [seg0, seg0 + count) of a segment.
struct RowPart {
    int node0, count, seg0;
};

struct Buffer {
    void* p = nullptr;
    size_t bytes = 0;
};

// Timing events owned by one host call; destroyed on every return path
// (an event recorded on a stream may be destroyed before it completes).
struct ScopedEvents {
    hipEvent_t e[2] = {nullptr, nullptr};
    ScopedEvents() {
        for (auto& x : e)
            if (hipEventCreate(&x) != hipSuccess) x = nullptr;
    }
    ~ScopedEvents() {
        for (auto& x : e)
            if (x) hipEventDestroy(x);
    }
    ScopedEvents(const ScopedEvents&) = delete;
    ScopedEvents& operator=(const ScopedEvents&) = delete;
    bool ok() const { return e[0] && e[1]; }
};

// A host thread kept for the handle's lifetime that queues Prepare's early
// level-0 path on prepStream while the caller's thread queues the rest
// (prepare.hip).  Creating a thread per Prepare cost ~100 us before its first
// launch (thread start + HIP's per-thread state).  HIP's current device is
// per host thread: every job runs after hipSetDevice(device).
class PrepWorker {
  public:
    explicit PrepWorker(int device) : device_(device), t_([this] { loop(); }) {}
    ~PrepWorker() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        t_.join();
    }
    PrepWorker(const PrepWorker&) = delete;
    PrepWorker& operator=(const PrepWorker&) = delete;
    // job(devOk): devOk = hipSetDevice succeeded on the worker
    void post(std::function<void(bool)> job) {
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = std::move(job);
            busy_ = true;
        }
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return !busy_; });
    }

  private:
    void loop() {
        std::unique_lock<std::mutex> g(m_);
        for (;;) {
            cv_.wait(g, [this] { return stop_ || (busy_ && job_); });
            if (stop_) return;
            std::function<void(bool)> job = std::move(job_);
            job_ = nullptr;
            g.unlock();
            job(hipSetDevice(device_) == hipSuccess);
            g.lock();
            busy_ = false;
            cv_.notify_all();
        }
    }
    int device_;
    std::mutex m_;
    std::condition_variable cv_;
    std::function<void(bool)> job_;
    bool busy_ = false, stop_ = false;
    std::thread t_;  // last: starts after the members above exist
};

}  // namespace mas

struct mas_context {
    mas_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // sizes
    int nV = 0, nE = 0, nF = 0, nnz = 0;
    int natL = 0, L = 0, maxNbr = 0;
    int allocCalls = 0;   // reference m_frameIndex semantics (B-1)
    bool allocated = false, prepared = false, profiling = false;
    bool fromBlob = false;  // restored by mas_load_blob: applies, no Prepare inputs (blob.hip)
    // level-0 factor (env MAS_FACTOR_VARIANT): 4 = k_factor_fused (assembly in
    // LDS slabs + register-blocked factor, one kernel, overlapped with the
    // coarse assembly on prepStream); 2 = k_level0_block + k_factor_rb;
    // 3 = 2 with the MFMA formation (not bitwise); 5 = 4 with the MFMA
    // formation, level 0 and the coarse blocks (not bitwise, the default;
    // mas_config.reference_formation = 1 selects 4); 0 = LDS-row k_factor
    int factorVariant = 5;
    // coarse levels (env MAS_COARSE_MODE): 3 = one launch with tagged
    // hand-offs (k_coarse1.hip, L >= 3); 2 = two launches, restrictions then
    // every solve (k_coarse.hip, L >= 3); 0 = one launch per level.  (The
    // side-stream overlap was measured slower: DESIGN.md section 4.)
    int coarseMode = -1;  // -1: 3 at L = 3 and with the grouped level 3, else 2 (measured)
    // level-3 residual (mas_config.reference_restriction, env MAS_REF_RESTRICT):
    // true = the sum of its children's R2 (default), false = the reference's
    // fold of every R1 in level-1 id order (deep_fold.h)
    bool groupedR3 = true;
    // coarse launches in their occupancy forms (k_coarse.hip): -1 = when the
    // level-1 level has >= kCoarseOccBlocks blocks, 0 = never, 1 = always;
    // env MAS_COARSE_OCC
    int coarseOcc = -1;
    int coarseWide = 0;     // k_solve123 in 512-thread workgroups (env MAS_COARSE_WIDE)
    int coarseNarrow = -1;  // single-wave coarse workgroups: -1 = at L = 3, 0 = never, 1 = always (env MAS_COARSE_NARROW)
    // fine kernel (env MAS_FINE_VARIANT, k_apply.hip): 6 = nontemporal inverse
    // loads, 2-wave workgroups dealt to the XCDs in contiguous chunks; 4 = the
    // same in 4-wave workgroups, 7 in one-wave ones (A/B); 1 = 4 without the
    // chunking (A/B); 3 = 1 in one-wave workgroups (A/B); 0 = default-policy
    // loads (A/B)
    int fineVariant = 6;
    int residentSplit = 0;  // env MAS_RESIDENT_SPLIT (A/B, launch_fine): first K blocks default-policy
    int invResident = -1;  // env MAS_INV_RESIDENT: -1 by size (fine_var, k_apply.hip), 0 / 1 forced
    // blocks (waves) per workgroup of the fine kernel in the PCG's applies,
    // one r.z partial per workgroup, summed by every SpMV workgroup (env
    // MAS_RZ_WPB: 2, 4 or 8): 4 measured 0.8-1.0 us per iteration faster
    // than 2 at 1M + contacts, 8 17 us slower (profiles/round5/ab/pcg_rz_wpb.txt)
    int rzWpb = 4;
    int totalClusters = 0, nBlk = 0, nFineBlk = 0, nStencil = 0;
    int nStencilEF = 0;  // of nStencil, the EF stencils (at most 5 vertices; EE / VF have 4)
    int nBlkPrev = 0;  // nBlk of the previous Prepare, read by the early path's thread (run_levels may change nBlk meanwhile)
    // sharded Prepare (mas_set_prepare_shard): the next Prepare assembles and
    // factors only the level-0 blocks of Morton shard prepRank / prepWorld;
    // [fineBlk0, fineBlk1) = the level-0 blocks the last Prepare factored
    int prepRank = 0, prepWorld = 1, fineBlk0 = 0, fineBlk1 = 0;
    // Sharded coarse assembly (coarse_split.hip): a
    // sharded Prepare assembles only the coarse rows whose subtree lies in its
    // vertex range (own), factors its level-1 blocks no other rank has rows in
    // (pre), exchanges the rows the other ranks need (its rows of level-1
    // blocks shared with a neighbour, every level >= 2 row it owns: parts) and
    // factors the shared level-1 blocks and every level >= 2 block after the
    // exchange (post).  When the equal split cuts a coarse row's subtree the
    // rank assembles every row (splitClean false, same exchange).
    bool splitPlanned = false;   // this Prepare exchanges coarse rows (sharded, L >= 2, fused factor)
    bool splitClean = false;     // ... and assembles only its own rows
    mas::OwnNodes own{};         // the rows this Prepare assembles
    unsigned long long splitHierId = ~0ull;  // the hierarchy / shard the plan below was made for
    int splitRank = -1, splitWorld = 0;
    std::vector<int> splitBnd;   // this rank's row range per level l: [splitBnd[2l], splitBnd[2l + 1])
    std::vector<std::vector<mas::RowPart>> splitParts;  // per rank: its rows in the exchange segment
    int splitSegRows = 0;        // rows per (padded) segment: the largest rank's
    std::vector<int> splitPre, splitPost;  // [begin, end) block ranges factored before / after the exchange
    int splitPackParts = 0, splitPackRows = 0, splitUnpackParts = 0, splitUnpackRows = 0;  // part table (splitPartsDev)
    bool rowsPending = false;    // the exchange of this Prepare has not run yet (mas_prepare_shard_complete)
    int odV0 = 0, odV1 = 0;      // the vertex range the early path's od covered (run_level0_early)
    long long recShardKey = 0;   // the shard the cached coarse records were built for (0: every row)
    mas_allgather_fn prepAllgather = nullptr;  // mas_set_prepare_allgather: the exchange inside Prepare
    void* prepAllgatherUser = nullptr;
    int levelSize[2 * 9] = {};

    // allocate-phase device data
    mas::Buffer pos, starts, idx, edges, faces;
    mas::Buffer morton, mortonSorted, iota, s2o, o2s;
    mas::Buffer nbrNum, nbr, nbrNumRem, nbrRem;
    mas::Buffer aabbPartial;
    // prepare-phase device data
    mas::Buffer rawContacts, stencilFlags, stencilSlots, stencils;
    mas::Buffer fineMask, nextMask, bankCount, bankPrefix, levelTotal;
    mas::Buffer cst, goingNext, vmap, coarseTables;
    // dense: the assembled 96x96 blocks.  Only the coarse blocks are stored
    // unless level-0 blocks are kept (cfg.keep_blocks or an unfused factor
    // variant); denseBase = the address block 0 would have (dense_base()).
    mas::Buffer dense, inv, slotTable, tileSlot, valuSlot;
    bool denseFine = false;  // the last Prepare stored the level-0 blocks
    hipStream_t prepStream = nullptr;  // fused level-0 assemble + factor, beside the coarse assembly
    hipEvent_t evPrepFork = nullptr, evPrepJoin = nullptr;
    hipEvent_t evFine[2] = {nullptr, nullptr};  // timing of the fused level-0 kernel (prepare_fine_ms)
    // early level-0 path (run_level0_early, fused variants): the level-0
    // contact records and additional rows are built on prepStream right after
    // the stencils and the fused kernel starts there, beside the level build;
    // add0 = level-0 additional rows, evAdd0 = they are ready (k_od waits)
    bool earlyFused = false;
    // CUs the fused kernel's queue leaves to the caller's stream (env
    // MAS_PREP_CU_RESERVE; round 4, one box: 0 / 16 / 32 / 48 / 64 -> 3.06 /
    // 3.21 / 2.69 / 2.88 / 2.90 ms).  0 since round 6: a CU-masked queue kept
    // alive beside another process's GPU queues left this process's apply
    // queue unserved (DESIGN.md section 4 "Prepare", round 6)
    int prepCuReserve = 0;
    int fusedChunks = 0;  // the fused kernel's launches (launch_factor_fused): 0 = by size, env MAS_FUSED_CHUNKS
    int fusedAfterLevels = 0;  // A/B (env MAS_FUSED_AFTER_LEVELS): the early fused kernel waits for the level build
    int earlyThread = 1;       // the early path queued from a second host thread (env MAS_EARLY_THREAD)
    std::unique_ptr<mas::PrepWorker> prepWorker;  // that thread (created by the first Prepare that needs it)
    // this Prepare runs the early path (decided before it is queued, so the
    // caller's thread need not wait for the worker to know it); the worker's
    // job is in flight until finish_early(), which returns its status
    bool earlyPlanned = false, earlyPending = false;
    int earlyRc = 0;
    std::string earlyErr;
    int earlyOd = -1;          // k_od in the early path: 1 always, 0 never, -1 (default) by early_od's rule
    bool odDone = false;       // this Prepare's od / record counts are queued already
    mas::FineAsm earlyFa{};    // its inputs, kept for launch_level0_fused
    hipEvent_t evAdd0 = nullptr;
    // the cached CSR records' fold beside od / k_diag1 / the table folds
    // (run_assemble; env MAS_FOLD_SIDE): -1 = for a sharded Prepare only
    int foldSide = -1;
    hipStream_t foldStream = nullptr;
    hipEvent_t evFoldFork = nullptr, evFoldJoin = nullptr;
    // the coarse split's pre level-1 factor, on foldStream beside the table
    // folds (run_assemble); run_prepare joins it last (evPreJoin)
    hipEvent_t evDiag1 = nullptr, evPreJoin = nullptr;
    bool preFactored = false;
    mas::Buffer add0, c0Cnt, c0Off, c0Keys, c0KeysS, c0Ids, c0IdsS, c0Val, a0Keys, a0KeysS, a0Ids, a0IdsS, a0Val;
    mas::Buffer additional, od, recCnt, recOff, rec, recKeys, recKeysSorted, recIds, recIdsSorted;
    mas::Buffer vkeys, tab, termCnt;
    // contact records (k_assemble.hip): block entries (d*), additional rows (a*), pushes (p*)
    mas::Buffer cdCnt, cdOff, cdKeys, cdKeysS, cdIds, cdIdsS, cdVal, cdEnt, cFineOff;
    mas::Buffer c0Ent;  // entry code per level-0 contact record (FineAsm::cent)
    mas::Buffer caCnt, caOff, caKeys, caKeysS, caIds, caIdsS, caVal;
    mas::Buffer cpCnt, cpOff, cpKeys, cpKeysS, cpIds, cpIdsS;
    mas::Buffer Rc, Zc, members, coarseMask, shardOff, shardPos1, l1src;
    mas::Buffer splitDev, prepSeg, prepGathered, splitPartsDev;  // coarse split: bounds + flag, segments, part table
    // Incremental level maps (DESIGN.md section 4 "Prepare").
    // The contact-free ("mesh") hierarchy of the current sort is built once and
    // kept; each Prepare checks on the device whether its contact stencils
    // change it (a pair joining two different mesh components inside a bank at
    // some level, k_hier_check).  If not, the level build is skipped and so is
    // everything derived from the hierarchy alone (coarse edge records and
    // their sort, the diagTable term lists, the apply tables); else the levels
    // are rebuilt with the contacts.  The hierarchy maps live in two slots: the
    // live buffers (cst, goingNext, vmap, coarseTables, fineMask, coarseMask)
    // and a spare set; a dirty Prepare swaps the mesh hierarchy into the spare
    // slot before rebuilding, a clean one swaps it back (no copies).
    mas::Buffer spCst, spGn, spVmap, spCoarseTables, spFine, spCoarseMask;
    bool meshHierValid = false;  // a slot holds the mesh hierarchy of the current sort
    bool liveIsMesh = false;     // ... and it is the live slot
    int meshLevelSize[2 * 9] = {};
    int hierCache = 1;           // env MAS_HIER_CACHE=0: rebuild the levels every Prepare (A/B)
    unsigned long long hierId = 0, meshHierId = 0, hierCounter = 0;  // identity of the live hierarchy
    unsigned long long recHierId = ~0ull, tabHierId = ~0ull;  // hierarchy the records / apply tables were built for
    int nRecCached = 0;
    int lastHierDirty = -1;      // level the last Prepare's contacts changed (L: none; -1: full build)
    bool rangesChanged = true;   // this Prepare's CSR ranges differ from recRanges
    bool lastHierBuilt = false;  // the last Prepare ran a level build
    mas::Buffer hierFlags;       // device words: [0] first dirty level, [1] ranges differ from recRanges
    mas::Buffer recRanges;       // the CSR ranges the cached records index off9 with
    // diagTable term lists per level (cached with the records): vertex list,
    // its per-node offsets, per-vertex term offsets, terms
    mas::Buffer vlistL[5], voffL[5], termOffL[5], termsL[5];
    // level-3 descendant lists (k_coarse.hip): sort scratch, list
    // offsets, deepIdx = level-1 id per list slot, deepPos = list slot of
    // every level-1 node, R1 in list order (deepR1), per-block arrival counters
    mas::Buffer deepKeys, deepVals, deepIdx, deepOff, deepPos, deepR1, deepCnt, deepIdxShard;
    int deepStride = 0;  // list slots per level-3 node (the longest list, rounded up to 4)
    // one-launch coarse form (k_coarse1.hip): tagged hand-off slots (level-3
    // lists, level-2 nodes, level-3 nodes), per level-1 node (parent, mask,
    // list slot); the apply epoch the tags carry (0 after Prepare)
    mas::Buffer c1Tags, l1info;
    unsigned coarse1Epoch = 0;
    int c1PollDelay = 0;  // A/B (env MAS_C1_POLL_DELAY): fold / solve waves sleep before their first poll
    // bank waves of the one-launch coarse form dealt to the XCDs in contiguous
    // chunks (env MAS_C1_CHUNK=0: round-robin, A/B): interleaved, bitwise equal,
    // pre-fine 14.65 -> 13.82 us at 1M + contacts, 47.5 -> 42.5 us at 4M tet
    // (profiles/round4/ab/c1chunk_*.json)
    int c1Chunk = 1;
    // k_coarse1's bounded waits never hang the device: a wait gives up after
    // this many polls and is counted (env MAS_C1_POLL_LIMIT; < 0 forces it: tests)
    int c1PollLimit = 1 << 16;
    bool c1Launched = false;    // k_coarse1 ran since the handle was created
    // pinned host-coherent word: the epoch of the latest apply whose k_coarse1
    // wait gave up, 0 when none since the last report (pending_giveup)
    int* c1Host = nullptr;
    // device status words: [0] blocks with a bad pivot (this Prepare), [1] the
    // lowest such block, [2] coarse hand-off waits that gave up (since mas_create)
    mas::Buffer devStatus;
    mas::Buffer pcgVec, pcgPartial, pcgState, pcgStage;  // PCG driver (k_pcg.hip)
    mas::Buffer pcgEllOff, pcgEllIdx, pcgEllCnt;         // PCG: the CSR Hessian in wave-slot ELL form
    mas::Buffer pcgRzPart;                               // PCG: r.z partials of the fine apply kernel
    bool pcgSym = false;   // PCG: A/B (env MAS_PCG_SYM=1): mirrored intra-group blocks not stored (k_pcg_ell; measured slower)
    bool pcgFuseP = true;  // PCG: p = z + beta p inside the next SpMV (env MAS_PCG_FUSE_P=0: its own pass, A/B)
    // set by the PCG driver for the applies of a solve (null otherwise): the
    // apply kernels exit at once when *applyDone != 0, and the fine kernel
    // writes one r.z partial per workgroup to applyRzPart
    const int* applyDone = nullptr;
    double* applyRzPart = nullptr;
    std::vector<int> l1First;  // first level-1 local id per level-0 bank (+ n1), for sharding
    int shardWorld = 0;
    // one-call sharded apply (mas_shard_apply_device): library-owned segments,
    // the communication stream and its fork/join events
    mas::Buffer shardSeg, shardGathered;
    hipStream_t commStream = nullptr;
    // mas_shard_apply_device (k_shard.hip): 0 = the collective and every kernel on the apply stream (default);
    // 1 / 2 = the collective on commStream beside the level-0 solves, the coarse levels on commStream (1) or
    // on the apply stream (2) (env MAS_SHARD_MODE, A/B)
    int shardMode = 0;
    hipEvent_t evRestrict = nullptr, evGathered = nullptr;
    // end of the previous mas_shard_apply_device call and the stream it ran
    // on: a call on another stream waits for it (the segments are the handle's)
    hipEvent_t evShardDone = nullptr;
    hipStream_t shardLastStream = nullptr;
    void* rcclComm = nullptr;  // ncclComm_t (comm_rccl.hip)
    int rcclRank = -1, rcclWorld = 0;
    hipEvent_t* shardPendingEv = nullptr;  // profiling events of an overlapped sharded apply in flight
    // pinned words of read_back (small device -> host reads), their sequence
    int* rbHost = nullptr;
    int rbSeq = 0;
    // staging for host-pointer entry points
    mas::Buffer diagStage, offStage, rangeStage, rStage, zStage;
    // mas_config.host_register = 1 (or env MAS_HOST_REGISTER=1): the caller's
    // host arrays of the host-pointer entry points, page-locked
    // (hipHostRegister) when the same (pointer, size) comes back a second
    // time, page-aligned whole pages only, so their copies run at the pinned
    // rate: one slot per argument, released when another array is passed
    // there and by mas_destroy.  Off by default: the library cannot know that
    // a caller's array outlives its registration.  Slots: diag, off, ranges,
    // r, z, pcg x, pcg b.
    struct HostPin {
        const void* p = nullptr;
        size_t bytes = 0;
        bool registered = false;
        int seen = 0;  // calls in a row with this (pointer, size); registered at the second
    } pins[7];
    int hostRegister = 0;
    // hipcub scratch
    mas::Buffer cubTemp;
    // look-back-free radix sort and scan (rsort.hip): ping-pong keys/values,
    // per-tile digit counts, scan tile sums; env MAS_SORT=0 selects rocprim (A/B)
    mas::Buffer rsKeys, rsVals, rsHist, rsPart;
    // the same scratch for work queued on prepStream (run_level0_early), which
    // runs beside the caller's stream: sharing one set raced and a regrowth
    // freed a buffer the other stream was still reading
    mas::Buffer rsKeysP, rsValsP, rsHistP, rsPartP;
    int sortImpl = 1;
    // events: [0..1] allocate, [2..3] prepare
    hipEvent_t ev[4] = {};
    // profiling ring: 4 events per apply (start, restrict end, coarse end, fine end)
    std::vector<hipEvent_t> prof;
    int profRecorded = 0;
    mas_stats stats{};

    template <class F>
    void for_each_buffer(F f) {
        mas::Buffer* all[] = {&pos, &starts, &idx, &edges, &faces, &morton, &mortonSorted, &iota, &s2o, &o2s,
                              &nbrNum, &nbr, &nbrNumRem, &nbrRem, &aabbPartial, &rawContacts, &stencilFlags,
                              &stencilSlots, &stencils, &fineMask, &nextMask, &bankCount, &bankPrefix, &levelTotal,
                              &cst, &goingNext, &vmap, &coarseTables, &dense, &inv, &slotTable, &tileSlot, &valuSlot, &additional, &od,
                              &recCnt, &recOff, &rec, &recKeys, &recKeysSorted, &recIds, &recIdsSorted, &vkeys,
                              &tab, &termCnt,
                              &cdCnt, &cdOff, &cdKeys, &cdKeysS, &cdIds, &cdIdsS, &cdVal, &cFineOff, &cdEnt, &c0Ent, &caCnt, &caOff,
                              &caKeys, &caKeysS, &caIds, &caIdsS, &caVal, &cpCnt, &cpOff, &cpKeys, &cpKeysS, &cpIds,
                              &cpIdsS, &Rc, &Zc, &splitDev, &prepSeg, &prepGathered, &splitPartsDev, &members, &coarseMask, &shardOff, &shardPos1, &l1src, &deepKeys, &deepVals, &deepIdx, &deepOff, &deepPos, &deepR1, &deepCnt, &deepIdxShard, &c1Tags, &l1info, &pcgVec, &pcgPartial, &pcgState, &pcgStage, &pcgEllOff, &pcgEllIdx, &pcgEllCnt, &pcgRzPart, &shardSeg, &shardGathered, &diagStage, &offStage, &rangeStage, &rStage, &zStage,
                              &cubTemp, &rsKeys, &rsVals, &rsHist, &rsPart, &rsKeysP, &rsValsP, &rsHistP, &rsPartP, &add0, &c0Cnt, &c0Off, &c0Keys, &c0KeysS, &c0Ids, &c0IdsS,
                              &c0Val, &a0Keys, &a0KeysS, &a0Ids, &a0IdsS, &a0Val,
                              &spCst, &spGn, &spVmap, &spCoarseTables, &spFine, &spCoarseMask, &hierFlags, &recRanges,
                              &devStatus};
        for (mas::Buffer* b : all) f(*b);
        for (int l = 0; l < 5; ++l)
            for (mas::Buffer* b : {&vlistL[l], &voffL[l], &termOffL[l], &termsL[l]}) f(*b);
    }
};

// ---- helpers shared by the .hip translation units ----
namespace mas {

int fail(mas_context* h, int code, const std::string& msg);
// While alive, fail() on this host thread stores its message in *sink instead
// of the handle (a helper thread of one call must not race the caller's
// writes of mas_context::err).
struct ErrorSink {
    explicit ErrorSink(std::string* sink);
    ~ErrorSink();
    ErrorSink(const ErrorSink&) = delete;
    ErrorSink& operator=(const ErrorSink&) = delete;
};
int hip_check(mas_context* h, hipError_t e, const char* what);
int ensure(mas_context* h, Buffer& b, size_t bytes);
template <class T>
inline T* P(Buffer& b) { return reinterpret_cast<T*>(b.p); }
template <class T>
inline const T* P(const Buffer& b) { return reinterpret_cast<const T*>(b.p); }
inline int ceil32(int x) { return (x + 31) / 32 * 32; }
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
// block b's 96x96 at dense_base(h) + 9216 b (b >= nFineBlk unless denseFine)
inline float* dense_base(mas_context* h) {
    return P<float>(h->dense) - (h->denseFine ? 0 : (ptrdiff_t)h->nFineBlk * kDenseFloats);
}

// phase entry points (host orchestration), defined per translation unit
int run_allocate(mas_context* h, const float* pos4, const int* starts, const int* idx, const int* edges4,
                 const int* faces4);
int run_prepare(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, const void* ef,
                const void* ee, const void* vf, const unsigned* efC, const unsigned* eeC, const unsigned* vfC,
                hipStream_t s);
int build_stencils(mas_context* h, const void* ef, const void* ee, const void* vf, const unsigned* efC,
                   const unsigned* eeC, const unsigned* vfC, hipStream_t s);
// the level maps of this Prepare (incremental: k_levels.hip); beforeRead: called
// once the device work is queued, before the first host read
int run_levels(mas_context* h, hipStream_t s, const int* d_ranges, const std::function<int()>& beforeRead = {});
int run_assemble(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, hipStream_t s);
// the level-0 contact path and the fused level-0 kernel on prepStream, right
// after the stencils (fused variants without keep_blocks); sets earlyFused
int run_level0_early(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, hipStream_t s);
// the early fused kernel itself, when it waits for the level build (fusedAfterLevels)
int launch_level0_fused(mas_context* h, hipStream_t s);
bool early_fused_wanted(const mas_context* h);
// waits for the early path's worker job (if one is in flight) and returns its status
int finish_early(mas_context* h);
bool early_od(const mas_context* h);  // od and the record counts computed by the early path
int early_buffers(mas_context* h);    // the early path's buffers the caller reads too (run_prepare sizes them)
int prep_stream_init(mas_context* h);  // prepStream (CU-masked) and its events
int run_factor(mas_context* h, hipStream_t s);
// factor blocks [b0, b1) in the coarse form (identity fix + k_factor_rb / k_factor) (k_factor.hip)
int factor_blocks(mas_context* h, int b0, int b1, hipStream_t s);
// coarse_split.hip: the split plan of a sharded Prepare (after the level build),
// the pack of this rank's rows, the exchange's second half (unpack + factor)
int plan_coarse_split(mas_context* h, hipStream_t s);
int pack_coarse_rows(mas_context* h, hipStream_t s);
int complete_coarse_rows(mas_context* h, const float* gathered, hipStream_t s);
// the Prepare status words (pivot checks): stats + the non-SPD warning / error (prepare.hip)
int report_pivots(mas_context* h, hipStream_t s);
// fused level-0 assemble + factor of blocks [blk0, blk1) (k_factor.hip)
int launch_factor_fused(mas_context* h, const FineAsm& a, int blk0, int blk1, hipStream_t s);
int run_apply(mas_context* h, float4* d_z, const float4* d_r, hipStream_t s);
int coarse_mode(const mas_context* h);  // the coarse launch form an apply uses (k_apply.hip)
int upload_slot_table(mas_context* h);
int prepare_apply_tables(mas_context* h, hipStream_t s);
int build_l1src(mas_context* h, hipStream_t s);
void launch_coarse_twopass(mas_context* h, const float4* r, hipStream_t s);
void launch_coarse_one(mas_context* h, const float4* r, hipStream_t s);  // k_coarse1.hip (L >= 3)
int build_coarse1_tables(mas_context* h, hipStream_t s);
bool coarse1_supported(const mas_context* h);  // the tag slots exist (k_coarse1.hip)
void launch_coarse_levels(mas_context* h, int lFirst, const float4* d_r, hipStream_t s);
void launch_coarse_deep(mas_context* h, const float4* src, const int* idx, hipStream_t s);
int deep_nodes(const mas_context* h);  // level-3 node ids incl. padding (0 below L = 4)
mas::DeepArgs deep_args(mas_context* h, const float4* src, const int* idx);
int build_deep_lists(mas_context* h, hipStream_t s);
int build_deep_shard_idx(mas_context* h, hipStream_t s);
// rsort.hip: stable sort by the low `bits` key bits; exclusive scan
// side = true: prepStream's scratch (rsKeysP ...), for work beside the caller's stream
int rs_sort_pairs(mas_context* h, const unsigned* kin, unsigned* kout, const int* vin, int* vout, int n, int bits,
                  hipStream_t s, const char* what, bool side = false);
int rs_exclusive_scan(mas_context* h, const int* in, int* out, int n, hipStream_t s, const char* what,
                      bool side = false);
int sort_pairs_u32(mas_context* h, const unsigned* kin, unsigned* kout, const int* vin, int* vout, int n, int bits,
                   hipStream_t s, const char* what);
// level-0 blocks [blk0, blkEnd) + prolongation; done / rzPart: PCG hooks (k_apply.hip)
void launch_fine(mas_context* h, int blk0, int blkEnd, const float4* r, float4* z, hipStream_t s,
                 const int* done = nullptr, double* rzPart = nullptr);
void launch_coarse_apply(mas_context* h, const float4* d_r, hipStream_t s);  // the coarse levels of run_apply
void launch_fine_z0(mas_context* h, int blk0, int blkEnd, const float4* r, float4* z, hipStream_t s);
void launch_prolong(mas_context* h, int v0, int v1, float4* z, hipStream_t s);
int fine_grid(const mas_context* h);  // workgroups of one fine launch over every level-0 block
int compute_l1_first(mas_context* h, hipStream_t s);
// up to 8 device ints -> out, through pinned memory (mas_capi.hip)
int read_back(mas_context* h, hipStream_t s, std::initializer_list<const int*> src, int* out);
// MAS_ERR_HIP when an apply's k_coarse1 wait gave up since the last report
// (reads and clears the pinned word c1Host; no synchronisation): an apply
// that completed with an incomplete z is reported by the next call
int pending_giveup(mas_context* h);
// the same split in two: enqueue the copy (its sequence number in *seq), and
// later wait for it (or a newer post) to land
int read_back_post(mas_context* h, hipStream_t s, std::initializer_list<const int*> src, int* seq);
int read_back_wait(mas_context* h, hipStream_t s, int seq, int* out, int n);
void release_comm(mas_context* h);  // comm_rccl.hip
// an allgather of `bytes` per rank over the handle's RCCL communicator on s (comm_rccl.hip)
int comm_allgather(mas_context* h, const void* send, void* recv, size_t bytes, hipStream_t s);
int copy_block_inverse(mas_context* h, int blk, float* out96);
int run_pcg(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, float4* d_x,
            const float4* d_b, int maxIters, float tol, int precondition, mas_pcg_result* res, hipStream_t s);

}  // namespace mas
